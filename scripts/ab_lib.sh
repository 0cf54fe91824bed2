#!/bin/bash
# Library A/B on one box: wespeaker_hubert_amd/libwsp_hip_old.so (built from an older tree) against
# the in-tree libwsp_hip.so, ROUNDS interleaved pairs of one bench line each (full JSON kept as
# gpurun_out/${TAG}_lib_<round>_<old|new>.json).  The in-tree library is restored at the end.
#   TAG=r6p ARCH=ECAPA_TDNN_c1024 ROUNDS=2 STEPS=10 bash scripts/ab_lib.sh
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=wespeaker_hubert_amd
cp $L/libwsp_hip.so /tmp/libwsp_hip_new.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in old new; do
    cp /tmp/libwsp_hip_$arm.so $L/libwsp_hip.so 2>/dev/null || cp $L/libwsp_hip_old.so $L/libwsp_hip.so
    f=gpurun_out/${TAG:-ab}_lib_${r}_${arm}.json
    timeout -k 10 300 python -u bench.py --arch ${ARCH:-ECAPA_TDNN_c1024} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
      --no-f32 --configs none --sustain-seconds 0 --no-kernel-roofline ${EXTRA:-} > $f 2> $f.err || { cp /tmp/libwsp_hip_new.so $L/libwsp_hip.so; tail -20 $f.err; exit 1; }
    python -c "import json; d = json.load(open('$f')); print('round $r $arm', d['value'], d['ms_per_step'])"
  done
done
cp /tmp/libwsp_hip_new.so $L/libwsp_hip.so
