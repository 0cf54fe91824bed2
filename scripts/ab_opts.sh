#!/bin/bash
# Model-option A/B for one workload: one bench line per arm (repeated ROUNDS times, interleaved),
# each saved whole as gpurun_out/${TAG}_ab_<round>_<arm>.json for per-class comparison.
#   TAG=r6m ARCH=ResNet293 ARMS="default x3_variant=7" ROUNDS=2 STEPS=6 bash scripts/ab_opts.sh
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-1}); do
  for arm in ${ARMS:-default}; do
    opts=""
    if [ "$arm" != "default" ]; then for kv in ${arm//,/ }; do opts="$opts --opt $kv"; done; fi
    f=gpurun_out/${TAG:-ab}_ab_${r}_${arm//[=,]/_}.json
    timeout -k 10 300 python -u bench.py --arch ${ARCH:-ResNet293} --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline \
      --no-f32 --configs none --sustain-seconds 0 --no-kernel-roofline $opts > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python -c "import json; d = json.load(open('$f')); print('round $r arm $arm', d['value'], d['ms_per_step'])"
  done
done
