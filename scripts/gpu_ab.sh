#!/bin/bash
# Parameterised A/B on one GPU box (replaces the r2 / r3 one-off launchers):
#   TESTS="tests/test_gpu_x.py ..."  pytest files run first (-x; a failure ends the script)
#   ARCH=ResNet293                    bench workload (default the C2 headline, sub-configs off)
#   ARMS="res_tail=1 res_tail=2"      one bench run per arm, repeated ROUNDS times, interleaved;
#                                     an arm is a space-free list of key=value options joined by ','
#   ROUNDS=2 STEPS=6
# Each step runs under its own time limit; the first failure ends the script.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 200 \
    --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
ARCH=${ARCH:-ECAPA_TDNN_c1024}
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in ${ARMS:-default}; do
    opts=""
    if [ "$arm" != "default" ]; then for kv in ${arm//,/ }; do opts="$opts --opt $kv"; done; fi
    timeout -k 10 300 python -u bench.py --arch $ARCH --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-f32 \
      --configs none --sustain-seconds 2 --no-kernel-roofline --no-hubert-b64 $opts \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python -c "
import json; d = json.load(open('gpurun_out/ab.json'))
top = sorted(((k, v['ms_per_step']) for k, v in d['kernels'].items() if '.' not in k), key=lambda kv: -kv[1])[:6]
print('round $r arm $arm', d['value'], (d['value_sustained'] or {}).get('value'), [(k, round(v, 2)) for k, v in top])"
  done
done
