#!/bin/bash
# r3: Res2Net chain variant checks + C2 A/B (res2_variant), each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_res2.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_res2_tests.log 2>&1 || { echo "res2 tests failed"; tail -30 gpurun_out/r3_res2_tests.log; exit 1; }
tail -2 gpurun_out/r3_res2_tests.log
for v in ${VARIANTS:-0 3 0 3}; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32 --configs none \
    --sustain-seconds 2 --opt res2_variant=$v > gpurun_out/r3_c2_res2_$v.json 2> gpurun_out/r3_c2_res2_$v.err || { echo "bench failed"; tail gpurun_out/r3_c2_res2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_c2_res2_$v.json'));print('res2_variant=$v', d['value'], d['value_sustained']['value'], d['kernels']['res2_k3'])"
done
