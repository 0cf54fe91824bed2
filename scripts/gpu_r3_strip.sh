#!/bin/bash
# r3: res2 strip kernel (res2_variant 4) parity + C2 A/B against variant 3, each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_res2.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_strip_tests.log 2>&1 || { echo "res2 tests failed"; tail -30 gpurun_out/r3_strip_tests.log; exit 1; }
tail -3 gpurun_out/r3_strip_tests.log
for v in ${VARIANTS:-3 4 3 4}; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --configs "" \
    --sustain-seconds 2 --opt res2_variant=$v > gpurun_out/r3_c2_res2v$v.json 2> gpurun_out/r3_c2_res2v$v.err || { echo "bench failed"; tail gpurun_out/r3_c2_res2v$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_c2_res2v$v.json'));k=d['kernels'];print('res2_variant=$v', d['value'], d['value_sustained']['value'], k['res2_k3'])"
done
