#!/bin/bash
# r3: bottleneck_tail checks + C3 A/B (res_tail on / off), each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -k tail -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_tail_tests.log 2>&1 || { echo "tail tests failed"; tail -30 gpurun_out/r3_tail_tests.log; exit 1; }
tail -3 gpurun_out/r3_tail_tests.log
for v in ${TAILS:-1 1}; do
  timeout -k 10 200 python -u bench.py --arch ResNet293 --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt res_tail=$v > gpurun_out/r3_c3_tail$v.json 2> gpurun_out/r3_c3_tail$v.err || { echo "bench failed"; tail gpurun_out/r3_c3_tail$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_c3_tail$v.json'));k=d['kernels'];print('res_tail=$v', d['value'], d['value_sustained']['value'], d['roofline']['frac'], {c: k[c]['avg_ms'] for c in k if c.startswith('res_tail.')})"
done
