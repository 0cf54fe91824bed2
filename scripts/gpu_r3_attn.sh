#!/bin/bash
# r3: pipelined attention checks + C4 A/B (attn_pipe on / off), each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hubert.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_attn_tests.log 2>&1 || { echo "attn tests failed"; tail -30 gpurun_out/r3_attn_tests.log; exit 1; }
tail -2 gpurun_out/r3_attn_tests.log
for v in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt attn_pipe=$v > gpurun_out/r3_c4_attn$v.json 2> gpurun_out/r3_c4_attn$v.err || { echo "bench failed"; tail gpurun_out/r3_c4_attn$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_c4_attn$v.json'));print('attn_pipe=$v', d['value'], d['value_sustained']['value'], d['kernels']['h_attn'])"
done
