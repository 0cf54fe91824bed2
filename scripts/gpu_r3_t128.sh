#!/bin/bash
# r3 experiment: 128-plane tail on tail128_kernel (res_tail 3) vs bottleneck_tail_kernel (1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 120 --timeout-method thread \
  -k "res_tail" > gpurun_out/t_t128.log 2>&1 || { tail -30 gpurun_out/t_t128.log; exit 1; }
tail -2 gpurun_out/t_t128.log
for v in 1 3 1 3; do
  timeout -k 10 200 python bench.py --arch ResNet293 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt res_tail=$v > gpurun_out/t128_$v.json 2> gpurun_out/t128_$v.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/t128_$v.json'))
k=d.get('kernels',{})
print('res_tail=$v', d['value'], d['ms_per_step'], d.get('value_sustained',{}).get('value'), {n:round(v['ms_per_step'],2) for n,v in k.items() if 'tail' in n})"
done
