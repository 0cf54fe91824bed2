#!/bin/bash
# r3: ResNet293 GEMM tile family 4 (256x128, default) vs 3 (128x128, two blocks per CU) per class
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py -x -q -k "res_tail" --timeout 120 --timeout-method thread \
  > gpurun_out/t_f60.log 2>&1 || { tail -20 gpurun_out/t_f60.log; exit 1; }
tail -1 gpurun_out/t_f60.log
for v in 4 3 4 3; do
  timeout -k 10 300 python bench.py --arch ResNet293 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt x3_variant=$v > gpurun_out/rx_$v.json 2> gpurun_out/rx_$v.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/rx_$v.json'))
k=d['kernels']
print('C3 x3_variant=$v', d['value'], d['value_sustained']['value'], {n:round(v['ms_per_step'],2) for n,v in k.items() if n.startswith('res_conv1x1.') or n in ('shortcut','res_conv3x3','stem')})"
done
