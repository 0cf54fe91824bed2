#!/bin/bash
# r3: tail tests + C3 bench with the 8-deep W2 ring for 128-plane tails
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_w2f.log 2>&1 || { tail -20 gpurun_out/t_w2f.log; exit 1; }
tail -1 gpurun_out/t_w2f.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --arch ResNet293 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 --sustain-seconds 2 \
    > gpurun_out/c3f.json 2> gpurun_out/c3f.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/c3f.json'))
print('C3', d['value'], d['value_sustained']['value'], d['roofline']['frac'], {n:round(v['ms_per_step'],2) for n,v in d['kernels'].items() if 'tail' in n})"
done
