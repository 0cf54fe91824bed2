#!/bin/bash
# r3: tail2 W2 ring depth 8 / 6 (128 / 64 planes) — kernel check + timing, tail tests, C3 bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "128 64 20 125" "64 64 40 249" "32 64 80 498"; do
  timeout -k 5 60 ./tools/tail_check $cfg 10 > gpurun_out/tc.log 2>&1 || { tail -5 gpurun_out/tc.log; exit 1; }
  echo "C=${cfg%% *}"; grep -E "variant 1|other|out:|y1n" gpurun_out/tc.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py -x -q -k res_tail --timeout 120 --timeout-method thread \
  > gpurun_out/t_w2.log 2>&1 || { tail -20 gpurun_out/t_w2.log; exit 1; }
tail -1 gpurun_out/t_w2.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --arch ResNet293 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 --sustain-seconds 2 \
    > gpurun_out/c3w.json 2> gpurun_out/c3w.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/c3w.json'))
print('C3', d['value'], d['value_sustained']['value'], d['roofline']['frac'], {n:round(v['ms_per_step'],2) for n,v in d['kernels'].items() if 'tail' in n})"
done
