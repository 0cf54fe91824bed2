#!/bin/bash
# r2c experiment: conv3x3_img 128-channel tiles (2 = 4 waves x 4 column tiles, 3 = 8 waves x 2)
# and ECAPA cat_gate on / off.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_catgate.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/t_r2c_b.log 2>&1 || exit 1
for v in 1 0 1 0; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32 --sustain-seconds 2 \
    --opt cat_gate=$v > gpurun_out/cg_$v.json 2> gpurun_out/cg_$v.err || exit 1
  cat gpurun_out/cg_$v.json >> gpurun_out/cg_all.jsonl
done
for arch in ResNet293 ResNet34; do
  for v in 2 3; do
    timeout -k 10 200 python bench.py --arch $arch --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
      --sustain-seconds 1 --opt conv3x3_img=$v > gpurun_out/img_${arch}_$v.json 2> gpurun_out/img_${arch}_$v.err || exit 1
    timeout -k 10 200 python bench.py --arch $arch --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
      --sustain-seconds 1 --opt conv3x3_img=$v --opt streams=1 > gpurun_out/img_${arch}_${v}_s1.json 2> gpurun_out/img_${arch}_${v}_s1.err || exit 1
  done
done
