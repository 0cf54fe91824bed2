#!/bin/bash
# r2c experiment: conv3x3_img with 128 channels (option conv3x3_img 2 / 3) vs 1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_img128.log 2>&1 || exit 1
for arch in ResNet293 ResNet34 SimAM_ResNet34_ASP; do
  for v in 1 2 3; do
    timeout -k 10 200 python bench.py --arch $arch --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
      --sustain-seconds 1 --opt conv3x3_img=$v > gpurun_out/img128_${arch}_$v.json 2> gpurun_out/img128_${arch}_$v.err || exit 1
  done
done
