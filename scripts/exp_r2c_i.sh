#!/bin/bash
# r2c check: ResNet default tile family 4 (256x128 swizzled) — ResNet tests, C3 / ResNet34 with 4 vs 3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/t_r2c_i.log 2>&1 || exit 1
for arch in ResNet34 ResNet293; do
  for v in 4 3 4 3; do
    timeout -k 10 200 python bench.py --arch $arch --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
      --sustain-seconds 2 --x3-variant $v >> gpurun_out/x3v_$arch.jsonl 2> gpurun_out/x3v_${arch}_$v.err || exit 1
  done
done
