#!/bin/bash
# r2c experiment: ResNet residual prefetch (option res_prefetch) on / off.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_r2c_d.log 2>&1 || exit 1
for arch in ResNet293 ResNet34; do
  for v in 1 0 1 0; do
    timeout -k 10 200 python bench.py --arch $arch --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
      --sustain-seconds 2 --opt res_prefetch=$v >> gpurun_out/rp_${arch}.jsonl 2> gpurun_out/rp_${arch}_$v.err || exit 1
  done
  for v in 1 0; do
    timeout -k 10 200 python bench.py --arch $arch --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
      --sustain-seconds 1 --opt res_prefetch=$v --opt streams=1 >> gpurun_out/rp_${arch}_s1.jsonl 2> gpurun_out/rp_${arch}_s1_$v.err || exit 1
  done
done
