#!/bin/bash
# r2c sweep: ResNet293 (C3) GEMM tile family (x3_variant 3 = 128x128 swizzled default, 4 = 256x128, 1 = 256x128 unswizzled).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in 3 4 1 3 4 1; do
  timeout -k 10 200 python bench.py --arch ResNet293 --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --x3-variant $v >> gpurun_out/c3_x3v.jsonl 2> gpurun_out/c3_x3v$v.err || exit 1
done
