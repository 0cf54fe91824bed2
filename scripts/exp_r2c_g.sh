#!/bin/bash
# r2c sweep: ResNet293 (C3) concurrent sub-batch streams 2 / 3 / 4.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for st in 2 3 4 2 3 4; do
  timeout -k 10 200 python bench.py --arch ResNet293 --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt streams=$st >> gpurun_out/c3_streams.jsonl 2> gpurun_out/c3_st$st.err || exit 1
done
