#!/bin/bash
# r2c sweep: C4 per-GPU batch (256 / 384 / 512) and streams (2 / 3); C2 streams 1 / 2.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for b in 256 384 512; do
  for st in 2 3; do
    timeout -k 10 240 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --batch $b --steps 6 --warmup 2 --no-cpu-baseline \
      --no-f32 --sustain-seconds 2 --opt streams=$st > gpurun_out/c4_b${b}_s$st.json 2> gpurun_out/c4_b${b}_s$st.err || exit 1
  done
done
for st in 2 1 2 1; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32 --sustain-seconds 2 \
    --opt streams=$st >> gpurun_out/c2_streams.jsonl 2> gpurun_out/c2_s$st.err || exit 1
done
