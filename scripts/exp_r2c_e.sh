#!/bin/bash
# r2c experiment: ResNet conv1 from whole rows in LDS (option conv1x1_rows) on / off.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_r2c_e.log 2>&1 || exit 1
for v in 1 0 1 0; do
  timeout -k 10 200 python bench.py --arch ResNet293 --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt conv1x1_rows=$v >> gpurun_out/c1r_c3.jsonl 2> gpurun_out/c1r_$v.err || exit 1
done
for v in 1 0; do
  timeout -k 10 200 python bench.py --arch ResNet293 --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 1 --opt conv1x1_rows=$v --opt streams=1 >> gpurun_out/c1r_c3_s1.jsonl 2> gpurun_out/c1r_s1_$v.err || exit 1
done
for v in 1 0; do
  timeout -k 10 240 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt cat_gate=$v >> gpurun_out/c4_cg.jsonl 2> gpurun_out/c4_cg_$v.err || exit 1
done
