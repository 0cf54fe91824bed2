#!/bin/bash
# r3 experiment: the 256x256 bf16x3 tile on 16x16x32 MFMAs (x3_variant 6) vs 32x32x16 (5).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "mf16" > gpurun_out/t_mf16.log 2>&1 || { tail -30 gpurun_out/t_mf16.log; exit 1; }
tail -2 gpurun_out/t_mf16.log
summ() {
  python -c "
import json,sys;d=json.load(open(sys.argv[1]))
k=d.get('kernels',{})
print(sys.argv[2], d['value'], d['ms_per_step'], d.get('value_sustained',{}).get('value'), {n:round(v['avg_ms'],4) for n,v in k.items() if n in ('conv1x1_CxC','conv_cat','h_cnn','h_fc1','h_fc2','h_qkv','h_out_proj','pool_linear1')})" "$@"
}
for v in 5 6 5 6; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32 --sustain-seconds 2 --configs none \
    --opt x3_variant=$v > gpurun_out/mf16_c2_$v.json 2> gpurun_out/mf16_c2_$v.err || exit 1
  summ gpurun_out/mf16_c2_$v.json "C2 x3_variant=$v"
done
for v in 5 6 5 6; do
  timeout -k 10 300 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt x3_variant=$v > gpurun_out/mf16_c4_$v.json 2> gpurun_out/mf16_c4_$v.err || exit 1
  summ gpurun_out/mf16_c4_$v.json "C4 x3_variant=$v"
done
