#!/bin/bash
# r3: C4 with HuBERT's CNN / fc1 / fc2 on the 16x16x32 tile (x3_variant 5 default selection) vs all on it (6)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hubert.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_c4mf.log 2>&1 || { tail -30 gpurun_out/t_c4mf.log; exit 1; }
tail -1 gpurun_out/t_c4mf.log
summ() {
  python -c "
import json,sys;d=json.load(open(sys.argv[1]))
k=d.get('kernels',{})
print(sys.argv[2], d['value'], d['ms_per_step'], d.get('value_sustained',{}).get('value'), {n:round(v['avg_ms'],4) for n,v in k.items() if n in ('h_cnn','h_fc1','h_fc2','h_qkv','h_out_proj','h_conv0','h_attn')})" "$@"
}
for v in 5 6 5 6; do
  timeout -k 10 300 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --opt x3_variant=$v > gpurun_out/c4mf_$v.json 2> gpurun_out/c4mf_$v.err || exit 1
  summ gpurun_out/c4mf_$v.json "C4 x3_variant=$v"
done
