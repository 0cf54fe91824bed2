#!/bin/bash
# r3: x3_variant 6 (W by LDS-DMA) parity + C2 / C4 A/B against variant 5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_gw_tests.log 2>&1 || { echo "parity tests failed"; tail -30 gpurun_out/r3_gw_tests.log; exit 1; }
tail -2 gpurun_out/r3_gw_tests.log
for v in 5 6 5 6; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --configs none \
    --sustain-seconds 2 --opt x3_variant=$v > gpurun_out/r3_gw_c2_$v.json 2> gpurun_out/r3_gw_c2_$v.err || { echo "bench failed"; tail gpurun_out/r3_gw_c2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_gw_c2_$v.json'));k=d['kernels'];print('C2 x3_variant=$v', d['value'], d['value_sustained']['value'], {c: round(k[c]['avg_ms'],4) for c in ('conv1x1_CxC','conv_cat','layer1','pool_linear1')})"
done
for v in 5 6; do
  timeout -k 10 300 python -u bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 0 --opt streams=1 --opt x3_variant=$v > gpurun_out/r3_gw_c4_$v.json 2> gpurun_out/r3_gw_c4_$v.err || { echo "bench failed"; tail gpurun_out/r3_gw_c4_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_gw_c4_$v.json'));k=d['kernels'];print('C4 x3_variant=$v', d['value'], {c: round(k[c]['ms_per_step'],2) for c in k if c in ('h_cnn','h_qkv','h_fc1','h_fc2','h_out_proj','h_pos_conv')})"
done
