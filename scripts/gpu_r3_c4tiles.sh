#!/bin/bash
# r3: HuBERT + ECAPA (C4) per-class times under each GEMM tile family (x3_variant 3 / 4 / 5), streams 1.
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-5 3 4 5}; do
  timeout -k 10 300 python -u bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 0 --opt streams=1 --opt x3_variant=$v > gpurun_out/r3_c4_x3v$v.json 2> gpurun_out/r3_c4_x3v$v.err || { echo "bench failed"; tail gpurun_out/r3_c4_x3v$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_c4_x3v$v.json'));k=d['kernels'];print('x3_variant=$v', d['value'], {c: round(k[c]['ms_per_step'],2) for c in k if c.startswith('h_') or c in ('conv1x1_CxC','conv_cat','layer1')})"
done
