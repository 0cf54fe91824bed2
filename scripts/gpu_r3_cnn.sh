#!/bin/bash
# r3: HuBERT CNN per-layer timing, streams=1, tile variants A/B.
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-5 4 3}; do
  timeout -k 10 300 python -u bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --configs none --opt streams=1 --x3-variant $v > gpurun_out/r3_cnn_$v.json 2> gpurun_out/r3_cnn_$v.err || { echo "bench failed"; tail gpurun_out/r3_cnn_$v.err; exit 1; }
  python - <<PY
import json;d=json.load(open('gpurun_out/r3_cnn_$v.json'))
print('x3_variant=$v', d['value'], d['ms_per_step'])
for k,v in d['kernels'].items():
    if k.startswith('h_'): print('  ', k, v['launches_per_step'], v['avg_ms'], v['ms_per_step'], v['tflops'])
PY
done
