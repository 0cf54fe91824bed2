#!/bin/bash
# r3: streams sweep after the tail / MF16 changes (C3 ResNet293, C4 HuBERT chain)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for st in 2 3 2 3; do
  timeout -k 10 300 python bench.py --arch ResNet293 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --no-profile --opt streams=$st > gpurun_out/st_c3_$st.json 2> gpurun_out/st_c3_$st.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/st_c3_$st.json'));print('C3 streams=$st',d['value'],d['value_sustained']['value'])"
done
for st in 2 3; do
  timeout -k 10 300 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 6 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --no-profile --opt streams=$st > gpurun_out/st_c4_$st.json 2> gpurun_out/st_c4_$st.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/st_c4_$st.json'));print('C4 streams=$st',d['value'],d['value_sustained']['value'])"
done
