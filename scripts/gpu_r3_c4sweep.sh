#!/bin/bash
# r3: C4 streams / batch sweep (one process per setting, each time-limited).
set -o pipefail
mkdir -p gpurun_out
for cfg in "--opt streams=1" "--opt streams=2" "--opt streams=1 --batch 384" "--opt streams=2 --batch 384"; do
  timeout -k 10 200 python -u bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 10 --warmup 2 --no-cpu-baseline --no-f32 \
    --sustain-seconds 2 --no-profile $cfg > gpurun_out/r3_c4_sweep.json 2> gpurun_out/r3_c4_sweep.err || { echo "bench failed"; tail gpurun_out/r3_c4_sweep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_c4_sweep.json'));print('$cfg', d['value'], d['value_sustained']['value'])"
done
