#!/bin/bash
# r3: C2 A/B over model options given as OPTS="k=v,k=v ..." (space-separated runs; "-" = defaults).
set -o pipefail
mkdir -p gpurun_out
i=0
for o in ${OPTS:--}; do
  i=$((i+1))
  args=""
  if [ "$o" != "-" ]; then for kv in ${o//,/ }; do args="$args --opt $kv"; done; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32 --configs none \
    --sustain-seconds 2 $args > gpurun_out/r3_c2opt_$i.json 2> gpurun_out/r3_c2opt_$i.err || { echo "bench failed ($o)"; tail gpurun_out/r3_c2opt_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_c2opt_$i.json'));print('$o', d['value'], d['value_sustained']['value'], d['ms_per_step'])"
done
