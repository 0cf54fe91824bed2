# r5: C2 headline with 1 vs 2 utterance-range streams, interleaved pairs
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for s in 1 2; do
    timeout -k 10 200 python bench.py --configs none --no-cpu-baseline --sustain-seconds 0 --no-f32 --opt streams=$s > gpurun_out/r5aj_s${s}_$i.json 2> gpurun_out/r5aj_s${s}_$i.err || { tail -5 gpurun_out/r5aj_s${s}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/r5aj_s${s}_$i.json').read().strip().splitlines()[-1]); print('streams $s round $i', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
  done
done
