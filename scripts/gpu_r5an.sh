# r5: C3 with 2 vs 3 utterance-range streams, interleaved pairs
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2; do
  for s in 2 3; do
    o=gpurun_out/r5an_s${s}_$i
    timeout -k 10 300 python bench.py --arch ResNet293 --configs none --no-cpu-baseline --sustain-seconds 0 --no-f32 --no-profile --opt streams=$s > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$o.json').read().strip().splitlines()[-1]); print('ResNet293 streams $s round $i', d['value'], d['ms_per_step'])"
  done
done
