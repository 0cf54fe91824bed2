# r5: C3 / C4 with 1 vs 2 streams (option streams), interleaved pairs
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for arch in HuBERT_ECAPA_GLOB_c512 ResNet293; do
for i in 1 2; do
  for s in 2 1; do
    o=gpurun_out/r5ak_${arch}_s${s}_$i
    timeout -k 10 300 python bench.py --arch $arch --configs none --no-cpu-baseline --sustain-seconds 0 --no-f32 --no-profile --opt streams=$s > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$o.json').read().strip().splitlines()[-1]); print('$arch streams $s round $i', d['value'], d['ms_per_step'])"
  done
done
done
