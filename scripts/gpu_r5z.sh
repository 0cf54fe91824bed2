# r5: fbank prefetch A/B (WSP_FBANK_PRE=0/1 interleaved, same box)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; return $rc; }
for i in 1 2; do
  for p in 0 1; do
    export WSP_FBANK_PRE=$p
    run r5z_${p}_$i 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5z_${p}_$i -o p -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile --no-f32 --sustain-seconds 0 --configs none || exit $?
  done
done
