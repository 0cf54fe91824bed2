#!/bin/bash
# r3 checkpoint: full parity suite, smoke, default bench (C2 + C3 + C4), C4 rocprofv3 stats + PMC.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  return $rc
}
run pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
echo bench ok
PROF_TAG=prof_r3j_c4 EXTRA="--arch HuBERT_ECAPA_GLOB_c512" BARGS="--steps 4 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" \
  timeout -k 10 560 bash scripts/gpu_profile.sh > gpurun_out/prof_c4.log 2>&1 || { tail -5 gpurun_out/prof_c4.log; exit 1; }
tail -2 gpurun_out/prof_c4.log
