#!/bin/bash
# Round checkpoint on one GPU: full parity suite, smoke, the headline bench and
# the C3 / C4 configurations, then rocprofv3 kernel stats + PMC passes of each
# (scripts/gpu_profile.sh, PROF_TAG per config).  Every step time-limited; a
# fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${ROUND_TAG:-r2}
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-4} "gpurun_out/$name.log"
  return $rc
}
if [ -z "${SKIP_TESTS:-}" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
run bench_c2 600 python bench.py || exit $?
run bench_c3 600 python bench.py --arch ResNet293 --no-cpu-baseline --no-f32 --steps 5 --warmup 1 || exit $?
run bench_c4 600 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --no-cpu-baseline --no-f32 || exit $?
if [ -z "${SKIP_PROF:-}" ]; then
  PROF_TAG=prof_${R}_c2 timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_c2.log 2>&1 || exit $?
  PROF_TAG=prof_${R}_c4 EXTRA="--arch HuBERT_ECAPA_GLOB_c512" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_c4.log 2>&1 || exit $?
  PROF_TAG=prof_${R}_c3 EXTRA="--arch ResNet293" BARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" \
    timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_c3.log 2>&1 || exit $?
  tail -n 3 gpurun_out/prof_c*.log
fi
exit 0
