#!/bin/bash
# The one parametrised GPU launcher (r6; replaces the per-experiment
# scripts/gpu_r5*.sh — DESIGN.md §12 keeps their provenance table).
#
#   TAG=r6a bash scripts/gpu_run.sh STEP [STEP ...]
#
# STEP (each under its own time limit; the first failure ends the call):
#   test[=<pytest -k expr>]   the -m gpu suite (or the -k subset)  -> gpurun_out/$TAG_test.log
#   smoke                     __graft_entry__.smoke()               -> gpurun_out/$TAG_smoke.log
#   bench[=<bench.py args>]   one bench line                         -> gpurun_out/$TAG_bench.json
#   stats[=<bench.py args>]   rocprofv3 --kernel-trace --stats of a short bench -> gpurun_out/$TAG_stats/
#   pmc[=<bench.py args>]     scripts/gpu_profile.sh (trace + separate PMC passes) -> gpurun_out/$TAG_pmc/
#   cmd=<command>             anything else (tools/gemm_check, scripts/class_times.py, ...)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-rx}
n=0
run() {  # name seconds command...
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log" | cut -c1-900
  return $rc
}
for step in "$@"; do
  n=$((n + 1))
  key=${step%%=*}
  arg=""
  [ "$key" != "$step" ] && arg=${step#*=}
  case "$key" in
    test)
      if [ -n "$arg" ]; then
        run ${T}_test$n 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$arg" || exit $?
      else
        run ${T}_test$n 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
      fi ;;
    smoke)
      run ${T}_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      timeout -k 10 600 python bench.py $arg > gpurun_out/${T}_bench$n.json 2> gpurun_out/${T}_bench$n.err
      rc=$?; echo "== ${T}_bench$n rc=$rc"; tail -c 1500 gpurun_out/${T}_bench$n.json
      [ $rc -eq 0 ] || { tail -n 20 gpurun_out/${T}_bench$n.err; exit $rc; } ;;
    stats)
      run ${T}_stats$n 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_stats$n -o p -- python3 bench.py \
        ${arg:---steps 20 --warmup 3 --no-cpu-baseline --no-profile --no-f32 --sustain-seconds 0 --configs none} || exit $? ;;
    pmc)
      PROF_TAG=${T}_pmc$n EXTRA="$arg" bash scripts/gpu_profile.sh > gpurun_out/${T}_pmc$n.log 2>&1
      rc=$?; echo "== ${T}_pmc$n rc=$rc"; grep -h "rc=" gpurun_out/${T}_pmc$n.log | tr '\n' ' '; echo
      [ $rc -eq 0 ] || exit $rc ;;
    cmd)
      run ${T}_cmd$n 600 bash -c "$arg" || exit $? ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
