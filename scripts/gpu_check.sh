#!/bin/bash
# One GPU session: parity tests, smoke, bench.  Every GPU step has its own
# time limit; a fault / abort / timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2"}
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 600 python bench.py $BENCH_ARGS || exit $?
exit $rc
