#!/bin/bash
# Focused GPU session: selected parity tests (TESTS, pytest -k KEXPR) then bench
# configurations (CFGS, '|'-separated).  Every GPU step is time-limited and a
# failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-8} "gpurun_out/$name.log"
  return $rc
}
if [ -n "${TESTS:-}" ]; then
  run pytest_q 600 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${KEXPR:+-k "$KEXPR"} || exit $?
fi
if [ -n "${CFGS:-}" ]; then
  IFS='|' read -ra CFG_LIST <<< "$CFGS"
  i=0
  for cfg in "${CFG_LIST[@]}"; do
    i=$((i+1))
    run bench_q$i 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --sustain-seconds 0 $cfg || exit $?
  done
fi
exit 0
