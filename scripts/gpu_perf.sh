#!/bin/bash
# Parity tests + bench variants in one GPU session (each step time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-6} "gpurun_out/$name.log"
  return $rc
}
rc=0
if [ -z "${SKIP_TESTS:-}" ]; then
  run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider; rc=$?
fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# CFGS: bench configurations separated by '|'
IFS='|' read -ra CFG_LIST <<< "${CFGS:---precision 1 --x3-variant 1}"
for cfg in "${CFG_LIST[@]}"; do
  tag=$(echo $cfg | tr -d ' -')
  run bench_$tag 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $cfg || exit $?
done
exit $rc
