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
run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "--precision 0" "--precision 1 --x3-variant 0" "--precision 1 --x3-variant 1"; do
  tag=$(echo $cfg | tr -d ' -')
  run bench_$tag 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $cfg || exit $?
done
exit $rc
