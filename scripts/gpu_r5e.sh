# r5: LayerNorm fold (LN1) — parity, per-class C4 times, C4 bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
run r5e_pytest_hubert 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hubert.py || exit $?
run r5e_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
run r5e_bench_c4 300 python -u bench.py --configs C4 || exit $?
