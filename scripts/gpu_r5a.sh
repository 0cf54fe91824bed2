# r5 GPU session: GEMM family check (6 / 7 / 8), the GPU test suite, headline bench A/B of the
# default tile family 7 against 8.  Each step under its own limit; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"; return $rc; }
run r5a_gemm_check 200 ./tools/gemm_check all 10 678 || exit $?
run r5a_bench_v7 400 python -u bench.py --configs C4,C5 --no-cpu-baseline --no-f32 || exit $?
run r5a_bench_v8 400 python -u bench.py --configs C4 --no-cpu-baseline --no-f32 --x3-variant 8 || exit $?
run r5a_pytest 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
