# r5: vectorised trial-score / AS-Norm writers — scoring GPU tests, C5 pipeline
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-900; return $rc; }
run r5ab_pytest 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eer.py tests/test_gpu_api.py tests/test_gpu_fullsize.py -k "score or norm or eer or trial or c5 or C5" || exit $?
run r5ab_c5 300 python -u scripts/bench_c5.py || exit $?
