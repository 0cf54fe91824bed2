# r5: LayerNorm fold, stats per lane
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-1200; return $rc; }
run r5f_pytest_fold 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_hubert.py -k "layernorm_fold or c4_bench_shape" || exit $?
run r5f_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
run r5f_class_c4_lf0 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 --opt ln_fold=0 || exit $?
