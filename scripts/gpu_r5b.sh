# r5: no-SLP family 7 / 8 GEMM check; per-class single-stream times of C4 and C3
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-3000; return $rc; }
run r5b_gemm_noslp 200 ./tools/gemm_check_noslp all 10 78 || exit $?
run r5b_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
run r5b_class_c3 300 python -u scripts/class_times.py --arch ResNet293 || exit $?
