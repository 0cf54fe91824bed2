# r5: attention with the next chunk's S^T MFMAs ahead of the softmax
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
run r5i_pytest_attn 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_hubert.py -k "attention or c4_bench_shape or ragged" || exit $?
run r5i_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
