# r5: direct pos_conv kernel — parity, per-class C4 times against the grouped GEMM, C4 bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-3000; return $rc; }
run r5c_pytest_posconv 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_hubert.py -k "direct_pos_conv or hidden_state or featurizer or ragged" || exit $?
run r5c_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
run r5c_class_c4_pc0 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 --opt pos_conv=0 || exit $?
run r5c_bench_c4 300 python -u bench.py --configs C4 || exit $?
