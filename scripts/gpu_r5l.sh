# r5: Res2Net strip addend loads 12 k-steps ahead — bit-identity tests, C2 per-class times
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
run r5l_pytest_res2 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_res2.py || exit $?
run r5l_class_c2 300 python -u scripts/class_times.py --arch ECAPA_TDNN_c1024 || exit $?
run r5l_pytest_tail 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv3x3.py || exit $?
run r5l_class_c3 300 python -u scripts/class_times.py --arch ResNet293 || exit $?
