# r5: split-K ResNet head linear — ResNet parity / batch-of-one tests, C3 classes
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
run r5u_pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv3x3.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_streams.py -k "ResNet or resnet or res_tail or conv3x3 or c3 or SimAM or simam" || exit $?
run r5u_class_c3 300 python -u scripts/class_times.py --arch ResNet293 || exit $?
