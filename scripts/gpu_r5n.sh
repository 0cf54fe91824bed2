# r5: tail2_kernel on 8-wave blocks — bit identity, C3 per-class / per-stage times
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
run r5n_pytest 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv3x3.py -k "tail_8_wave" || exit $?
run r5n_c3_w0 300 python -u scripts/class_times.py --arch ResNet293 --opt tail_waves8=0 || exit $?
run r5n_c3_w7 300 python -u scripts/class_times.py --arch ResNet293 --opt tail_waves8=7 || exit $?
run r5n_c3_w0b 300 python -u scripts/class_times.py --arch ResNet293 --opt tail_waves8=0 || exit $?
