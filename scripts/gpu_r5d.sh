# r5: pos_conv with 128-k W stages
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
run r5d_pytest_posconv 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_hubert.py -k "direct_pos_conv" || exit $?
run r5d_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
