# r5: conv0 on packed f32 — HuBERT parity subset, C4 classes
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
run r5r_pytest 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hubert.py -k "hidden_state or featurizer or short_input or batch_rows or ragged or c4_bench" || exit $?
run r5r_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
