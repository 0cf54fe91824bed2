# r5: HuBERT CNN layers 4..6 batch-wide — HuBERT tests, C4 classes, C4 bench pair
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
run r5s_pytest 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hubert.py tests/test_gpu_streams.py || exit $?
run r5s_class_c4 300 python -u scripts/class_times.py --arch HuBERT_ECAPA_GLOB_c512 || exit $?
A="--arch HuBERT_ECAPA_GLOB_c512 --no-cpu-baseline --no-f32 --steps 20"
run r5s_bench_a 300 python -u bench.py $A || exit $?
