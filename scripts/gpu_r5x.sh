# r5: fbank per-lane twiddle table — fbank tests, C2 stats + LDS PMC
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
run r5x_pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "fbank or Fbank or frontend or c2 or C2 or ecapa or ECAPA" || exit $?
run r5x_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5x_stats -o p -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile --no-f32 --sustain-seconds 0 --configs none || exit $?
run r5x_pmc 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/r5x_pmc -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-f32 --sustain-seconds 0 --configs none || exit $?
