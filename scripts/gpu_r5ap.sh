# r5: small linear with 2-row blocks for K >= 2048 — ECAPA parity, C2 stats
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
run r5ap_pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "ecapa or ECAPA or hubert_ecapa or c2 or smoke or api or eer" || exit $?
run r5ap_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5ap_stats -o p -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile --no-f32 --sustain-seconds 0 --configs none || exit $?
