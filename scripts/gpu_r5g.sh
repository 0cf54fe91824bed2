# r5: C4 bench A/B, ln_fold 1 vs 0, two interleaved pairs
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; python3 -c "
import json,sys; d=json.loads(open('gpurun_out/$name.log').read().strip().splitlines()[-1]); c=d.get('configs',{}).get('C4',d); print(c.get('value'), c.get('ms_per_step'))"; return $rc; }
A="--arch HuBERT_ECAPA_GLOB_c512 --no-cpu-baseline --no-f32 --steps 20"
run r5g_lf1a 300 python -u bench.py $A --opt ln_fold=1 || exit $?
run r5g_lf0a 300 python -u bench.py $A --opt ln_fold=0 || exit $?
run r5g_lf1b 300 python -u bench.py $A --opt ln_fold=1 || exit $?
run r5g_lf0b 300 python -u bench.py $A --opt ln_fold=0 || exit $?
