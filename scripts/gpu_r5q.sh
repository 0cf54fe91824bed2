# r5: C2 streams A/B (1 vs 2), interleaved pairs
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/$name.log').read().strip().splitlines()[-1]); print(d.get('value'), d.get('ms_per_step'), (d.get('value_sustained') or {}).get('value'))"; return $rc; }
A="--configs none --no-cpu-baseline --no-f32 --steps 40"
run r5q_s1a 300 python -u bench.py $A --opt streams=1 || exit $?
run r5q_s2a 300 python -u bench.py $A --opt streams=2 || exit $?
run r5q_s1b 300 python -u bench.py $A --opt streams=1 || exit $?
run r5q_s2b 300 python -u bench.py $A --opt streams=2 || exit $?
run r5q_s3a 300 python -u bench.py $A --opt streams=3 || exit $?
