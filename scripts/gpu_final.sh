#!/bin/bash
# Final round checkpoint: full GPU suite, smoke, default bench, C2 rocprof + PMC at HEAD
# (PROF_TAG from ROUND_TAG).  Every step time-limited; the first failure ends it.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${ROUND_TAG:-rx}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || { tail -40 gpurun_out/${R}_tests.log; exit 1; }
tail -2 gpurun_out/${R}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail -20 gpurun_out/${R}_smoke.log; exit 1; }
tail -2 gpurun_out/${R}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail -20 gpurun_out/${R}_bench.err; exit 1; }
tail -c 900 gpurun_out/${R}_bench.json
PROF_TAG=${R}_c2 EXTRA="--configs none" bash scripts/gpu_profile.sh > gpurun_out/${R}_prof_c2.log 2>&1 || { tail -20 gpurun_out/${R}_prof_c2.log; exit 1; }
grep -h "rc=" gpurun_out/${R}_prof_c2.log | tr '\n' ' '
