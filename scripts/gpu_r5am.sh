# r5 end-of-session check at HEAD: full GPU suite + smoke (library rebuilt from the r5ai sources)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r5am_tests.log 2>&1 || { tail -40 gpurun_out/r5am_tests.log; exit 1; }
tail -2 gpurun_out/r5am_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5am_smoke.log 2>&1 || { tail -20 gpurun_out/r5am_smoke.log; exit 1; }
tail -2 gpurun_out/r5am_smoke.log
