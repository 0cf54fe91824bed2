# r5 final checkpoint (fbank rework, split-K heads, scoring writers): full GPU suite, smoke, default bench
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
R=r5ai
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || { tail -40 gpurun_out/${R}_tests.log; exit 1; }
tail -2 gpurun_out/${R}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail -20 gpurun_out/${R}_smoke.log; exit 1; }
tail -2 gpurun_out/${R}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail -20 gpurun_out/${R}_bench.err; exit 1; }
tail -c 1500 gpurun_out/${R}_bench.json
