set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { tail -40 gpurun_out/r4f_tests.log; exit 1; }
tail -2 gpurun_out/r4f_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { tail -20 gpurun_out/r4f_smoke.log; exit 1; }
tail -2 gpurun_out/r4f_smoke.log
