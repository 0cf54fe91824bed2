# r5: split-K head partial-slice test
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "split_k or resnet_matches_oracle" > gpurun_out/r5ae.log 2>&1; rc=$?
tail -n 30 gpurun_out/r5ae.log; exit $rc
