#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -q --timeout 120 --timeout-method thread \
  -k "res_tail" > gpurun_out/t_t2dbg.log 2>&1; grep -E "PASS|FAIL|passed|failed" gpurun_out/t_t2dbg.log | tail -30
