#!/bin/bash
# r3: tail2 ring depths, interleaved rounds (tools/tail_check)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "128 64 20 125" "64 64 40 249" "32 64 80 498"; do
  timeout -k 5 120 ./tools/tail_check $cfg 10 > gpurun_out/tc.log 2>&1 || { tail -5 gpurun_out/tc.log; exit 1; }
  echo "C=${cfg%% *}"; grep -E "round|tail2 <|out:|y1n" gpurun_out/tc.log
done
