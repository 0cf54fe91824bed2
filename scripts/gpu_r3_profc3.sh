#!/bin/bash
# r3 final: C3 rocprofv3 kernel-trace stats + PMC passes at HEAD
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PROF_TAG=prof_r3l_c3 EXTRA="--arch ResNet293" BARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" \
  timeout -k 10 560 bash scripts/gpu_profile.sh > gpurun_out/prof_c3l.log 2>&1 || { tail -5 gpurun_out/prof_c3l.log; exit 1; }
tail -2 gpurun_out/prof_c3l.log
