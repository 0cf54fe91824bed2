#!/bin/bash
# r3 profiles at HEAD: rocprofv3 kernel-trace stats + PMC passes of C2 (headline only) and C3.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PROF_TAG=prof_r3i_c2 EXTRA="--configs none" timeout -k 10 560 bash scripts/gpu_profile.sh > gpurun_out/prof_c2.log 2>&1 || { tail -5 gpurun_out/prof_c2.log; exit 1; }
tail -3 gpurun_out/prof_c2.log
PROF_TAG=prof_r3i_c3 EXTRA="--arch ResNet293" BARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" \
  timeout -k 10 560 bash scripts/gpu_profile.sh > gpurun_out/prof_c3.log 2>&1 || { tail -5 gpurun_out/prof_c3.log; exit 1; }
tail -3 gpurun_out/prof_c3.log
