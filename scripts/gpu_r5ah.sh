# r5 final profiles at HEAD: rocprofv3 kernel stats + PMC passes of C2, C3 and C4 (scripts/gpu_profile.sh)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
PROF_TAG=prof_r5y_c2 EXTRA="--configs none" timeout -k 10 560 bash scripts/gpu_profile.sh > gpurun_out/prof_r5y_c2.log 2>&1 || { tail -n 5 gpurun_out/prof_r5y_c2.log; exit 1; }
tail -n 2 gpurun_out/prof_r5y_c2.log
PROF_TAG=prof_r5y_c3 EXTRA="--arch ResNet293" BARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" \
  timeout -k 10 560 bash scripts/gpu_profile.sh > gpurun_out/prof_r5y_c3.log 2>&1 || { tail -n 5 gpurun_out/prof_r5y_c3.log; exit 1; }
tail -n 2 gpurun_out/prof_r5y_c3.log
PROF_TAG=prof_r5y_c4 EXTRA="--arch HuBERT_ECAPA_GLOB_c512" BARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" \
  timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_r5y_c4.log 2>&1 || { tail -n 5 gpurun_out/prof_r5y_c4.log; exit 1; }
grep -v "^[WE]2026" gpurun_out/prof_r5y_c4.log | tail -n 8
