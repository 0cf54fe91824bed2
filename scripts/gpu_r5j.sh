# r5 profile at HEAD: rocprofv3 kernel stats + PMC passes of C4 (scripts/gpu_profile.sh)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
PROF_TAG=prof_r5_c4 EXTRA="--arch HuBERT_ECAPA_GLOB_c512" BARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" \
  timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_r5_c4.log 2>&1 || { tail -n 5 gpurun_out/prof_r5_c4.log; exit 1; }
grep -v "^[WE]2026" gpurun_out/prof_r5_c4.log | tail -n 8
