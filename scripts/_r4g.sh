set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err || { tail -20 gpurun_out/r4g_bench.err; exit 1; }
tail -c 1200 gpurun_out/r4g_bench.json
PROF_TAG=r4g_c2 bash scripts/gpu_profile.sh || exit 1
PROF_TAG=r4g_c4 EXTRA="--arch HuBERT_ECAPA_GLOB_c512" BARGS="--steps 6 --warmup 2 --no-cpu-baseline --no-hubert-b64" bash scripts/gpu_profile.sh || exit 1
