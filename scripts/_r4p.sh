set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 || { tail -40 gpurun_out/r4p_tests.log; exit 1; }
tail -2 gpurun_out/r4p_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4p_smoke.log 2>&1 || { tail -20 gpurun_out/r4p_smoke.log; exit 1; }
tail -2 gpurun_out/r4p_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r4p_bench.json 2> gpurun_out/r4p_bench.err || { tail -20 gpurun_out/r4p_bench.err; exit 1; }
tail -c 700 gpurun_out/r4p_bench.json
PROF_TAG=r4p_c2 EXTRA="--configs none" bash scripts/gpu_profile.sh > gpurun_out/r4p_prof_c2.log 2>&1 || { tail -20 gpurun_out/r4p_prof_c2.log; exit 1; }
PROF_TAG=r4p_c4 EXTRA="--arch HuBERT_ECAPA_GLOB_c512" BARGS="--steps 6 --warmup 2 --no-cpu-baseline --no-hubert-b64" bash scripts/gpu_profile.sh > gpurun_out/r4p_prof_c4.log 2>&1 || { tail -20 gpurun_out/r4p_prof_c4.log; exit 1; }
PROF_TAG=r4p_c3 EXTRA="--arch ResNet293" BARGS="--steps 4 --warmup 2 --no-cpu-baseline" bash scripts/gpu_profile.sh > gpurun_out/r4p_prof_c3.log 2>&1 || { tail -20 gpurun_out/r4p_prof_c3.log; exit 1; }
grep -h "rc=" gpurun_out/r4p_prof_c2.log gpurun_out/r4p_prof_c4.log gpurun_out/r4p_prof_c3.log | tr '\n' ' '
