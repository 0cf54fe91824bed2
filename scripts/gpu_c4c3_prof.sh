set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hubert.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_h.log 2>&1; rc=$?; echo "== pytest_h rc=$rc"; tail -3 gpurun_out/pytest_h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --no-cpu-baseline --no-f32 > gpurun_out/bench_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --arch HuBERT_ECAPA_GLOB_c512 --no-cpu-baseline --no-f32 --opt attn_lds=0 --sustain-seconds 0 > gpurun_out/bench_c4_old.log 2>&1 || exit $?
PROF_TAG=prof_r2_c4 EXTRA="--arch HuBERT_ECAPA_GLOB_c512" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_c4.log 2>&1 || exit $?
PROF_TAG=prof_r2_c3 EXTRA="--arch ResNet293" BARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_c3.log 2>&1 || exit $?
tail -n 2 gpurun_out/prof_c3.log
