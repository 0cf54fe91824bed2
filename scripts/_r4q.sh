set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hubert.py tests/test_gpu_streams.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4q_tests.log 2>&1 || { tail -30 gpurun_out/r4q_tests.log; exit 1; }
tail -1 gpurun_out/r4q_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 8 --warmup 2 --no-cpu-baseline --no-f32 --sustain-seconds 2 --no-kernel-roofline --no-hubert-b64 > gpurun_out/r4q_c4.json 2> gpurun_out/r4q_c4.err || { tail -20 gpurun_out/r4q_c4.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4q_c4.json'));k=d['kernels'];print('C4', d['value'], d['value_sustained']['value'], {n:round(k[n]['ms_per_step'],2) for n in ('h_conv0','h_cnn','h_fc1','h_ln','h_proj') if n in k})"
done
