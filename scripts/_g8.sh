set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hubert.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "dma or bit_identical or segmented or matches_oracle_batched or chain" > gpurun_out/g8_tests.log 2>&1 || { tail -30 gpurun_out/g8_tests.log; exit 1; }
tail -1 gpurun_out/g8_tests.log
for r in 1 2; do
for v in 6 7 P; do
  if [ $v = P ]; then export WSP_G_PERSIST=1; vv=7; else unset WSP_G_PERSIST; vv=$v; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --configs none --sustain-seconds 2 --opt x3_variant=$vv > gpurun_out/g8_c2_v$v.json 2> gpurun_out/g8_c2.err || { tail -20 gpurun_out/g8_c2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/g8_c2_v$v.json'));k=d['kernels'];print('C2 v$v', d['value'], d['value_sustained']['value'], {n:k[n]['avg_ms'] for n in ('conv1x1_CxC','conv_cat') if n in k})"
done
done
unset WSP_G_PERSIST
for r in 1 2; do
for v in 6 7; do
  timeout -k 10 300 python -u bench.py --arch HuBERT_ECAPA_GLOB_c512 --steps 8 --warmup 2 --no-cpu-baseline --no-f32 --sustain-seconds 2 --no-kernel-roofline --no-hubert-b64 --opt x3_variant=$v > gpurun_out/g8_c4_v$v.json 2> gpurun_out/g8_c4.err || { tail -20 gpurun_out/g8_c4.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/g8_c4_v$v.json'));k=d['kernels'];print('C4 v$v', d['value'], d['value_sustained']['value'], {n:round(k[n]['ms_per_step'],2) for n in ('h_cnn','h_fc1','h_fc2','h_qkv','h_out_proj','h_proj') if n in k})"
done
done
