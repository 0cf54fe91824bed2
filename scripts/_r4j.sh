set -u -o pipefail
mkdir -p gpurun_out
for m in 4 1; do
  timeout -k 5 120 ./tools/g7_check 127488 1024 1024 10 1 $m > gpurun_out/r4j_g7_m$m.log 2>&1 || { tail -5 gpurun_out/r4j_g7_m$m.log; exit 1; }
  echo "mode $m"; grep -E "round [23]|max|column" gpurun_out/r4j_g7_m$m.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hubert.py tests/test_gpu_fullsize.py tests/test_gpu_catgate.py tests/test_gpu_streams.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1 || { tail -30 gpurun_out/r4j_tests.log; exit 1; }
tail -1 gpurun_out/r4j_tests.log
for r in 1 2; do
for v in 6 7; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --configs none --sustain-seconds 2 --opt x3_variant=$v > gpurun_out/r4j_c2_v$v.json 2> gpurun_out/r4j_c2.err || { tail -20 gpurun_out/r4j_c2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4j_c2_v$v.json'));k=d['kernels'];print('C2 v$v', d['value'], d['value_sustained']['value'], {n:k[n]['avg_ms'] for n in ('conv1x1_CxC','conv_cat','layer1','pool_linear1','se') if n in k})"
done
done
