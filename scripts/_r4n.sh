set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hubert.py tests/test_gpu_fullsize.py tests/test_gpu_api.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1 || { tail -30 gpurun_out/r4n_tests.log; exit 1; }
tail -1 gpurun_out/r4n_tests.log
for r in 1 2; do
for cfg in "x3_variant=6 streams=1" "x3_variant=7 streams=1" "x3_variant=7 streams=2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --configs none --sustain-seconds 2 --opt $1 --opt $2 > gpurun_out/r4n_c2.json 2> gpurun_out/r4n_c2.err || { tail -20 gpurun_out/r4n_c2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4n_c2.json'));k=d['kernels'];print('C2 $1 $2', d['value'], d['value_sustained']['value'], {n:k[n]['avg_ms'] for n in ('layer1','conv1x1_CxC','conv_cat') if n in k})"
done
done
