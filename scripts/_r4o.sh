set -u -o pipefail
mkdir -p gpurun_out
for m in 1 2; do
  timeout -k 5 120 ./tools/g7_check 127488 1024 1024 10 1 $m > gpurun_out/r4o_g_m$m.log 2>&1 || { tail -5 gpurun_out/r4o_g_m$m.log; exit 1; }
  echo "mode $m"; grep -E "round [123]|max|column" gpurun_out/r4o_g_m$m.log
done
timeout -k 5 120 ./tools/g7_check 63744 3072 768 10 3 0 > gpurun_out/r4o_g_fc1.log 2>&1 || { tail -5 gpurun_out/r4o_g_fc1.log; exit 1; }
echo fc1; grep -E "round [23]|max" gpurun_out/r4o_g_fc1.log
timeout -k 5 120 ./tools/g7_check 63744 768 3072 10 0 2 > gpurun_out/r4o_g_fc2.log 2>&1 || { tail -5 gpurun_out/r4o_g_fc2.log; exit 1; }
echo fc2; grep -E "round [23]|max" gpurun_out/r4o_g_fc2.log
for r in 1 2; do
for v in 7 8; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --configs none --sustain-seconds 2 --opt x3_variant=$v > gpurun_out/r4o_c2.json 2> gpurun_out/r4o_c2.err || { tail -20 gpurun_out/r4o_c2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4o_c2.json'));k=d['kernels'];print('C2 v$v', d['value'], d['value_sustained']['value'], {n:k[n]['avg_ms'] for n in ('layer1','conv1x1_CxC','conv_cat') if n in k})"
done
done
