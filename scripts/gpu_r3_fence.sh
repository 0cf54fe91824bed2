#!/bin/bash
# r3: scheduling-fence check: conv3x3 / tail parity, then C3 (ResNet293) and ResNet34 benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_fence_tests.log 2>&1 || { echo "conv3x3 tests failed"; tail -30 gpurun_out/r3_fence_tests.log; exit 1; }
tail -2 gpurun_out/r3_fence_tests.log
for a in ResNet293 ResNet34; do
  timeout -k 10 300 python -u bench.py --arch $a --steps 10 --warmup 2 --no-cpu-baseline --no-f32 --configs "" \
    --sustain-seconds 2 > gpurun_out/r3_fence_$a.json 2> gpurun_out/r3_fence_$a.err || { echo "bench failed"; tail gpurun_out/r3_fence_$a.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3_fence_$a.json'));k=d['kernels'];print('$a', d['value'], d['value_sustained']['value'], d['roofline']['frac'], {c: round(k[c]['ms_per_step'],2) for c in k if '.' in c or c.startswith('res_')})"
done
