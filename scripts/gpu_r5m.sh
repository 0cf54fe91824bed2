# r5: family 7 persistent form (gemm_check variant 8) vs family 7 — bit identity + timing
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for c in cxc_bn conv_cat fc1 fc2 qkv out_proj cnn_c1 rb_ragged tiT_1x1 k3_ragged; do
  timeout -k 10 120 ./tools/gemm_check $c 10 78 > gpurun_out/r5p_$c.log 2>&1; rc=$?
  echo "== $c rc=$rc"; grep -E "differ|round 2|MISMATCH|identical|does not" gpurun_out/r5p_$c.log | cut -c1-200
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
