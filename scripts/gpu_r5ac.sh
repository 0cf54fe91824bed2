# r5: family 7 staggered first-round blocks (gemm_check variant 8 = family 7 + stagger) — bit identity + timing
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
for st in 2 4 8; do
  for c in cxc_bn layer1 conv_cat; do
    WSP_STAGGER=$st run r5ac_${c}_s$st 200 ./tools/gemm_check $c 10 78 || exit $?
  done
done
