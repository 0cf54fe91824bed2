#!/bin/bash
# rocprofv3 kernel-trace stats of the bench + separate PMC passes (HBM bytes,
# MFMA / wave-cycle counters).  Every step time-limited; a fault ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/${PROF_TAG:-prof}
mkdir -p $OUT
EXTRA=${EXTRA:-""}  # workload flags for every pass, e.g. "--arch HuBERT_ECAPA_GLOB_c512"
BARGS=${BARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 2 ]; }
timeout -k 10 300 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py $BARGS $EXTRA > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -n 3 $OUT/trace.log; ok $rc || exit $rc
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-f32 --sustain-seconds 0 $EXTRA > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($pmc) rc=$rc"; tail -n 2 $OUT/pmc$i.log; ok $rc || exit $rc
done
exit 0
