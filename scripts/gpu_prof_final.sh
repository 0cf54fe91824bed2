#!/bin/bash
# rocprofv3 kernel stats + PMC passes of the given configurations (CONFIGS:
# space-separated c2 / c3 / c4) at the default bench settings, into
# gpurun_out/prof_${ROUND_TAG}_<cfg>.  Every step time-limited; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${ROUND_TAG:-r2b}
for c in ${CONFIGS:-c2}; do
  case $c in
    c2) EXTRA="--configs none" ; BARGS="--steps 10 --warmup 2 --no-cpu-baseline" ;;
    c3) EXTRA="--arch ResNet293" ; BARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" ;;
    c4) EXTRA="--arch HuBERT_ECAPA_GLOB_c512" ; BARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-f32 --sustain-seconds 0" ;;
  esac
  PROF_TAG=prof_${R}_$c EXTRA="$EXTRA" BARGS="$BARGS" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "== prof $c rc=$rc"; tail -n 3 gpurun_out/prof_$c.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
