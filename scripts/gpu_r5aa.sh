# r5: C2 per-class single-stream times at HEAD
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/class_times.py --arch ECAPA_TDNN_c1024 > gpurun_out/r5aa_class_c2.json 2> gpurun_out/r5aa_class_c2.err || { tail -20 gpurun_out/r5aa_class_c2.err; exit 1; }
cat gpurun_out/r5aa_class_c2.json
