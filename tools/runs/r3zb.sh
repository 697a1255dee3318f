# K2 window sort: classify + sort share (k2exp1 exits after the sort) and the
# SQ counters of the bench's launch groups with the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/k1_ab.py default build_var/k2exp1 > gpurun_out/r3zb_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zb_kernels.txt; exit 1; }
cat gpurun_out/r3zb_kernels.txt
SQ_BENCH=1 bash tools/sq_counters.sh r3zb || { echo SQ_FAILED; exit 1; }
python3 tools/sq_report.py r3zb > gpurun_out/r3zb_sq.txt 2>&1 || true
grep -A40 "== huff_encode$" gpurun_out/r3zb_sq.txt | head -36
