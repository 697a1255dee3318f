# round 3: the fused single-pass encoder (k_encode_tile, MYYUV_ENCODER=fused)
# against split K1 -> K2: SQ counters of the bench's launch groups for both,
# and the bench A/B (state its ceiling with counters)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SQ_BENCH=1 bash tools/sq_counters.sh r3split && MYYUV_ENCODER=fused SQ_BENCH=1 bash tools/sq_counters.sh r3fused
cd $GRAFT_REPO_ROOT
python3 tools/sq_report.py r3split > gpurun_out/r3s_sq_split.txt && python3 tools/sq_report.py r3fused > gpurun_out/r3s_sq_fused.txt
timeout -k 10 900 bash tools/ab_bench.sh default MYYUV_ENCODER=fused && cp gpurun_out/ab_bench.txt gpurun_out/r3s_ab.txt && cat gpurun_out/r3s_ab.txt
