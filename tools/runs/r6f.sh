# round 6: k_fdct_fix grid at q90 (per-block lists), and the fused encoder
# against K1 -> K2 (kernel times, bench A/B, SQ counters of the bench groups)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r6f_fixgrid.txt
for G in 0 64 128 256 512 1024; do
  MYYUV_FIX_GRID=$G MYYUV_FIX_QMAX=100 KB_Q=90 timeout -k 10 200 python3 -u tools/kbench.py 10 8192x8192 > gpurun_out/r6f_kb.txt 2>&1 || { tail gpurun_out/r6f_kb.txt; exit 1; }
  echo "grid $G $(grep -E 'fdct_fix|fdct_quant|roundtrip' gpurun_out/r6f_kb.txt | tr -s ' ' | tr '\n' ' ')" >> gpurun_out/r6f_fixgrid.txt
done
cat gpurun_out/r6f_fixgrid.txt
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default MYYUV_ENCODER=fused > gpurun_out/r6f_kab.txt 2>&1; cat gpurun_out/r6f_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default MYYUV_ENCODER=fused > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r6f_ab.txt && cat gpurun_out/r6f_ab.txt
SQ_BENCH=1 timeout -k 10 600 bash tools/sq_counters.sh r6f_split && echo SQ_SPLIT_OK
MYYUV_ENCODER=fused SQ_BENCH=1 timeout -k 10 600 bash tools/sq_counters.sh r6f_fused && echo SQ_FUSED_OK
