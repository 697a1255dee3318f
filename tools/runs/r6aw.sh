# round 6: occupancy re-check in the 4 x 32 bench shape: the fused decoder at
# 4 / 6 waves per SIMD, K2's window kernel at 4 / 6 (default 5 / 5): bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_bench.sh default build_var/k5w4 build_var/k5w6 build_var/k2w4 build_var/k2w6 > gpurun_out/r6aw_ab.txt 2>&1 || { cat gpurun_out/r6aw_ab.txt; exit 1; }
cat gpurun_out/r6aw_ab.txt
