# round 6: k_fdct_fix's grid in the bench (q50: MYYUV_FIX_GRID caps it below
# the resident count) -- bench A/B of 64 / 256 / 1024 workgroups; then
# k_huff_encode_wide's grid behind the CAP-16 tier (MYYUV_WIDE_TIER_GRID)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_bench.sh default MYYUV_FIX_GRID=64 MYYUV_FIX_GRID=256 MYYUV_FIX_GRID=1024 > gpurun_out/r6z_ab.txt 2>&1 || exit 1
cat gpurun_out/r6z_ab.txt
bash tools/ab_bench.sh default MYYUV_WIDE_TIER_GRID=64 MYYUV_WIDE_TIER_GRID=256 > gpurun_out/r6z_ab2.txt 2>&1 || exit 1
cat gpurun_out/r6z_ab2.txt
