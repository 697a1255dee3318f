# occupancy re-check at the 3 x 24 shape with the CAP-16 tier: K2 at 4 / 6 workgroups per CU, K1's grid at 75 %
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_bench.sh default build_var/k2w4 build_var/k2w6 MYYUV_K1_GRID_PCT=75 > gpurun_out/r3zzm_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zzm_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zzm_ab.txt
cat gpurun_out/r3zzm_ab.txt
