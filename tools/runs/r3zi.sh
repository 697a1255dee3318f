# overflow pass lanes per workgroup (64 in-tree; wl32 / wl16: fewer blocks per wave, a shorter
# union of the lanes' loops) in the 4 x 8 pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/k1_ab.py default build_var/wl32 build_var/wl16 > gpurun_out/r3zi_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zi_kernels.txt; exit 1; }
cat gpurun_out/r3zi_kernels.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/wl32 build_var/wl16 > gpurun_out/r3zi_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zi_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zi_ab.txt
cat gpurun_out/r3zi_ab.txt
