# span decoder variants: 256-block spans (in-tree, 4 waves/SIMD), unsorted, 128-block spans, 64-block spans at 5 waves
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/k1_ab.py MYYUV_DECODER=wave default build_var/s256ns build_var/s128w4 build_var/s64w5 > gpurun_out/r3zt_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zt_kernels.txt; exit 1; }
cat gpurun_out/r3zt_kernels.txt
timeout -k 10 700 bash tools/ab_bench.sh MYYUV_DECODER=wave default build_var/s128w4 build_var/s64w5 > gpurun_out/r3zt_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zt_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zt_ab.txt
cat gpurun_out/r3zt_ab.txt
