# round 5: the fused single-pass encoder (MYYUV_ENCODER=fused) against K1 -> K2
# with the round-5 kernels: kernel times and bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default MYYUV_ENCODER=fused > gpurun_out/r5y_kab.txt 2>&1; cat gpurun_out/r5y_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default MYYUV_ENCODER=fused > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5y_ab.txt && cat gpurun_out/r5y_ab.txt
