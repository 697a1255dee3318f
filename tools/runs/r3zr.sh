# K2: four message-length buckets (<= 8 / 16 / 32 / longer; msz4) and runs lightest first (light)
# against the in-tree build (three buckets, heaviest first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/k1_ab.py default build_var/msz4 build_var/light > gpurun_out/r3zr_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zr_kernels.txt; exit 1; }
cat gpurun_out/r3zr_kernels.txt
timeout -k 10 600 bash tools/ab_bench.sh default build_var/msz4 build_var/light > gpurun_out/r3zr_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zr_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zr_ab.txt
cat gpurun_out/r3zr_ab.txt
