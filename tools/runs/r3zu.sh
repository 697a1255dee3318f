# span decoder ablations, kernels alone: no symbol decode (MYYUV_K5_EXP=1) in both decoders, no DC fast path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/k1_ab.py MYYUV_DECODER=wave default build_var/waveexp1 build_var/spanexp1 build_var/spannodc build_var/s128nodc > gpurun_out/r3zu_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zu_kernels.txt; exit 1; }
cat gpurun_out/r3zu_kernels.txt
