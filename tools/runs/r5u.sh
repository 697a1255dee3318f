# round 5: per-phase cycles of the fused decoder and K2's stages with the
# round-5 kernels (stamp build, -DMYYUV_STAMPS)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 200 python3 tools/dec_phase.py 12 > gpurun_out/r5u_dec_phase.txt 2>&1; cat gpurun_out/r5u_dec_phase.txt
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 300 python3 tools/k2_time.py > gpurun_out/r5u_k2_time.txt 2>&1; cat gpurun_out/r5u_k2_time.txt
