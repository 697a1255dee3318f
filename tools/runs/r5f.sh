# round 5: the fused decoder's wave cycles per phase (stamp build), one
# 24-frame launch group decoded alone
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 200 python3 tools/dec_phase.py 12 > gpurun_out/r5f_dec_phase.txt 2>&1; cat gpurun_out/r5f_dec_phase.txt
