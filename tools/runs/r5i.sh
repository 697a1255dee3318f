# round 5: per-phase cycles of the 64-block fused decoder (stamp build):
# setup, staging, table parse, symbol loop, transform; 12-frame launch alone
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 200 python3 tools/dec_phase.py 12 > gpurun_out/r5i_dec_phase.txt 2>&1; cat gpurun_out/r5i_dec_phase.txt
