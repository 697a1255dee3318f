# round 5: K2 per-stage wave cycles (stamp build), bench frame
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 300 python3 tools/k2_time.py > gpurun_out/r5j_k2_time.txt 2>&1; cat gpurun_out/r5j_k2_time.txt
