# round 5 diagnostic: K2's per-wave window phases (stamp build): prologue,
# fetch + coefficient load + build, emission + lists, epilogue; and the
# decoder's phases with the round's final kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 200 python3 tools/k2_phase.py 24 > gpurun_out/r5as_k2_phase.txt 2>&1; cat gpurun_out/r5as_k2_phase.txt
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 200 python3 tools/dec_phase.py 12 > gpurun_out/r5as_dec_phase.txt 2>&1; cat gpurun_out/r5as_dec_phase.txt
