# round 6: payloads of chef-big q50 from the in-tree build and the
# iterative-minreg scheduler build, for tools/diag/payload_diff.py
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/diag/dump_payload.py chef-with-trumpet-big-DCT-50.myyuv gpurun_out/r6ar_default.bin &&
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/s_iterative-minreg/libmyyuv_hip.so timeout -k 10 120 python3 tools/diag/dump_payload.py chef-with-trumpet-big-DCT-50.myyuv gpurun_out/r6ar_minreg.bin
