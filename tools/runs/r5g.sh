# round 5: per-phase decoder cycles, the 64-block fused decoder (stamps64:
# decode = setup + staging + parse + symbols, then the transform) against the
# 128-block span decoder (stamps), one 12-frame launch group alone
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in stamps64 stamps; do
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/$v/libmyyuv_hip.so timeout -k 10 200 python3 tools/dec_phase.py 12 > gpurun_out/r5g_$v.txt 2>&1; echo "== $v"; cat gpurun_out/r5g_$v.txt
done
