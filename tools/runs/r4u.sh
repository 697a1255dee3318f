# round 4: (1) K1's 32 spread lists (default) against every unit in list 0
# (nosp, same source); (2) the fused decoder's transform with eight lanes per
# block (xf::idct_rows8: half the transform's registers): xf8 (5 waves per
# SIMD), xf8w6 (6 waves, 80 VGPRs); parity tests of xf8w6, per-kernel times,
# the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/xf8w6/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4u_xf8w6_tests.log 2>&1; echo "xf8w6 tests rc=$?"; tail -2 gpurun_out/r4u_xf8w6_tests.log
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/nosp build_var/xf8 build_var/xf8w6 > gpurun_out/r4u_kab.txt 2>&1; cat gpurun_out/r4u_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/xf8w6 build_var/nosp > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4u_ab.txt && cat gpurun_out/r4u_ab.txt
