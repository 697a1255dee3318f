# round 4: the fused decoder's fast inverse transform (FMA chains, a proof per
# output, k_idct_fix for the unproven blocks): decfast (96 VGPRs, 88 B of
# spills), decfast4 (4 waves per SIMD: 113 VGPRs, no spills), decnl (fast
# path, no fix list: the ceiling, output may differ), dec0 (the reference's
# order, as before); per-kernel times and the bench (which checks the
# decoded frames against the pinned hash)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 500 python3 tools/k1_ab.py build_var/dec0 build_var/decfast build_var/decfast4 build_var/decnl > gpurun_out/r4m_kab.txt 2>&1; cat gpurun_out/r4m_kab.txt
timeout -k 10 700 bash tools/ab_bench.sh build_var/dec0 build_var/decfast build_var/decfast4 > /dev/null; cp gpurun_out/ab_bench.txt gpurun_out/r4m_ab.txt; cat gpurun_out/r4m_ab.txt; tail -3 gpurun_out/ab_one.err
# the parity tests must see the exact path's absence: decnl should fail them
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/decnl/libmyyuv_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "decompress or noise or edge" > gpurun_out/r4m_decnl_tests.log 2>&1; echo "decnl tests rc=$?"; tail -3 gpurun_out/r4m_decnl_tests.log
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/decfast/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m_decfast_tests.log 2>&1; echo "decfast tests rc=$?"; tail -3 gpurun_out/r4m_decfast_tests.log
