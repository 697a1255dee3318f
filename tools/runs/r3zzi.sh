# with the CAP-16 tier taking the batches' long lists: K2's classify sends blocks with >= 11 / 13 / 16 possible
# distinct symbols straight to the overflow list (dn11/13/16), and the wave pass for batches' rest lists (bw)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/dn11/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zzi_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zzi_tests.log; exit 1; }
tail -1 gpurun_out/r3zzi_tests.log
timeout -k 10 400 python3 tools/k1_ab.py default build_var/dn11 build_var/dn13 build_var/dn16 build_var/bw > gpurun_out/r3zzi_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zzi_kernels.txt; exit 1; }
cat gpurun_out/r3zzi_kernels.txt
timeout -k 10 700 bash tools/ab_bench.sh default build_var/dn11 build_var/dn13 build_var/dn16 build_var/bw > gpurun_out/r3zzi_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zzi_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zzi_ab.txt
cat gpurun_out/r3zzi_ab.txt
