# round 6: k_scan_chain's sizes per thread, second A/B: 32 against 16, six
# alternating rounds (tools/ab_bench.sh twice), full GPU tests on 32.
# (A first try with 64 failed a host-batch decode test with a HIP runtime
# error: not a candidate.)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/spt32/libmyyuv_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6az_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6az_tests.log; exit 1; }
echo "spt32 $(tail -1 gpurun_out/r6az_tests.log)"
bash tools/ab_bench.sh default build_var/spt32 > gpurun_out/r6az_ab1.txt 2>&1 || { cat gpurun_out/r6az_ab1.txt; exit 1; }
bash tools/ab_bench.sh build_var/spt32 default > gpurun_out/r6az_ab2.txt 2>&1 || { cat gpurun_out/r6az_ab2.txt; exit 1; }
cat gpurun_out/r6az_ab1.txt gpurun_out/r6az_ab2.txt
