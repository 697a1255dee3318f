# round 5: K2 windows of 8 tiles (win8) again: GPU tests of the win8 build
# (MYYUV_HIP_LIB), six alternating bench rounds against default (4 tiles)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/win8/libmyyuv_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5az_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5az_tests.log; exit 1; }
tail -1 gpurun_out/r5az_tests.log
timeout -k 10 700 bash tools/ab_bench.sh build_var/win8 default > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5az_ab.txt && cat gpurun_out/r5az_ab.txt
timeout -k 10 700 bash tools/ab_bench.sh default build_var/win8 > /dev/null && cat gpurun_out/ab_bench.txt >> gpurun_out/r5az_ab.txt && cat gpurun_out/ab_bench.txt
