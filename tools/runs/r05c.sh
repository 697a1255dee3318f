set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r05c_tests.log; exit 1; }
tail -2 gpurun_out/r05c_tests.log
for L in build_var/base yuv-manipulations-2_amd; do
  for Q in 50 90; do
    KB_Q=$Q MYYUV_HIP_LIB=$PWD/$L/libmyyuv_hip.so timeout -k 10 120 python3 tools/kbench.py 20 8192x8192 || exit 1
  done
done
timeout -k 10 600 bash tools/ab_bench.sh build_var/base default && cp gpurun_out/ab_bench.txt gpurun_out/r05c_ab.txt
