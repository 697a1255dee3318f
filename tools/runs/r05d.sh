set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r05d_tests.log; exit 1; }
tail -1 gpurun_out/r05d_tests.log
MYYUV_HIP_LIB=$PWD/build_var/s32/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d_tests_s32.log 2>&1 || { echo TESTS_S32_FAILED; tail -40 gpurun_out/r05d_tests_s32.log; exit 1; }
tail -1 gpurun_out/r05d_tests_s32.log
for L in build_var/base yuv-manipulations-2_amd build_var/s24 build_var/s32 build_var/s40; do
  for Q in 50 90; do
    KB_Q=$Q MYYUV_HIP_LIB=$PWD/$L/libmyyuv_hip.so timeout -k 10 120 python3 tools/kbench.py 20 8192x8192 | grep -E "q$Q|wide" || exit 1
  done
done
timeout -k 10 900 bash tools/ab_bench.sh build_var/base default build_var/s24 build_var/s32 build_var/s40 && cp gpurun_out/ab_bench.txt gpurun_out/r05d_ab.txt
