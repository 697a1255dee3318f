set -o pipefail
cd $GRAFT_REPO_ROOT
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/bw/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q -k "batch and not sorted" --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04c_tests.log; exit 1; }
tail -1 gpurun_out/r04c_tests.log
timeout -k 10 900 bash tools/ab_bench.sh build_var/base build_var/bw
