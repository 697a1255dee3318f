set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03f_tests.log; exit 1; }
tail -2 gpurun_out/r03f_tests.log
timeout -k 10 900 bash tools/ab_bench.sh build_var/base default
