set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_reference_binding.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02e_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02e_tests.log; exit 1; }
tail -15 gpurun_out/r02e_tests.log
