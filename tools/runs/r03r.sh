set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03r_tests.log; exit 1; }
tail -2 gpurun_out/r03r_tests.log
timeout -k 10 200 python3 tools/h2d_probe.py
timeout -k 10 300 python3 tools/host_api_rate.py
