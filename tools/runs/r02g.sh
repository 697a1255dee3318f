set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02g_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02g_tests.log; exit 1; }
tail -2 gpurun_out/r02g_tests.log
bash tools/profile.sh r02g 20 && echo PROFILE_OK
