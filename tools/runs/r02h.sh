set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02h_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02h_tests.log; exit 1; }
tail -2 gpurun_out/r02h_tests.log
MYYUV_K2_STASH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 300 --timeout-method thread -k "split" > gpurun_out/r02h_stash.log 2>&1 || { echo STASH_TESTS_FAILED; tail -40 gpurun_out/r02h_stash.log; exit 1; }
tail -2 gpurun_out/r02h_stash.log
bash tools/ab_bench.sh default MYYUV_K2_STASH=1
