# the batch tests, with a 9-frame 1024x1024 q90 batch whose overflow list passes the CAP-16 tier's gate
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "batch_device_matches" --timeout 300 --timeout-method thread > gpurun_out/r3zzp_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zzp_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r3zzp_tests.log | tail -10
