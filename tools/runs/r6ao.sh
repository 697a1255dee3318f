# round 6: which kernels the iterative-minreg scheduler build (r6an: a bad code
# in the bench) gets wrong: the GPU tests on that build, without -x
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/s_iterative-minreg/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > gpurun_out/r6ao_tests.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/r6ao_tests.log | tail -60
