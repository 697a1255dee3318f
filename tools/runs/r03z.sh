set -o pipefail
cd $GRAFT_REPO_ROOT
for v in l32 l16; do
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/$v/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q -k "noise or chef or batch" --timeout 300 --timeout-method thread > gpurun_out/r03z_tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -40 gpurun_out/r03z_tests_$v.log; exit 1; }
tail -1 gpurun_out/r03z_tests_$v.log
done
timeout -k 10 900 bash tools/ab_bench.sh build_var/base build_var/l32 build_var/l16
