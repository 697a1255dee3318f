# the CAP-16 overflow tier for batches too (MYYUV_R16_BATCH=1) at the 3 x 16 launch shape, whose 16-frame lists
# (~132k blocks) exceed one resident round of the CAP-64 pass
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/r16b/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zze_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zze_tests.log; exit 1; }
tail -1 gpurun_out/r3zze_tests.log
timeout -k 10 500 bash tools/ab_bench.sh default build_var/r16b > gpurun_out/r3zze_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zze_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zze_ab.txt
cat gpurun_out/r3zze_ab.txt
