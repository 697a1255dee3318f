# CAP-16 tier occupancy: 3 (in-tree) against 5, 6 and 8 waves per SIMD (96 / 80 / 64 VGPRs, spilling)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/r16w5/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zzl_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zzl_tests.log; exit 1; }
tail -1 gpurun_out/r3zzl_tests.log
timeout -k 10 700 bash tools/ab_bench.sh default build_var/r16w5 build_var/r16w6 build_var/r16w8 > gpurun_out/r3zzl_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zzl_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zzl_ab.txt
cat gpurun_out/r3zzl_ab.txt
