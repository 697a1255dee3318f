# CAP-16 tier occupancy: 131 VGPRs (3 waves/SIMD, in-tree) against 128 (4 waves, no spills) and 96 (5 waves, 8 spills)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/r16w4/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zzk_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zzk_tests.log; exit 1; }
tail -1 gpurun_out/r3zzk_tests.log
timeout -k 10 700 bash tools/ab_bench.sh default build_var/r16w4 build_var/r16w5 > gpurun_out/r3zzk_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zzk_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zzk_ab.txt
cat gpurun_out/r3zzk_ab.txt
