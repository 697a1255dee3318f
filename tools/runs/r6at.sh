# round 6: the fused decoder's groups in XCD-major order (dec_group_of,
# MYYUV_DEC_XCD) vs dispatch order: GPU tests on the XCD-major build, one
# 32-frame launch group alone per kernel, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/xcd1/libmyyuv_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6at_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6at_tests.log; exit 1; }
tail -1 gpurun_out/r6at_tests.log
K1AB_B=32 timeout -k 10 300 python3 tools/k1_ab.py build_var/xcd0 build_var/xcd1 > gpurun_out/r6at_alone.txt 2>&1 || { tail -20 gpurun_out/r6at_alone.txt; exit 1; }
grep -o "^[^ ]* .*decode_idct=[0-9.]*" gpurun_out/r6at_alone.txt | head
bash tools/ab_bench.sh build_var/xcd0 build_var/xcd1 > gpurun_out/r6at_ab.txt 2>&1 || { cat gpurun_out/r6at_ab.txt; exit 1; }
cat gpurun_out/r6at_ab.txt
