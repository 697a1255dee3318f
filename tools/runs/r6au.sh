# round 6: the CAP-16 tier's windows for batches: 4 / 2 64-block batches per
# wave, each window counting-sorted by message length (MYYUV_R16_WIN), vs list
# order (default = the in-tree build): GPU tests on win4, one 32-frame launch
# group alone, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/win4/libmyyuv_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6au_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6au_tests.log; exit 1; }
tail -1 gpurun_out/r6au_tests.log
K1AB_B=32 timeout -k 10 300 python3 tools/k1_ab.py default build_var/win4 build_var/win2 > gpurun_out/r6au_alone.txt 2>&1 || { tail -20 gpurun_out/r6au_alone.txt; exit 1; }
grep "r16" gpurun_out/r6au_alone.txt | head
bash tools/ab_bench.sh default build_var/win4 build_var/win2 > gpurun_out/r6au_ab.txt 2>&1 || { cat gpurun_out/r6au_ab.txt; exit 1; }
cat gpurun_out/r6au_ab.txt
