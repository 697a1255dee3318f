# round 6: the fused decoder over spans of 4 groups per wave, decoded in 4
# passes dealt by chunk size: GPU tests (three arrangements), kernel times of
# the bench frame and configs[2] (np2 variant beside), bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6u_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6u_tests.log; exit 1; }
tail -1 gpurun_out/r6u_tests.log
: > gpurun_out/r6u_kb.txt
for q in 50 90; do
  for v in 1 0; do
    echo "== q$q deal=$v" >> gpurun_out/r6u_kb.txt
    MYYUV_DEC_DEAL=$v KB_Q=$q timeout -k 10 120 python3 tools/kbench.py 20 >> gpurun_out/r6u_kb.txt 2>&1 || exit 1
    MYYUV_DEC_DEAL=$v KB_Q=$q timeout -k 10 120 python3 tools/kbench.py 20 8192x8192 >> gpurun_out/r6u_kb.txt 2>&1 || exit 1
  done
  echo "== q$q np2" >> gpurun_out/r6u_kb.txt
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/np2/libmyyuv_hip.so KB_Q=$q timeout -k 10 120 python3 tools/kbench.py 20 >> gpurun_out/r6u_kb.txt 2>&1 || exit 1
done
grep -E "==|huff_decode|q[59]0:" gpurun_out/r6u_kb.txt
bash tools/ab_bench.sh default MYYUV_DEC_DEAL=0 build_var/np2 > gpurun_out/r6u_ab.txt 2>&1 || exit 1
cat gpurun_out/r6u_ab.txt
