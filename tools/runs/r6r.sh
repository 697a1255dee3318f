# round 6: the fused decoder over blocks dealt to the lanes by chunk size (k_deal, 4096-block segments, XCD-major group order)
# GPU tests (three arrangements), kernel times of the
# bench frame and configs[2], bench A/B against MYYUV_DEC_DEAL=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6r_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6r_tests.log; exit 1; }
tail -1 gpurun_out/r6r_tests.log
: > gpurun_out/r6r_kb.txt
for q in 50 90; do
  for v in 1 0; do
    echo "== q$q sort=$v" >> gpurun_out/r6r_kb.txt
    MYYUV_DEC_DEAL=$v KB_Q=$q timeout -k 10 120 python3 tools/kbench.py 20 >> gpurun_out/r6r_kb.txt 2>&1 || exit 1
    MYYUV_DEC_DEAL=$v KB_Q=$q timeout -k 10 120 python3 tools/kbench.py 20 8192x8192 >> gpurun_out/r6r_kb.txt 2>&1 || exit 1
  done
done
grep -E "==|huff_decode|deal|q[59]0:" gpurun_out/r6r_kb.txt
bash tools/ab_bench.sh default MYYUV_DEC_DEAL=0 > gpurun_out/r6r_ab.txt 2>&1 || exit 1
cat gpurun_out/r6r_ab.txt
