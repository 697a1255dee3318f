# round 6: K1's per-block fix lists: GPU tests, then kernel times on the
# 8192x8192 tiled frame at q50 / q90 and on the bench frame at q90 (kbench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6e_tests.log; exit 1; }
tail -1 gpurun_out/r6e_tests.log
for Q in 50 90; do
  KB_Q=$Q timeout -k 10 200 python3 -u tools/kbench.py 10 8192x8192 > gpurun_out/r6e_cfg2_q$Q.txt 2>&1 || { echo KB_FAILED; tail gpurun_out/r6e_cfg2_q$Q.txt; exit 1; }
  echo "== 8192^2 q$Q"; cat gpurun_out/r6e_cfg2_q$Q.txt
done
KB_Q=90 timeout -k 10 200 python3 -u tools/kbench.py 10 > gpurun_out/r6e_big_q90.txt 2>&1 && echo "== big q90" && cat gpurun_out/r6e_big_q90.txt
