# round 6: K2 / overflow-tier coefficient loads through a buffer descriptor
# (MYYUV_K2_BUF) against flat loads with zero-buffer selects; GPU tests
# (incl. the batch split into launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6i_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6i_tests.log; exit 1; }
tail -1 gpurun_out/r6i_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/k2flat > gpurun_out/r6i_kab.txt 2>&1; cat gpurun_out/r6i_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/k2flat > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r6i_ab.txt && cat gpurun_out/r6i_ab.txt
for Q in 50 90; do KB_Q=$Q timeout -k 10 200 python3 -u tools/kbench.py 10 8192x8192 > gpurun_out/r6i_cfg2_q$Q.txt 2>&1 && echo "== 8192^2 q$Q" && grep -v amdgpu.ids gpurun_out/r6i_cfg2_q$Q.txt; done
