# round 5: K1's nonzero count by v_bcnt of the flags instead of packed adds:
# GPU tests, per-kernel times and the bench A/B against the previous commit
# (build_var/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bd_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5bd_tests.log; exit 1; }
tail -1 gpurun_out/r5bd_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5bd_kab.txt 2>&1; cat gpurun_out/r5bd_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5bd_ab.txt && cat gpurun_out/r5bd_ab.txt
