# round 6: K1's stores as buffer stores with out-of-range drops (MYYUV_K1_BUF)
# against flat stores with sink pointers: GPU tests of the in-tree build, then
# kernel times and bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6h_tests.log; exit 1; }
tail -1 gpurun_out/r6h_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/k1flat > gpurun_out/r6h_kab.txt 2>&1; cat gpurun_out/r6h_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/k1flat > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r6h_ab.txt && cat gpurun_out/r6h_ab.txt
