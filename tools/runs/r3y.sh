# K2 window sort (kWinTiles 4 in-tree; 1 / 2 / 8 variants; base = HEAD d156368), second build:
# coefficient loads inside the class branches (no spills in the run loop), classify loads double-buffered
# GPU tests on the in-tree build, per-kernel times, then the bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3y_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3y_tests.log; exit 1; }
tail -1 gpurun_out/r3y_tests.log
timeout -k 10 400 python3 tools/k1_ab.py build_var/base default build_var/win1 build_var/win2 build_var/win8 > gpurun_out/r3y_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3y_kernels.txt; exit 1; }
cat gpurun_out/r3y_kernels.txt
timeout -k 10 500 bash tools/ab_bench.sh build_var/base default build_var/win2 > gpurun_out/r3y_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3y_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3y_ab.txt
cat gpurun_out/r3y_ab.txt
