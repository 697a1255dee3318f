# K2 window sort + message-length sub-buckets (in-tree: 4 tiles, split 8/16); nosplit = class keys only; win2s = 2 tiles with the split
# GPU tests on the in-tree build, per-kernel times, then the bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3za_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3za_tests.log; exit 1; }
tail -1 gpurun_out/r3za_tests.log
timeout -k 10 400 python3 tools/k1_ab.py build_var/base default build_var/nosplit build_var/win2s > gpurun_out/r3za_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3za_kernels.txt; exit 1; }
cat gpurun_out/r3za_kernels.txt
timeout -k 10 500 bash tools/ab_bench.sh build_var/base default build_var/nosplit > gpurun_out/r3za_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3za_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3za_ab.txt
cat gpurun_out/r3za_ab.txt
