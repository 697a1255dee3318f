# round 5: K2 windows of 8 tiles for launches of >= 16384 tiles (the bench's
# 24-frame groups), 4 below (single frames); K4 reads the launch's window:
# GPU tests, per-kernel times, six alternating bench rounds against the
# previous commit (build_var/base), the 8192x8192 frame and batch4k
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bb_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5bb_tests.log; exit 1; }
tail -1 gpurun_out/r5bb_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5bb_kab.txt 2>&1; cat gpurun_out/r5bb_kab.txt
timeout -k 10 700 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5bb_ab.txt && cat gpurun_out/r5bb_ab.txt
timeout -k 10 700 bash tools/ab_bench.sh build_var/base default > /dev/null && cat gpurun_out/ab_bench.txt >> gpurun_out/r5bb_ab.txt && cat gpurun_out/ab_bench.txt
: > gpurun_out/r5bb_kbench.txt
for lib in default build_var/base; do
  L=$GRAFT_REPO_ROOT/$lib/libmyyuv_hip.so; [ $lib = default ] && L=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so
  echo "== $lib 8192x8192 q50" >> gpurun_out/r5bb_kbench.txt
  MYYUV_HIP_LIB=$L timeout -k 10 120 python3 tools/kbench.py 10 8192x8192 >> gpurun_out/r5bb_kbench.txt 2>&1 || exit 1
done
grep -E "==|huff_encode |compress wall" gpurun_out/r5bb_kbench.txt
