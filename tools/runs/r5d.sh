# round 5: k_tile_scan with its tile totals loaded 8 at a time (one round
# trip per tile before); the CAP-16 overflow tier for single-frame lists over
# 4,096 blocks (build_var/gate4k, -DMYYUV_R16_GATE=4096; default 81,920):
# GPU tests, single-frame kernel times at 8192x8192 q50/q90 and 4032x3008,
# the bench A/B against the previous commit (build_var/r5c)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5d_tests.log; exit 1; }
tail -1 gpurun_out/r5d_tests.log
: > gpurun_out/r5d_kbench.txt
for lib in build_var/r5c default build_var/gate4k; do
  L=$GRAFT_REPO_ROOT/$lib/libmyyuv_hip.so; [ $lib = default ] && L=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so
  for Q in 50 90; do
    echo "== $lib 8192x8192 q$Q" >> gpurun_out/r5d_kbench.txt
    KB_Q=$Q MYYUV_HIP_LIB=$L timeout -k 10 120 python3 tools/kbench.py 10 8192x8192 >> gpurun_out/r5d_kbench.txt 2>&1 || exit 1
  done
  echo "== $lib 4032x3008 q50" >> gpurun_out/r5d_kbench.txt
  MYYUV_HIP_LIB=$L timeout -k 10 120 python3 tools/kbench.py 10 >> gpurun_out/r5d_kbench.txt 2>&1 || exit 1
done
cat gpurun_out/r5d_kbench.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/r5c > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5d_ab.txt && cat gpurun_out/r5d_ab.txt
