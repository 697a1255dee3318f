# round 5: k_tile_scan with a DPP scan and the plane headers from LDS (no read
# back of the tile prefixes): GPU tests, per-kernel times (24-frame launches
# and the 8192x8192 frame) and the bench A/B against the previous commit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ao_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5ao_tests.log; exit 1; }
tail -1 gpurun_out/r5ao_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5ao_kab.txt 2>&1; cat gpurun_out/r5ao_kab.txt
: > gpurun_out/r5ao_kbench.txt
for rnd in 1 2; do
for lib in build_var/base default; do
  L=$GRAFT_REPO_ROOT/$lib/libmyyuv_hip.so; [ $lib = default ] && L=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so
  echo "== $lib 8192x8192 q50" >> gpurun_out/r5ao_kbench.txt
  MYYUV_HIP_LIB=$L timeout -k 10 120 python3 tools/kbench.py 10 8192x8192 >> gpurun_out/r5ao_kbench.txt 2>&1 || exit 1
done
done
grep -E "==|scan_tiles" gpurun_out/r5ao_kbench.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5ao_ab.txt && cat gpurun_out/r5ao_ab.txt
