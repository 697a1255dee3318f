# round 3: CAP-16 register tier for the overflow blocks (k_huff_encode_r16), then wave / CAP-64 passes for the rest
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3g_tests.log; exit 1; }
tail -2 gpurun_out/r3g_tests.log
timeout -k 10 300 python3 tools/k1_ab.py default build_var/r2 > gpurun_out/r3g_kab.txt 2>&1; cat gpurun_out/r3g_kab.txt
for q in 50 90; do for lib in default build_var/r2; do
  if [ $lib = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=$lib/libmyyuv_hip.so; fi
  KB_Q=$q MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 tools/kbench.py 5 8192x8192 >> gpurun_out/r3g_cfg2.txt 2>&1 || exit 1
done; done
cat gpurun_out/r3g_cfg2.txt
timeout -k 10 900 bash tools/ab_bench.sh default build_var/r2 && cp gpurun_out/ab_bench.txt gpurun_out/r3g_ab.txt
