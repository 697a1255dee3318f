# CAP-16 register tier for overflow lists longer than one resident round of the CAP-64 lane pass
# (k_huff_encode_r16 gated on the device by the list length): GPU tests, 8192^2 q50/q90 single frames,
# batch kernels and bench A/B against HEAD (prev), tier for single frames only, K1 untouched
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zy_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zy_tests.log; exit 1; }
tail -1 gpurun_out/r3zy_tests.log
: > gpurun_out/r3zy_cfg2.txt
for q in 50 90; do for lib in default build_var/prev; do
  if [ $lib = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=$lib/libmyyuv_hip.so; fi
  echo "== q$q $lib" >> gpurun_out/r3zy_cfg2.txt
  KB_Q=$q MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 tools/kbench.py 5 8192x8192 >> gpurun_out/r3zy_cfg2.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/r3zy_cfg2.txt
timeout -k 10 300 python3 tools/k1_ab.py build_var/prev default > gpurun_out/r3zy_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zy_kernels.txt; exit 1; }
cat gpurun_out/r3zy_kernels.txt
timeout -k 10 500 bash tools/ab_bench.sh build_var/prev default > gpurun_out/r3zy_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zy_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zy_ab.txt
cat gpurun_out/r3zy_ab.txt
