# round 3: CAP-16 overflow tier for single-frame launches only (batches keep the
# CAP-64 lane pass): GPU tests, 8192^2 q50/q90 single frames, batch kernels and bench A/B against HEAD (dg2x)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3t_tests.log; exit 1; }
tail -1 gpurun_out/r3t_tests.log
: > gpurun_out/r3t_cfg2.txt
for q in 50 90; do for lib in default build_var/dg2x; do
  if [ $lib = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=$lib/libmyyuv_hip.so; fi
  KB_Q=$q MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 tools/kbench.py 5 8192x8192 >> gpurun_out/r3t_cfg2.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/r3t_cfg2.txt
timeout -k 10 300 python3 tools/k1_ab.py default build_var/dg2x > gpurun_out/r3t_kab.txt 2>&1; cat gpurun_out/r3t_kab.txt
timeout -k 10 900 bash tools/ab_bench.sh default build_var/dg2x && cp gpurun_out/ab_bench.txt gpurun_out/r3t_ab.txt && cat gpurun_out/r3t_ab.txt
