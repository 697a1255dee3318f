# round 3: single-frame overflow tiers in parallel (CAP-16 lane pass on the call's
# stream, the >16-symbol wave pass beside it on an aux stream); batches unchanged
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3v_tests.log; exit 1; }
tail -1 gpurun_out/r3v_tests.log
NRUNS=6 timeout -k 10 300 python -u tools/diag/first_diff.py 90 > gpurun_out/r3v_det.log 2>&1 && grep -v amdgpu.ids gpurun_out/r3v_det.log | head -2
: > gpurun_out/r3v_cfg2.txt
for q in 50 70 90; do for lib in default build_var/dg2x; do
  if [ $lib = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=$lib/libmyyuv_hip.so; fi
  echo "q=$q $lib" >> gpurun_out/r3v_cfg2.txt
  KB_Q=$q MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 tools/kbench.py 5 8192x8192 2>/dev/null >> gpurun_out/r3v_cfg2.txt || exit 1
done; done
cat gpurun_out/r3v_cfg2.txt
