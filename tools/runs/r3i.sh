# bisect: which DPP change breaks tiled 8192^2 q90 (each variant reverts one of them)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in default bisA bisB bisC bisD; do
  if [ $v = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=build_var/$v/libmyyuv_hip.so; fi
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python -u -m pytest tests/test_gpu_known_answers.py -m gpu -q -k "tiled_8192" --timeout 150 --timeout-method thread > gpurun_out/r3i_$v.log 2>&1
  echo "$v: $(tail -1 gpurun_out/r3i_$v.log)"
done
