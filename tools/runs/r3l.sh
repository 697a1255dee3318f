# repeated 8192^2 q90 split compressions against the oracle: the DPP build,
# the build with every DPP change reverted, and the two single reverts that passed once
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in allbis default bisB bisD; do
  if [ $v = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=build_var/$v/libmyyuv_hip.so; fi
  NRUNS=8 MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 240 python -u tools/diag/first_diff.py 90 > gpurun_out/r3l_$v.log 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r3l_$v.log | head -4
done
