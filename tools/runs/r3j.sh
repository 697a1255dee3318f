# where the DPP build's repeated 8192^2 q90 split compressions differ from the oracle
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in default; do
  if [ $v = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=build_var/$v/libmyyuv_hip.so; fi
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 240 python -u tools/diag/first_diff.py 90 > gpurun_out/r3k_$v.log 2>&1 || exit 1
  echo "== $v"; cat gpurun_out/r3k_$v.log
done
