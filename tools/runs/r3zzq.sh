# the CAP-16 tier's gate for single frames: 81,920 (in-tree) against 32,768 / 16,384 listed blocks, on the 8192^2
# frame at q50 (~46k listed) and q90, kernel times per frame (tools/kbench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r3zzq_cfg2.txt
for q in 50 90; do for lib in default build_var/g32k build_var/g16k; do
  if [ $lib = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=$lib/libmyyuv_hip.so; fi
  echo "== q$q $lib" >> gpurun_out/r3zzq_cfg2.txt
  KB_Q=$q MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 tools/kbench.py 5 8192x8192 >> gpurun_out/r3zzq_cfg2.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/r3zzq_cfg2.txt
