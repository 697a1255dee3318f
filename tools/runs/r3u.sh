# round 3: single-frame 8192^2 overflow passes across qualities, CAP-16 tier build vs HEAD (dg2x)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r3u_cfg2.txt
for q in 60 70 75 80 85; do for lib in default build_var/dg2x; do
  if [ $lib = default ]; then L=yuv-manipulations-2_amd/libmyyuv_hip.so; else L=$lib/libmyyuv_hip.so; fi
  echo "q=$q $lib" >> gpurun_out/r3u_cfg2.txt
  KB_Q=$q MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 tools/kbench.py 5 8192x8192 2>/dev/null | grep -E "huff_encode_(wide|r16|wave)" >> gpurun_out/r3u_cfg2.txt || exit 1
done; done
cat gpurun_out/r3u_cfg2.txt
