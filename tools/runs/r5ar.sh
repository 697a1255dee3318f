# round 5: k_tile_scan's register footprint in the pipeline (98 VGPRs at
# 62a3ac7, 90 before; its pipeline busy time doubled): ts8 (8 totals kept per
# thread, 82 VGPRs), ts8w (64 VGPRs, 28 spilled) against default; the
# 8192x8192 frame's tile scan for each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r5ar_kbench.txt
for lib in default build_var/ts8 build_var/ts8w; do
  L=$GRAFT_REPO_ROOT/$lib/libmyyuv_hip.so; [ $lib = default ] && L=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so
  echo "== $lib 8192x8192 q50" >> gpurun_out/r5ar_kbench.txt
  MYYUV_HIP_LIB=$L timeout -k 10 120 python3 tools/kbench.py 10 8192x8192 >> gpurun_out/r5ar_kbench.txt 2>&1 || exit 1
done
grep -E "==|scan_tiles" gpurun_out/r5ar_kbench.txt
timeout -k 10 700 bash tools/ab_bench.sh default build_var/ts8 build_var/ts8w > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5ar_ab.txt && cat gpurun_out/r5ar_ab.txt
