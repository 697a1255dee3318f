# round 5: K2 windows of 8 tiles (win8) on the other configs: the 8192x8192
# frame (q50, q90; kbench) and the batch4k side line (configs[3])
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r5ba_kbench.txt
for lib in default build_var/win8; do
  L=$GRAFT_REPO_ROOT/$lib/libmyyuv_hip.so; [ $lib = default ] && L=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so
  for q in 50 90; do
    echo "== $lib 8192x8192 q$q" >> gpurun_out/r5ba_kbench.txt
    KB_Q=$q MYYUV_HIP_LIB=$L timeout -k 10 120 python3 tools/kbench.py 10 8192x8192 >> gpurun_out/r5ba_kbench.txt 2>&1 || exit 1
  done
  MYYUV_HIP_LIB=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --breakdown-steps 0 --no-kernel-events > gpurun_out/r5ba_side.json 2> gpurun_out/r5ba_side.err || { tail -5 gpurun_out/r5ba_side.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5ba_side.json')); print('$lib batch4k', d['side']['batch4k']['value'])" | tee -a gpurun_out/r5ba_kbench.txt
done
grep -E "==|huff_encode |compress wall|batch4k" gpurun_out/r5ba_kbench.txt
