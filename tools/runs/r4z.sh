# round 4: the driver's own command shape (20 steps, warmup 5, K1 + fix
# stamped in the timed region), the final build against 864e0a1 (b864),
# three alternating rounds: does the driver-shape figure follow the A/B?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4z_driver_shape.txt
for rnd in 1 2 3; do
  for d in default build_var/b864; do
    lib=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so; [ "$d" != default ] && lib=$GRAFT_REPO_ROOT/$d/libmyyuv_hip.so
    MYYUV_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-side > gpurun_out/r4z_one.json 2> gpurun_out/r4z_one.err || { tail -5 gpurun_out/r4z_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r4z_one.json')); print('$d', d['value'], d['roofline']['avg_launch_us'])" | tee -a gpurun_out/r4z_driver_shape.txt
  done
done
