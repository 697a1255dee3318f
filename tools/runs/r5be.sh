# round 5: launch shapes again with K2's 8-tile windows (20 steps, the driver's
# shape), three alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r5be_shapes20.txt
for rnd in 1 2 3; do
for shape in "4 24" "4 32" "3 32" "4 20"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r5be_shape.json 2>gpurun_out/r5be_shape.err || { tail -5 gpurun_out/r5be_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5be_shape.json')); print('shape $1 x $2 (20 steps)', d['value'])" | tee -a gpurun_out/r5be_shapes20.txt
done
done
