# round 5: launch shapes with the round-5 kernels (40 steps, no events), two
# rounds: 4 x 24 (default), 4 x 32, 4 x 16, 3 x 32, 4 x 20
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r5h_shapes.txt
for rnd in 1 2; do
for shape in "4 24" "4 32" "4 16" "3 32" "4 20"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r5h_shape.json 2>gpurun_out/r5h_shape.err || { tail -5 gpurun_out/r5h_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5h_shape.json')); print('shape $1 x $2 (40 steps)', d['value'])" | tee -a gpurun_out/r5h_shapes.txt
done
done
