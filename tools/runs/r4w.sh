# round 4: launch shapes with four streams around 4 x 24 (the final build), 20 steps, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4w_shapes.txt
for rnd in 1 2; do
for shape in "4 24" "4 32" "4 28" "4 20"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r4w_shape.json 2>gpurun_out/r4w_shape.err || { tail -5 gpurun_out/r4w_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4w_shape.json')); print('shape $1 x $2', d['value'])" | tee -a gpurun_out/r4w_shapes.txt
done
done
