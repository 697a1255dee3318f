# round 4: launch shapes after the K1 fast path (r4i: 4 x 24 +2 % over 3 x 24
# at 20 steps): 20- and 40-step runs, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4j_shapes.txt
for rnd in 1 2; do
for shape in "3 24 20" "4 24 20" "4 20 20" "5 16 20" "5 24 20" "3 24 40" "4 24 40" "5 16 40"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps $3 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r4j_shape.json 2>gpurun_out/r4j_shape.err || { tail -5 gpurun_out/r4j_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4j_shape.json')); print('shape $1 x $2 steps $3', d['value'])" | tee -a gpurun_out/r4j_shapes.txt
done
done
