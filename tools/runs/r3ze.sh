# launch-group shape sweep (--inflight x --batch) around 4 x 7, default run
# (40 steps) and the driver's command shape (20 steps, 5 warmup)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r3ze_shape.txt
for round in 1 2; do
  for shape in "4 7" "4 8" "4 9" "4 10" "5 6" "5 7" "6 5" "6 6" "8 4"; do
    set -- $shape
    timeout -k 10 120 python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events --inflight $1 --batch $2 > gpurun_out/r3ze_one.json 2> gpurun_out/r3ze_one.err || { tail -5 gpurun_out/r3ze_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r3ze_one.json')); print('inflight $1 batch $2 steps 40', d['value'])" >> gpurun_out/r3ze_shape.txt
  done
  for shape in "3 7" "4 7" "4 8" "5 6"; do
    set -- $shape
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --breakdown-steps 0 --no-side --inflight $1 --batch $2 > gpurun_out/r3ze_one.json 2> gpurun_out/r3ze_one.err || { tail -5 gpurun_out/r3ze_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r3ze_one.json')); print('inflight $1 batch $2 steps 20 (driver shape)', d['value'])" >> gpurun_out/r3ze_shape.txt
  done
done
cat gpurun_out/r3ze_shape.txt
