# launch shape sweep with the CAP-16 overflow tier for batches (lists past one CAP-64 round)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r3zzg_shape.txt
: > $OUT
for round in 1 2; do
  for shape in "3 24" "3 32" "4 24" "3 40" "4 32" "3 48"; do
    set -- $shape
    for steps in 20 40; do
      timeout -k 10 120 python3 bench.py --steps $steps --warmup 4 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events \
        --inflight $1 --batch $2 > gpurun_out/shape_one.json 2> gpurun_out/shape_one.err || { cat gpurun_out/shape_one.err | tail -5; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/shape_one.json')); print('$1 x $2 steps $steps', d['value'], d['config'].get('frames_per_step', ''))" >> $OUT
    done
  done
done
cat $OUT
