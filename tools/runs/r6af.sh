# round 6: launch shape 4 x 32 (default) against 4 x 24 in the driver's
# command shape (20 steps, 5 warmup, K1 events on; side lines off), 3 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r6af_ab.txt
: > $OUT
for round in 1 2 3; do
  for b in 32 24; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-side --batch $b > gpurun_out/r6af_one.json 2> gpurun_out/r6af_one.err || { tail -5 gpurun_out/r6af_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r6af_one.json')); print('batch $b', d['value'], d['ms_per_step'])" >> $OUT
  done
done
cat $OUT
