# round 6: launch-group size and groups in flight for the bench workload
# after this round's kernel changes (24 x 4 is the default): three rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r6ac}_sweep.txt
CFGS=${CFGS:-"24,4 16,4 32,4 24,3 32,3"}
: > $OUT
for round in 1 2 3; do
  for cfg in $CFGS; do
    set -- ${cfg/,/ }
    timeout -k 10 150 python3 bench.py --steps 30 --warmup 4 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events --batch $1 --inflight $2 > gpurun_out/r6ac_one.json 2> gpurun_out/r6ac_one.err || { tail -5 gpurun_out/r6ac_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r6ac_one.json')); print('batch $1 inflight $2', d['value'])" >> $OUT
  done
done
cat $OUT
