# round 6: hardware queues per process (GPU_MAX_HW_QUEUES 4, the box default,
# or 8) with 4 / 6 / 8 launch groups in flight: bench, three rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r6ak_sweep.txt
: > $OUT
for round in 1 2 3; do
  for cfg in "4 32 4" "8 32 4" "8 32 6" "8 24 8"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 150 python3 bench.py --steps 30 --warmup 4 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events --batch $2 --inflight $3 > gpurun_out/r6ak_one.json 2> gpurun_out/r6ak_one.err || { tail -5 gpurun_out/r6ak_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r6ak_one.json')); print('hwq $1 batch $2 inflight $3', d['value'])" >> $OUT
  done
done
cat $OUT
