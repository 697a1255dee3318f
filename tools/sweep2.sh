# inflight x batch sweep of the bench configuration (no events, no side lines)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=gpurun_out/sweep2.txt
: > $OUT
CFGS=("${@:-3 4}")
for round in 1 2; do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    steps=$(( 480 / ($1 * $2) ))
    timeout -k 10 120 python3 bench.py --inflight $1 --batch $2 --steps $steps --warmup 2 --cpu-seconds 0 \
      --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/sw_one.json 2>gpurun_out/sw_one.err || { cat gpurun_out/sw_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/sw_one.json')); print('inflight $1 batch $2', d['value'])" >> $OUT
  done
done
cat $OUT
