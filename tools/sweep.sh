#!/bin/bash
# bench.py over (inflight, batch) pairs: tools/sweep.sh "3:4 3:6 ..." (gpurun)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
: > gpurun_out/sweep.txt
for p in $1; do
  i=${p%%:*}; b=${p##*:}
  timeout -k 10 120 python3 bench.py --inflight $i --batch $b --steps 480 --warmup 48 --cpu-seconds 0 \
    --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/sweep_one.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_one.json')); print('$i x $b', d['value'])" >> gpurun_out/sweep.txt
done
cat gpurun_out/sweep.txt
