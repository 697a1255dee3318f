#!/bin/bash
# Sweep of hardware queues x streams in flight x launch-group size (gpurun):
# two alternating rounds of the bench configuration, no events, no side lines;
# HWQ_CFGS="queues inflight batch;..." overrides the list
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/hwq_sweep.txt
: > $OUT
for round in 1 2; do
  IFS=';' read -ra CFGS <<< "${HWQ_CFGS:-4 3 6;8 3 6;8 4 6;8 4 4;8 6 4;8 6 3;8 8 3}"
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 120 python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 \
      --breakdown-steps 0 --no-side --no-kernel-events --inflight $2 --batch $3 > gpurun_out/hq_one.json 2>gpurun_out/hq_one.err || { cat gpurun_out/hq_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/hq_one.json')); print('hwq=$1 inflight=$2 batch=$3', d['value'])" >> $OUT
  done
done
cat $OUT
