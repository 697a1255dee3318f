#!/bin/bash
# Throughput cost of the live K1 roofline events: none / launch group 0 / all groups
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for round in 1 2 3; do
  for m in "--no-kernel-events" "--events-ctx0" ""; do
    timeout -k 10 120 python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --breakdown-steps 0 --no-side $m \
      > gpurun_out/ev_one.json 2>gpurun_out/ev_one.err || { cat gpurun_out/ev_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ev_one.json')); r=d['roofline'] or {}; print('${m:-all}', d['value'], r.get('avg_launch_us'), r.get('frac'))"
  done
done
