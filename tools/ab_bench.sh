#!/bin/bash
# A/B of library builds in the bench configuration: tools/ab_bench.sh <dir>... (gpurun)
# ("default" = the in-tree build); three alternating rounds, no events, no side lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/ab_bench.txt
: > $OUT
for round in 1 2 3; do
  for d in "$@"; do
    if [ "$d" = default ]; then lib=$R/yuv-manipulations-2_amd/libmyyuv_hip.so; else lib=$R/$d/libmyyuv_hip.so; fi
    MYYUV_HIP_LIB=$lib timeout -k 10 120 python3 bench.py --steps 480 --warmup 48 --cpu-seconds 0 \
      --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/ab_one.json 2>gpurun_out/ab_one.err || { cat gpurun_out/ab_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$d', d['value'])" >> $OUT
  done
done
cat $OUT
