#!/bin/bash
# A/B of library builds / environment knobs: value and K1's live roofline
# fraction (events on), two alternating rounds.  Variants as tools/ab_bench.sh.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/ab_roof.txt
: > $OUT
for round in 1 2; do
  for d in "$@"; do
    lib=$R/yuv-manipulations-2_amd/libmyyuv_hip.so; envs=""
    case "$d" in
      default) ;;
      *=*) envs="$d" ;;
      *) lib=$R/$d/libmyyuv_hip.so ;;
    esac
    env $envs MYYUV_HIP_LIB=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 \
      --breakdown-steps 0 --no-side > gpurun_out/ab_one.json 2>gpurun_out/ab_one.err || { cat gpurun_out/ab_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$d', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'])" >> $OUT
  done
done
cat $OUT
