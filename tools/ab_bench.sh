#!/bin/bash
# A/B of library builds or environment knobs in the bench configuration (gpurun):
#   tools/ab_bench.sh <variant>...
# a variant is "default" (the in-tree build), a directory holding a
# libmyyuv_hip.so, or VAR=value (the in-tree build with that environment);
# three alternating rounds, no events, no side lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/ab_bench.txt
: > $OUT
for round in 1 2 3; do
  for d in "$@"; do
    lib=$R/yuv-manipulations-2_amd/libmyyuv_hip.so; envs=""
    case "$d" in
      default) ;;
      *=*) envs="$d" ;;
      *) lib=$R/$d/libmyyuv_hip.so ;;
    esac
    env $envs MYYUV_HIP_LIB=$lib timeout -k 10 120 python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 \
      --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/ab_one.json 2>gpurun_out/ab_one.err || { cat gpurun_out/ab_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$d', d['value'])" >> $OUT
  done
done
cat $OUT
