#!/bin/bash
# A/B the bench across alternative builds of libmyyuv_hip.so:
#   tools/ab.sh <tag> <lib-dir>...   (each dir holds a libmyyuv_hip.so)
# writes gpurun_out/ab_<tag>/<name>.{json,err}; event timing per kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
for d in "$@"; do
  n=$(basename $d)
  MYYUV_HIP_LIB=$d/libmyyuv_hip.so timeout -k 10 120 python3 $R/bench.py --steps 30 --warmup 5 --cpu-seconds 0 > $OUT/$n.json 2> $OUT/$n.err || exit 1
done
