#!/bin/bash
# diagnostic: instruction-cache counters per kernel for alternative builds
#   tools/icache.sh <tag> <lib-dir>...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/ic_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for d in "$@"; do
  n=$(basename $d)
  MYYUV_HIP_LIB=$R/$d/libmyyuv_hip.so timeout -k 10 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQC_TC_INST_REQ SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $OUT/$n -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-kernel-events > $OUT/$n.json 2> $OUT/$n.err || exit 1
done
