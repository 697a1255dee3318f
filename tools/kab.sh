#!/bin/bash
# diagnostic: tools/kbench.py over alternative builds: tools/kab.sh <tag> <lib-dir>...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/kab_$TAG.txt
: > $OUT
for d in "$@"; do
  MYYUV_HIP_LIB=$R/$d/libmyyuv_hip.so timeout -k 10 120 python3 $R/tools/kbench.py 20 $KB_SIZE >> $OUT 2>&1 || exit 1
done
