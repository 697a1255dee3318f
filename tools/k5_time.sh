#!/bin/bash
# diagnostic: K5 variants, correctness (tools/k5_diff.py, 3 decodes) + timing (kbench)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/k5t_$TAG.txt
: > $OUT
for d in "$@"; do
  echo "== $d" >> $OUT
  MYYUV_HIP_LIB=$R/$d/libmyyuv_hip.so timeout -k 10 120 python3 $R/tools/k5_diff.py 2>&1 | grep iter >> $OUT || true
  MYYUV_HIP_LIB=$R/$d/libmyyuv_hip.so timeout -k 10 120 python3 $R/tools/kbench.py 20 2>&1 | grep -E "rc=|huff_decode|dequant" >> $OUT || exit 1
done
