#!/bin/bash
# BASELINE configs[2]: rocprofv3 HBM traffic and per-kernel time on the
# 8192x8192 tiled frame (SURVEY.md §8d generator) at q50 and q90, one
# compress_device + decompress_device per step (tools/kbench.py).
# Passes per quality: kernel trace + stats, --pmc FETCH_SIZE, --pmc WRITE_SIZE,
# laid out as tools/traffic.py expects: gpurun_out/prof_<tag>_q<Q>/{trace,fetch,write}.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02cfg2}
STEPS=${2:-10}
cd /tmp && export TMPDIR=/tmp
for Q in 50 90; do
  OUT=$R/gpurun_out/prof_${TAG}_q$Q
  mkdir -p $OUT
  export KB_Q=$Q
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $R/tools/kbench.py $STEPS 8192x8192 > $OUT/kbench_trace.txt 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
    python3 $R/tools/kbench.py $STEPS 8192x8192 > $OUT/kbench_fetch.txt 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
    python3 $R/tools/kbench.py $STEPS 8192x8192 > $OUT/kbench_write.txt 2>&1
  cat $OUT/kbench_trace.txt
done
echo done
