#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun):
#   1. kernel trace + stats (per-kernel durations)
#   2. --pmc FETCH_SIZE      (own pass: TCC slots)
#   3. --pmc WRITE_SIZE      (own pass)
# (--no-side: the bench workload's launches only, so the trace's per-kernel
# averages and the per-launch bytes are those of the timed region's launch
# groups; the side measurements launch other frame sizes)
# Output under $GRAFT_REPO_ROOT/gpurun_out/prof_<tag>/.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
STEPS=${2:-20}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps $STEPS --warmup 3 --cpu-seconds 0 --breakdown-steps 0 --no-side > $OUT/bench_trace.json 2> $OUT/bench_trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
  python3 $R/bench.py --steps $STEPS --warmup 3 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
  python3 $R/bench.py --steps $STEPS --warmup 3 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > $OUT/bench_write.json 2> $OUT/bench_write.err
echo done > $OUT/DONE
