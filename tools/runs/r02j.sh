set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_r02j
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 3 --cpu-seconds 0 --breakdown-steps 0 --no-side > $OUT/bench_trace.json 2> $OUT/bench_trace.err && echo TRACE_OK
