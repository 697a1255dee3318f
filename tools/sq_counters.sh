#!/bin/bash
# diagnostic: SQ counters for every kernel of the bench workload (few steps),
# one rocprofv3 --pmc pass per group.  Usage: tools/sq_counters.sh <tag>
# Output: gpurun_out/sq_<tag>/<group>/run_counter_collection.csv
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { local g=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" -d $OUT/$g -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-kernel-events > $OUT/$g.json 2> $OUT/$g.err; }
run g1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1
run g2 SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_MISC || exit 1
echo done > $OUT/DONE
