#!/bin/bash
# diagnostic: SQ counters for every kernel of the codec round trip (few steps),
# one rocprofv3 --pmc pass per group.  Usage: tools/sq_counters.sh <tag> [lib-dir]
# (lib-dir: an alternative build; runs tools/kbench.py, no correctness checks)
# Output: gpurun_out/sq_<tag>/<group>/run_counter_collection.csv
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}
LIB=${2:+$R/$2/libmyyuv_hip.so}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export MYYUV_HIP_LIB=$LIB
# SQ_BENCH=1: the bench's batched launch groups (bench.py, 2 steps) instead of kbench's single frames
if [ -n "$SQ_BENCH" ]; then
  run() { local g=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" -d $OUT/$g -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > $OUT/$g.txt 2> $OUT/$g.err; }
else
  run() { local g=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" -d $OUT/$g -o run --output-format csv -- python3 $R/tools/kbench.py 5 > $OUT/$g.txt 2> $OUT/$g.err; }
fi
run g1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1
run g2 SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_LDS || exit 1
run g3 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_FLAT SQ_IFETCH SQ_INSTS_MFMA || exit 1
echo done > $OUT/DONE
