#!/bin/bash
# diagnostic: SQ counters for the kernels of the bench workload (few steps)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/k2c
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { timeout -k 10 200 rocprofv3 --pmc "$@" -d $OUT/$1 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-kernel-events > $OUT/$1.json 2> $OUT/$1.err; }
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS || exit 1
run SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_IFETCH SQ_ACTIVE_INST_MISC SQ_INSTS_FLAT || exit 1
