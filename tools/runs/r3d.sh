# round 3: SQ instruction counters of the bench's launch groups, this build and the round-2 build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/pcie_copy > gpurun_out/r3d_pcie.txt 2>&1 || { echo PCIE_FAILED; exit 1; }
SQ_BENCH=1 bash tools/sq_counters.sh r3new && SQ_BENCH=1 bash tools/sq_counters.sh r3old build_var/r2
cd $GRAFT_REPO_ROOT
python3 tools/sq_report.py r3new > gpurun_out/r3d_sq_new.txt && python3 tools/sq_report.py r3old > gpurun_out/r3d_sq_old.txt
grep -E "^==|INSTS_VALU |INSTS_SALU |INSTS_LDS |WAVES |ACTIVE_INST_VALU" gpurun_out/r3d_sq_new.txt | paste - - - - - - | head -20
