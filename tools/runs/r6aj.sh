# round 6: each kernel's marginal cost in the bench shape (4 x 32, chef-big
# q50): throughput with that kernel's launches skipped (tools/kskip.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KSKIP_NF=4 KSKIP_B=32 timeout -k 10 600 python3 tools/kskip.py > gpurun_out/r6aj_kskip.txt 2>&1 || { tail -20 gpurun_out/r6aj_kskip.txt; exit 1; }
cat gpurun_out/r6aj_kskip.txt
