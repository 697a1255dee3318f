# round 5 final: SQ counters of the bench's launch groups (one --pmc pass per
# counter group, tools/sq_counters.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SQ_BENCH=1 timeout -k 10 900 bash tools/sq_counters.sh r5aj && echo SQ_OK
