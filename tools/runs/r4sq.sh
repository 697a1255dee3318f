# round 4: SQ counters of the final build's bench launch groups (tools/sq_counters.sh, one --pmc pass per group)
set -o pipefail
cd $GRAFT_REPO_ROOT
SQ_BENCH=1 bash tools/sq_counters.sh r4fin && echo SQ_OK
