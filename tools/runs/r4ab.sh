# round 4 first GPU call: baseline check at HEAD (r4a), then calibration, SQ counters, trace (r4b)
bash $GRAFT_REPO_ROOT/tools/runs/r4a.sh && bash $GRAFT_REPO_ROOT/tools/runs/r4b.sh
