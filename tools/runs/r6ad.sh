# round 6: launch-group sizes 24 / 32 / 40 / 48 with four groups in flight (tools/runs/r6ac.sh's loop)
cd $GRAFT_REPO_ROOT && TAG=r6ad CFGS="24,4 32,4 40,4 48,4" bash tools/runs/r6ac.sh
