# round-3 final profiles: kernel trace + calibrated HBM traffic of the bench workload, and BASELINE configs[2]
# (8192^2 tiled, q50 / q90, one frame per launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/profile.sh r3zz 20 && echo PROFILE_OK && bash tools/cfg2_profile.sh r3cfg2 10 && echo CFG2_OK
