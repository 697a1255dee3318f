set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile.sh r05a 20 && echo PROFILE_OK
bash tools/cfg2_profile.sh r05cfg2 10 && echo CFG2_OK
