set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/ab_bench.sh build_var/s8w4 build_var/s4ni build_var/s8ni build_var/s8niw4
