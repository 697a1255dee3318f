set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/ab_bench.sh build_var/base build_var/w16g1280 build_var/w16g1280_64g256
