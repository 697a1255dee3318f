# K2 workgroups per CU (MYYUV_K2_WAVES 4 / 5 (base) / 6) at 3 x 7 launch groups
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/ab_bench.sh build_var/base build_var/w4 build_var/w6 && cp gpurun_out/ab_bench.txt gpurun_out/r05i_ab.txt
