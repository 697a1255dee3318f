# round 5: the bench A/B of r5av again (one of its rounds read 295.6k)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5av2_ab.txt && cat gpurun_out/r5av2_ab.txt
timeout -k 10 500 bash tools/ab_bench.sh build_var/base default > /dev/null && cat gpurun_out/ab_bench.txt >> gpurun_out/r5av2_ab.txt && cat gpurun_out/ab_bench.txt
