# round 5: r5ae's bench A/B repeated (decoder transform without fences)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5ae2_ab.txt && cat gpurun_out/r5ae2_ab.txt
