# round 5: K2 windows of 8 tiles (win8: 32 runs per workgroup, the window
# prologue spread over twice the runs) against 4 (default): per-kernel times
# and the bench A/B; GPU tests of win8
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/win8 > gpurun_out/r5ay_kab.txt 2>&1; cat gpurun_out/r5ay_kab.txt
timeout -k 10 700 bash tools/ab_bench.sh default build_var/win8 > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5ay_ab.txt && cat gpurun_out/r5ay_ab.txt
