# round 4: K1's 32 spread lists (default) against every unit in list 0 (nosp,
# the same source) and the round's single-counter build (nobatch): K1 per
# launch and the bench, three alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/nosp build_var/nobatch > gpurun_out/r4u_kab.txt 2>&1; cat gpurun_out/r4u_kab.txt
timeout -k 10 600 bash tools/ab_bench.sh default build_var/nosp build_var/nobatch > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4u_ab.txt && cat gpurun_out/r4u_ab.txt
