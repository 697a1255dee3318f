# round 4: K1's unproven-unit list batched per wave (default) against one
# atomic per unit (nobatch) and the previous commit (prevlist, 864e0a1);
# K2 compiled for 6 workgroups per CU (k2w6); the decoder with its
# non-constant blocks' transform replaced by a copy (dexp4: the transform's
# share, stores kept)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/nobatch build_var/k2w6 build_var/dexp4 > gpurun_out/r4r_kab.txt 2>&1; cat gpurun_out/r4r_kab.txt
timeout -k 10 800 bash tools/ab_bench.sh default build_var/nobatch build_var/prevlist build_var/k2w6 > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4r_ab.txt && cat gpurun_out/r4r_ab.txt
