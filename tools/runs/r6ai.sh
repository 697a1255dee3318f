# round 6: loop-exit granularity: the decoder's positions per "any lane left"
# test (MYYUV_K5_GROUP 1 / 2 default / 4) and the encoders' positions per
# wave-uniform step (MYYUV_POS_GROUP 2 / 4 default / 8): bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_bench.sh default build_var/k5g1 build_var/k5g4 build_var/pg2 build_var/pg8 > gpurun_out/r6ai_ab.txt 2>&1 || exit 1
cat gpurun_out/r6ai_ab.txt
