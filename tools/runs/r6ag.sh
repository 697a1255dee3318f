# round 6: the CAP-16 tier's occupancy with the LDS heap: 4 / 6 waves per SIMD
# against 5 (default): bench A/B + one 32-frame launch group alone
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_bench.sh default build_var/r16w4 build_var/r16w6 > gpurun_out/r6ag_ab.txt 2>&1 || exit 1
cat gpurun_out/r6ag_ab.txt
K1AB_B=32 timeout -k 10 300 python3 tools/k1_ab.py default build_var/r16w4 build_var/r16w6 > gpurun_out/r6ag_alone.txt 2>&1 || exit 1
grep -o "^[^ ]* .*huff_encode_r16=[0-9.]*" gpurun_out/r6ag_alone.txt
