# round 6: K2's window for long launches (8 tiles, default) against 4
# after the ovf class and length buckets: bench A/B + one launch group alone
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_bench.sh default build_var/win4 > gpurun_out/r6ab_ab.txt 2>&1 || exit 1
cat gpurun_out/r6ab_ab.txt
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/win4 > gpurun_out/r6ab_alone.txt 2>&1 || exit 1
grep -o "^[^ ]* .*huff_encode=[0-9.]*" gpurun_out/r6ab_alone.txt
