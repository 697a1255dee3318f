# round 5: K2 at 6 waves per SIMD (k2w6: 80 VGPRs, 9 spilled) and the
# decoder's tail unit with 1 / 3 unconditional steps (al1 / al3; shipped: 2):
# per-kernel times and the bench A/B of k2w6 against HEAD (build_var/base = default)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py build_var/k2w6 build_var/al1 build_var/al3 build_var/base > gpurun_out/r5ap_kab.txt 2>&1; cat gpurun_out/r5ap_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh build_var/k2w6 build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5ap_ab.txt && cat gpurun_out/r5ap_ab.txt
