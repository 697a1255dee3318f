# round 4: the fused decoder's non-constant blocks written to HBM and listed
# (32 lists) for k_idct_list, K6's body at K6's occupancy (70 VGPRs) instead
# of the decoding wave's (96): aclist (decoder at 5 waves), aclist7 (7 waves,
# spills); parity tests of the aclist build, per-kernel times, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/aclist/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t_aclist_tests.log 2>&1; echo "aclist tests rc=$?"; tail -3 gpurun_out/r4t_aclist_tests.log
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/nobatch build_var/aclist build_var/aclist7 > gpurun_out/r4t_kab.txt 2>&1; cat gpurun_out/r4t_kab.txt
timeout -k 10 600 bash tools/ab_bench.sh default build_var/aclist build_var/aclist7 > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4t_ab.txt && cat gpurun_out/r4t_ab.txt
