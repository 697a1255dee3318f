# round 5: K1's butterfly fast path (fdct_bfly.h) and K4 in XCD-aware tile
# order: GPU tests, K1 alone
# against round 4's FMA-chain K1 (build_var/r4base), the bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5b_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5b_tests.log; exit 1; }
tail -1 gpurun_out/r5b_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/r4base > gpurun_out/r5b_kab.txt 2>&1; cat gpurun_out/r5b_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/r4base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5b_ab.txt && cat gpurun_out/r5b_ab.txt
# (K4 in XCD-aware tile order in the same build) calibrated traffic of the bench workload
timeout -k 10 1000 bash tools/profile.sh r5b 10 && echo profiled
