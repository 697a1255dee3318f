# round 3: DPP for K1's row-mask quad exchange and the wave scans / max of K2, K4, tile scan
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3h_tests.log; exit 1; }
tail -2 gpurun_out/r3h_tests.log
timeout -k 10 300 python3 tools/k1_ab.py default build_var/r2 > gpurun_out/r3h_kab.txt 2>&1; cat gpurun_out/r3h_kab.txt
timeout -k 10 900 bash tools/ab_bench.sh default build_var/r2 && cp gpurun_out/ab_bench.txt gpurun_out/r3h_ab.txt
