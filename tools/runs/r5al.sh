# round 5: K4 with two tiles per workgroup, each round trip's loads of both
# in flight together (default: 16 source words per chunk, 68 VGPRs; k4vw12:
# 12 words, 60 VGPRs; k4t1: the restructured kernel at one tile): GPU tests,
# per-kernel times and the bench A/B against the previous commit (build_var/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5al_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5al_tests.log; exit 1; }
tail -1 gpurun_out/r5al_tests.log
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/k4vw12 build_var/k4t1 build_var/base > gpurun_out/r5al_kab.txt 2>&1; cat gpurun_out/r5al_kab.txt
timeout -k 10 700 bash tools/ab_bench.sh default build_var/k4vw12 build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5al_ab.txt && cat gpurun_out/r5al_ab.txt
