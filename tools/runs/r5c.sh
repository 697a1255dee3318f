# round 5: variant cleanup (no product change), the SLP vectorizer off at the
# -fgpu-rdc link step: GPU tests (with the fix-grid walk case), per-kernel
# times, bench A/B against the same objects linked with SLP on, SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5c_tests.log; exit 1; }
tail -1 gpurun_out/r5c_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/slpon > gpurun_out/r5c_kab.txt 2>&1; cat gpurun_out/r5c_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/slpon > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5c_ab.txt && cat gpurun_out/r5c_ab.txt
SQ_BENCH=1 timeout -k 10 900 bash tools/sq_counters.sh r5c && echo SQ_OK
