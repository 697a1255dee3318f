# round 5: K4 (k_stream_out) in fewer dependent round trips: kernel arguments
# consumed at once, plane fields by static index, the first loads unconditional
# and waited once (chunk words predicated again), surplus workgroups return after them, DPP scan and next-lane
# move: GPU tests, kernel times and bench A/B against HEAD (build_var/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5q_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5q_tests.log; exit 1; }
tail -1 gpurun_out/r5q_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5q_kab.txt 2>&1; cat gpurun_out/r5q_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5q_ab.txt && cat gpurun_out/r5q_ab.txt
