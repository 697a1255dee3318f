# round 3: streamlined decoder symbol loop — full GPU tests + bench A/B against the round-start build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
timeout -k 10 900 bash tools/ab_bench.sh default build_var/r3base && cp gpurun_out/ab_bench.txt gpurun_out/r3q_ab.txt && cat gpurun_out/r3q_ab.txt
