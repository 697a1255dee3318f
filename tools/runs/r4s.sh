# round 4: K1's unproven units in 32 lists (unit ua in list ua % 32: the
# appends spread over 32 counters, no state carried through K1's loop):
# every GPU test (with the new K1-grid test of the lists), smoke, the bench
# against one counter (nobatch) and the previous commit (prevlist), and
# configs[2] at q90 (kernel trace only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4s_tests.log; exit 1; }
tail -1 gpurun_out/r4s_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4s_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r4s_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 bash tools/ab_bench.sh default build_var/nobatch build_var/prevlist > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4s_ab.txt && cat gpurun_out/r4s_ab.txt
cd /tmp && export TMPDIR=/tmp
for Q in 50 90; do
  OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_r4scfg2_q$Q; mkdir -p $OUT
  KB_Q=$Q timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py 10 8192x8192 > $OUT/kbench_trace.txt 2>&1 || exit 1
done
echo CFG2_TRACE_OK
cd $GRAFT_REPO_ROOT && bash tools/runs/r4t.sh
