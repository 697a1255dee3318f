# round 4: K1's exact path moved out of line (k_fdct_fix over the units K1
# lists; K1 63 VGPRs): every GPU test, smoke, then per-kernel times and the
# bench A/B against the fix grid at the resident count (MYYUV_FIX_GRID=0) and
# the in-kernel exact path with the column-sequential stage 2 (build_var/seq)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4h_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4h_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r4h_smoke.log; exit 1; }
echo smoke ok
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default MYYUV_FIX_GRID=0 build_var/seq > gpurun_out/r4h_kab.txt 2>&1; cat gpurun_out/r4h_kab.txt
timeout -k 10 800 bash tools/ab_bench.sh default MYYUV_FIX_GRID=0 build_var/seq > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4h_ab.txt && cat gpurun_out/r4h_ab.txt
