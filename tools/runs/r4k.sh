# round 4: K1 writes a per-block word (row mask, msz, class, DC) and K2
# classifies from it instead of re-reading the coefficient rows (in-tree),
# against the previous commit (build_var/base); decoder ablations
# (MYYUV_K5_EXP 1: no symbol loop, 2: no table parse either, 3: no transform)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4k_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4k_tests.log; exit 1; }
tail -1 gpurun_out/r4k_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r4k_smoke.log; exit 1; }
echo smoke ok
K1AB_B=24 timeout -k 10 500 python3 tools/k1_ab.py default build_var/base build_var/dexp1 build_var/dexp2 build_var/dexp3 > gpurun_out/r4k_kab.txt 2>&1; cat gpurun_out/r4k_kab.txt
timeout -k 10 600 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4k_ab.txt && cat gpurun_out/r4k_ab.txt
