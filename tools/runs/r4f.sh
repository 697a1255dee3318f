# round 4: the fast forward transform (FMA chains + rigorous bound, exact
# fallback per unit; xform_common.hpp fdct_core) with K2's DC from LDS, as the
# in-tree build: every GPU test, smoke, then A/B against the DC-only build
# (round-3 K1) and the fast transform compiled for 6 waves per SIMD, and
# per-kernel times at 24-frame launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4f_tests.log; exit 1; }
tail -1 gpurun_out/r4f_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r4f_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 700 bash tools/ab_bench.sh default build_var/k2dc build_var/fastdct_o6 > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4f_ab.txt && cat gpurun_out/r4f_ab.txt
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/k2dc build_var/fastdct_o6 > gpurun_out/r4f_kab.txt 2>&1; cat gpurun_out/r4f_kab.txt
