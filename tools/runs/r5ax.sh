# round 5: K2's count scan by every wave into its own LDS copy (one barrier
# less before the runs): GPU tests, K2's window phases, per-kernel times and
# six alternating bench rounds against the previous commit (build_var/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ax_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5ax_tests.log; exit 1; }
tail -1 gpurun_out/r5ax_tests.log
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 200 python3 tools/k2_phase.py 24 > gpurun_out/r5ax_k2_phase.txt 2>&1; cat gpurun_out/r5ax_k2_phase.txt
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5ax_kab.txt 2>&1; cat gpurun_out/r5ax_kab.txt
timeout -k 10 700 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5ax_ab.txt && cat gpurun_out/r5ax_ab.txt
timeout -k 10 700 bash tools/ab_bench.sh build_var/base default > /dev/null && cat gpurun_out/ab_bench.txt >> gpurun_out/r5ax_ab.txt && cat gpurun_out/ab_bench.txt
