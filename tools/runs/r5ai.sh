# round 5: the decoder transform in 8-block units (stamps8, all units) and
# hybrid (working tree: 16-block units, the last 1-8 blocks as one 8-block
# unit) against 16-block units (HEAD): per-phase wave cycles of stamp builds,
# then GPU tests, per-kernel times and the bench A/B of the hybrid
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in stamps stamps8 stampsh; do
  echo "== $v"
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/$v/libmyyuv_hip.so timeout -k 10 200 python3 tools/dec_phase.py 12 > gpurun_out/r5ai_phase_$v.txt 2>&1 || { echo PHASE_FAILED; cat gpurun_out/r5ai_phase_$v.txt; exit 1; }
  cat gpurun_out/r5ai_phase_$v.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ai_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5ai_tests.log; exit 1; }
tail -1 gpurun_out/r5ai_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5ai_kab.txt 2>&1; cat gpurun_out/r5ai_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5ai_ab.txt && cat gpurun_out/r5ai_ab.txt
