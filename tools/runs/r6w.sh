# round 6: K2's ovf class (blocks with >= 16 symbol slots straight to the
# overflow worklist, no CAP-8 build): GPU tests, kernel times (bench frame,
# 8192^2 q50/q90) against no ovf class, bench A/B with thresholds 13 / 16 / 20
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6w_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6w_tests.log; exit 1; }
tail -1 gpurun_out/r6w_tests.log
KB_Q=50 bash tools/kab.sh r6w_4k_q50 build_var/noovf yuv-manipulations-2_amd || exit 1
for q in 50 90; do
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6w_8k_q$q build_var/noovf yuv-manipulations-2_amd || exit 1
done
grep -E "libmyyuv|huff_encode|compress wall" gpurun_out/kab_r6w_*.txt
bash tools/ab_bench.sh build_var/noovf default build_var/ovf13 build_var/ovf20 > gpurun_out/r6w_ab.txt 2>&1 || exit 1
cat gpurun_out/r6w_ab.txt
