# round 6: the CAP-16 tier's LDS heap with predicated, unrolled walks (no
# divergent loops): GPU tests, kernel times (8192^2 q50/q90, chef-big q90),
# bench A/B against the looped walks (build_var/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6v_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6v_tests.log; exit 1; }
tail -1 gpurun_out/r6v_tests.log
for q in 50 90; do
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6v_8k_q$q build_var/base yuv-manipulations-2_amd || exit 1
done
grep -E "libmyyuv|r16|wave|wide|compress wall" gpurun_out/kab_r6v_*.txt
bash tools/ab_bench.sh build_var/base default > gpurun_out/r6v_ab.txt 2>&1 || exit 1
cat gpurun_out/r6v_ab.txt
