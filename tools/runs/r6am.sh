# round 6: the CAP-16 tier's phase 1 by sorting (r16::distinct_sorted) vs the
# per-position search: GPU tests on the sorted build, kernel times (single
# frames), bench A/B (default = the in-tree search build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/sort1/libmyyuv_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6am_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6am_tests.log; exit 1; }
tail -1 gpurun_out/r6am_tests.log
for q in 50 90; do
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6am_8k_q$q yuv-manipulations-2_amd build_var/sort1 build_var/sort1w4 || exit 1
done
grep -h "r16" gpurun_out/kab_r6am_*.txt | head -20
bash tools/ab_bench.sh default build_var/sort1 build_var/sort1w4 > gpurun_out/r6am_ab.txt 2>&1 || exit 1
cat gpurun_out/r6am_ab.txt
