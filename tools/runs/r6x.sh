# round 6: the decoder's table walk as one predicated loop per wave
# (MYYUV_K5_WALK=1) against the divergent per-lane loops (build_var/walk0):
# GPU tests, decode kernel times, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6x_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6x_tests.log; exit 1; }
tail -1 gpurun_out/r6x_tests.log
for q in 50 90; do
  KB_Q=$q bash tools/kab.sh r6x_4k_q$q build_var/walk0 yuv-manipulations-2_amd || exit 1
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6x_8k_q$q build_var/walk0 yuv-manipulations-2_amd || exit 1
done
grep -E "libmyyuv|huff_decode" gpurun_out/kab_r6x_*.txt
bash tools/ab_bench.sh build_var/walk0 default > gpurun_out/r6x_ab.txt 2>&1 || exit 1
cat gpurun_out/r6x_ab.txt
