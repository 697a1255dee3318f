# round 6: K2's message-length buckets 6 / 12 / 20 (MYYUV_K2_MSZ_SPLIT=3,
# default build) against 8 / 16 (build_var/split2): GPU tests, K2 kernel times,
# bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6y_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6y_tests.log; exit 1; }
tail -1 gpurun_out/r6y_tests.log
KB_Q=50 bash tools/kab.sh r6y_4k_q50 build_var/split2 yuv-manipulations-2_amd || exit 1
KB_Q=50 KB_SIZE=8192x8192 bash tools/kab.sh r6y_8k_q50 build_var/split2 yuv-manipulations-2_amd || exit 1
grep -E "libmyyuv|huff_encode " gpurun_out/kab_r6y_*.txt
bash tools/ab_bench.sh build_var/split2 default > gpurun_out/r6y_ab.txt 2>&1 || exit 1
cat gpurun_out/r6y_ab.txt
