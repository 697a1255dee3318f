# round 6: single-frame CAP-16 tier gate (default 16384 / 0 / 24576) and the
# wave pass for batches' tier remainders (MYYUV_BATCH_WAVE_LIMIT=4096)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6o_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6o_tests.log; exit 1; }
tail -1 gpurun_out/r6o_tests.log
for q in 50 90; do
  KB_Q=$q bash tools/kab.sh r6o_4k_q$q yuv-manipulations-2_amd build_var/gs0 build_var/gs24k || exit 1
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6o_8k_q$q yuv-manipulations-2_amd build_var/gs0 build_var/gs24k || exit 1
done
bash tools/ab_bench.sh default build_var/bw4k > gpurun_out/r6o_ab.txt 2>&1 || exit 1
cat gpurun_out/r6o_ab.txt
