# round 6: k_huff_encode_r16 with its heap in LDS columns (r16::LdsHeap16):
# GPU tests, then kernel times (single frames, gate 0 variants) and bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6n_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6n_tests.log; exit 1; }
tail -1 gpurun_out/r6n_tests.log
for q in 50 90; do
  KB_Q=$q bash tools/kab.sh r6n_4k_q$q build_var/base build_var/g0 build_var/g0lds || exit 1
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6n_8k_q$q build_var/base yuv-manipulations-2_amd build_var/g0lds || exit 1
done
bash tools/ab_bench.sh build_var/base default build_var/reg > gpurun_out/r6n_ab.txt 2>&1 || exit 1
cat gpurun_out/r6n_ab.txt
