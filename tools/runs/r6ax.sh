# round 6: k_tile_scan's workgroup sized to a single frame's tiles (up to 1,024
# threads, one batch of loads each; batches keep 256): GPU tests on the in-tree
# build, single-frame kernel times (ts_old = before), bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ax_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6ax_tests.log; exit 1; }
tail -1 gpurun_out/r6ax_tests.log
for q in 50 90; do
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6ax_8k_q$q build_var/ts_old yuv-manipulations-2_amd || exit 1
  KB_Q=$q bash tools/kab.sh r6ax_4k_q$q build_var/ts_old yuv-manipulations-2_amd || exit 1
done
grep -h "scan_tiles\|compress wall\|round trip wall\|q[59]0: rc" gpurun_out/kab_r6ax_*.txt
bash tools/ab_bench.sh build_var/ts_old default > gpurun_out/r6ax_ab.txt 2>&1 || { cat gpurun_out/r6ax_ab.txt; exit 1; }
cat gpurun_out/r6ax_ab.txt
