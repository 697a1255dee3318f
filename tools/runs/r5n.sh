# round 5: decoder round-1 staging by LDS-DMA issued with the size bytes (one
# load round trip less before the parse) + DPP size scan: GPU tests, kernel
# times and bench A/B against HEAD (build_var/base); the persistent decoder's
# grid sweep (build_var/persist, MYYUV_DEC_GRID); launch shapes at 20 steps;
# k_tile_scan's totals kept in registers between its passes (8192x8192 kbench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5n_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5n_tests.log; exit 1; }
tail -1 gpurun_out/r5n_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5n_kab.txt 2>&1; cat gpurun_out/r5n_kab.txt
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/persist/libmyyuv_hip.so K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py MYYUV_DEC_GRID=5120 MYYUV_DEC_GRID=100000000 > gpurun_out/r5n_persist_grid.txt 2>&1; cat gpurun_out/r5n_persist_grid.txt
: > gpurun_out/r5n_kbench.txt
for lib in build_var/base default; do
  L=$GRAFT_REPO_ROOT/$lib/libmyyuv_hip.so; [ $lib = default ] && L=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so
  echo "== $lib 8192x8192 q50" >> gpurun_out/r5n_kbench.txt
  MYYUV_HIP_LIB=$L timeout -k 10 120 python3 tools/kbench.py 10 8192x8192 >> gpurun_out/r5n_kbench.txt 2>&1 || exit 1
done
grep -E "==|scan_tiles|huff_decode" gpurun_out/r5n_kbench.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5n_ab.txt && cat gpurun_out/r5n_ab.txt
: > gpurun_out/r5n_shapes20.txt
for rnd in 1 2 3; do
for shape in "4 24" "4 16"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r5n_shape.json 2>gpurun_out/r5n_shape.err || { tail -5 gpurun_out/r5n_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5n_shape.json')); print('shape $1 x $2 (20 steps)', d['value'])" | tee -a gpurun_out/r5n_shapes20.txt
done
done
