# round 4: the decoder's table parse from a 20-byte register prefix of each
# chunk (treg) against reading every group header from LDS as the walk
# reaches it (default): parity tests of treg, per-kernel times, the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/treg/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4x_treg_tests.log 2>&1; echo "treg tests rc=$?"; tail -2 gpurun_out/r4x_treg_tests.log
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/treg > gpurun_out/r4x_kab.txt 2>&1; cat gpurun_out/r4x_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/treg > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4x_ab.txt && cat gpurun_out/r4x_ab.txt
: > gpurun_out/r4x_shapes.txt
for rnd in 1 2; do
for shape in "4 24" "4 32"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r4x_shape.json 2>gpurun_out/r4x_shape.err || { tail -5 gpurun_out/r4x_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4x_shape.json')); print('shape $1 x $2 (40 steps)', d['value'])" | tee -a gpurun_out/r4x_shapes.txt
done
done
