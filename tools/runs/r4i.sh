# round 4: the r16 tier's leftovers (blocks with more than 16 distinct
# symbols: ~14 per bench frame, ~340 per 24-frame launch) through the
# wave-per-block pass instead of the lane-per-block CAP-64 pass in batches
# (build_var/bwl: MYYUV_BATCH_WAVE_LIMIT=24576); launch shapes of the new K1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/bwl > gpurun_out/r4i_kab.txt 2>&1; cat gpurun_out/r4i_kab.txt
timeout -k 10 600 bash tools/ab_bench.sh default build_var/bwl > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4i_ab.txt && cat gpurun_out/r4i_ab.txt
: > gpurun_out/r4i_shapes.txt
for shape in "3 24" "3 32" "4 24" "4 16" "3 24" "3 32" "4 24" "4 16"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r4i_shape.json 2>gpurun_out/r4i_shape.err || { tail -5 gpurun_out/r4i_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4i_shape.json')); print('shape $1 x $2', d['value'])" | tee -a gpurun_out/r4i_shapes.txt
done
