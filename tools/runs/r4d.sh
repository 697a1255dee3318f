# round 4: FETCH/WRITE calibration (K1/K6/K2/K4 shapes), SQ counters of the
# shipped 3 x 24 build, kernel trace + traffic + overlap, marginal cost per
# kernel (kskip at 3 x 24), launch shapes 3 x 24 / 4 x 24
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/runs/r4b.sh || { echo R4B_FAILED; exit 1; }
cd $R
timeout -k 10 600 python3 tools/kskip.py > gpurun_out/r4d_kskip.txt 2>&1; tail -14 gpurun_out/r4d_kskip.txt
for shape in "3 24" "4 24" "3 24" "4 24"; do
  set -- $shape
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r4d_shape.json 2>gpurun_out/r4d_shape.err || { tail -5 gpurun_out/r4d_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4d_shape.json')); print('shape $1 x $2', d['value'])" | tee -a gpurun_out/r4d_shapes.txt
done
