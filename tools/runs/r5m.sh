# round 5: persistent decoder grid sweep (MYYUV_DEC_GRID) against HEAD (build_var/base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default MYYUV_DEC_GRID=2560 MYYUV_DEC_GRID=5120 MYYUV_DEC_GRID=10240 MYYUV_DEC_GRID=100000000 build_var/base > gpurun_out/r5m_kab.txt 2>&1; cat gpurun_out/r5m_kab.txt
# driver-shape (20 steps) launch shapes 4 x 24 against 4 x 16, three rounds (HEAD build)
: > gpurun_out/r5m_shapes20.txt
for rnd in 1 2 3; do
for shape in "4 24" "4 16"; do
  set -- $shape
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/base/libmyyuv_hip.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --inflight $1 --batch $2 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events > gpurun_out/r5m_shape.json 2>gpurun_out/r5m_shape.err || { tail -5 gpurun_out/r5m_shape.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5m_shape.json')); print('shape $1 x $2 (20 steps)', d['value'])" | tee -a gpurun_out/r5m_shapes20.txt
done
done
