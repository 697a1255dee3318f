# more hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4) with more launch groups in flight
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r3zj_hwq.txt
for round in 1 2; do
  for cfg in "4 4 8" "8 4 8" "8 5 8" "8 6 6" "8 6 8" "8 8 6" "16 8 8"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 150 python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events --inflight $2 --batch $3 > gpurun_out/r3zj_one.json 2> gpurun_out/r3zj_one.err || { tail -5 gpurun_out/r3zj_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r3zj_one.json')); print('hwq $1 inflight $2 batch $3 steps 40', d['value'])" >> gpurun_out/r3zj_hwq.txt
  done
  for cfg in "4 4 8" "8 6 8" "8 8 6"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --breakdown-steps 0 --no-side --inflight $2 --batch $3 > gpurun_out/r3zj_one.json 2> gpurun_out/r3zj_one.err || { tail -5 gpurun_out/r3zj_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r3zj_one.json')); print('hwq $1 inflight $2 batch $3 steps 20 (driver shape)', d['value'])" >> gpurun_out/r3zj_hwq.txt
  done
done
cat gpurun_out/r3zj_hwq.txt
