# launch-group size in the driver's command shape (--steps 20 --warmup 5), three alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
: > gpurun_out/r05e_batch.txt
for round in 1 2 3; do
  for B in 6 7 8; do
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --batch $B --cpu-seconds 0 --no-side --breakdown-steps 0 > gpurun_out/r05e_one.json 2> gpurun_out/r05e_one.err || { tail -20 gpurun_out/r05e_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05e_one.json')); print('batch $B', d['value'], d['ms_per_step'])" >> gpurun_out/r05e_batch.txt
  done
done
cat gpurun_out/r05e_batch.txt
