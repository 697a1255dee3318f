# stream priorities of the three launch-group streams, driver shape, three alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
: > gpurun_out/r05h_prio.txt
for round in 1 2 3; do
  for P in 0 -1,0,0 -1,-1,0; do
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stream-priority=$P --cpu-seconds 0 --no-side --breakdown-steps 0 > gpurun_out/r05h_one.json 2> gpurun_out/r05h_one.err || { tail -20 gpurun_out/r05h_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05h_one.json')); print('prio $P', d['value'])" >> gpurun_out/r05h_prio.txt
  done
done
cat gpurun_out/r05h_prio.txt
