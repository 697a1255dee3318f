# round 5: repeated bench runs of the working tree (K2 LDS-atomic
# classification) with the per-kernel breakdown, to see which kernel an
# outlier run (~295k) slows
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r5av3.txt
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --no-side > gpurun_out/r5av3_one.json 2> gpurun_out/r5av3_one.err || { tail -5 gpurun_out/r5av3_one.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5av3_one.json')); print(d['value'], d['kernel_us'])" | tee -a gpurun_out/r5av3.txt
done
