# K2 occupancy (workgroups per CU: 5 in-tree, 6 = k2w6, 4 = k2w4) and the
# launch-group shape (--inflight x --batch) with the window-sorted K2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/k1_ab.py default build_var/k2w6 build_var/k2w4 > gpurun_out/r3zd_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zd_kernels.txt; exit 1; }
cat gpurun_out/r3zd_kernels.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/k2w6 build_var/k2w4 > gpurun_out/r3zd_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zd_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zd_ab.txt
cat gpurun_out/r3zd_ab.txt
: > gpurun_out/r3zd_shape.txt
for round in 1 2; do
  for shape in "3 7" "3 6" "3 8" "4 6" "4 7" "2 10"; do
    set -- $shape
    timeout -k 10 120 python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --breakdown-steps 0 --no-side --no-kernel-events --inflight $1 --batch $2 > gpurun_out/r3zd_one.json 2> gpurun_out/r3zd_one.err || { tail -5 gpurun_out/r3zd_one.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r3zd_one.json')); print('inflight $1 batch $2', d['value'])" >> gpurun_out/r3zd_shape.txt
  done
done
cat gpurun_out/r3zd_shape.txt
