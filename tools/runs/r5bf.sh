# round 5: last check of the in-tree build as __graft_entry__.build() left it
# (HEAD 708a298): GPU tests, smoke, one driver-shape bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bf_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5bf_tests.log; exit 1; }
tail -1 gpurun_out/r5bf_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5bf_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r5bf_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5bf_bench20.json 2> gpurun_out/r5bf_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r5bf_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5bf_bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_isolated']['avg_launch_us'], d['side']['batch4k']['value'], d['verified']['timed_region'][:60])"
