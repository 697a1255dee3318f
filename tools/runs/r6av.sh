# round 6: final HEAD check (GPU tests incl. the random sweep, smoke, driver-shape bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6av_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6av_tests.log; exit 1; }
tail -1 gpurun_out/r6av_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6av_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r6av_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6av_bench20.json 2> gpurun_out/r6av_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6av_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6av_bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_isolated']['frac'], d['verified'])"
