# round 4 validation of the shipped build (K1 fast path + out-of-line exact
# path, K1's block words for K2, 4 x 24): GPU tests, smoke, driver-shape and
# default bench lines, batch4k, then the kernel trace + calibrated HBM traffic
# of the bench workload, configs[2], and the SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4n_tests.log; exit 1; }
tail -1 gpurun_out/r4n_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r4n_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4n_bench20.json 2> gpurun_out/r4n_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r4n_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4n_bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_isolated'], d['roofline_decode_isolated']['avg_launch_us'], d['side']['host_api']['value'], d['cpu_baseline']['value'], d['side']['batch4k']['value'])"
timeout -k 10 400 python -u bench.py --cpu-seconds 0 > gpurun_out/r4n_bench.json 2> gpurun_out/r4n_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r4n_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4n_bench.json')); print('bench', d['value'], d['kernel_us'])"
bash tools/profile.sh r4n 20 && echo PROFILE_OK && bash tools/cfg2_profile.sh r4cfg2 10 && echo CFG2_OK
SQ_BENCH=1 bash tools/sq_counters.sh r4n && echo SQ_OK
