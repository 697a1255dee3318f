# round 6 validation after K2's ovf class and length buckets:
# GPU tests, smoke, driver-shape and default bench lines, kernel trace +
# calibrated traffic of the bench workload, configs[2] trace + traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6aa_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6aa_tests.log; exit 1; }
tail -1 gpurun_out/r6aa_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6aa_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r6aa_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6aa_bench20.json 2> gpurun_out/r6aa_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6aa_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6aa_bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_isolated'], d['side']['host_api']['value'], d['side']['host_batch']['value'], d['cpu_baseline']['value'], d['side']['batch4k']['value'])"
timeout -k 10 400 python -u bench.py --cpu-seconds 0 > gpurun_out/r6aa_bench.json 2> gpurun_out/r6aa_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6aa_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6aa_bench.json')); print('bench', d['value'], d['kernel_us'])"
bash tools/profile.sh r6aa 20 && echo PROFILE_OK
cd $GRAFT_REPO_ROOT && bash tools/cfg2_profile.sh r6aacfg2 10 > gpurun_out/r6aa_cfg2.txt 2>&1 && echo CFG2_OK
cd $GRAFT_REPO_ROOT && K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default > gpurun_out/r6aa_alone.txt 2>&1 && cat gpurun_out/r6aa_alone.txt | tail -15
