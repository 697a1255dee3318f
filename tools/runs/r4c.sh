# round 4: GPU tests with the cooperative stream writer as the default (split
# arrangement) and the lane writer (fused arrangement), smoke, driver-shape
# bench, then A/B lane vs coop (bench, 3 alternating rounds) and per-kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4c_tests.log; exit 1; }
tail -1 gpurun_out/r4c_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r4c_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4c_bench20.json 2> gpurun_out/r4c_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r4c_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4c_bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['side']['host_api']['value'], d['cpu_baseline']['value'], d['side']['batch4k']['value'], d['kernel_us'])"
timeout -k 10 900 bash tools/ab_bench.sh MYYUV_STREAM_OUT=lane MYYUV_STREAM_OUT=coop build_var/r16nosort > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4c_ab.txt && cat gpurun_out/r4c_ab.txt
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py MYYUV_STREAM_OUT=lane MYYUV_STREAM_OUT=coop build_var/r16nosort > gpurun_out/r4c_kab.txt 2>&1; cat gpurun_out/r4c_kab.txt
