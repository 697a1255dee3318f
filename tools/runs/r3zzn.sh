# final validation (CAP-16 tier at 5 waves/SIMD, 3 x 24): GPU tests, smoke, driver-shape and default bench lines,
# batch4k, then the kernel trace + HBM traffic of the bench workload and configs[2]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zzn_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zzn_tests.log; exit 1; }
tail -1 gpurun_out/r3zzn_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3zzn_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r3zzn_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3zzn_bench20.json 2> gpurun_out/r3zzn_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r3zzn_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3zzn_bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_decode_isolated']['avg_launch_us'], d['side']['host_api']['value'], d['cpu_baseline']['value'], d['side']['batch4k']['value'])"
timeout -k 10 400 python -u bench.py --cpu-seconds 0 > gpurun_out/r3zzn_bench.json 2> gpurun_out/r3zzn_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r3zzn_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3zzn_bench.json')); print('bench', d['value'])"
for shape in "3 24" "3 24"; do set -- $shape
timeout -k 10 300 python -u bench.py --workload batch4k --steps 10 --warmup 2 --cpu-seconds 0 --no-side --inflight $1 --batch $2 > gpurun_out/r3zzn_b4k.json 2> gpurun_out/r3zzn_b4k.err || { echo B4K_FAILED; tail -30 gpurun_out/r3zzn_b4k.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3zzn_b4k.json')); print('batch4k $1 x $2', d['value'], d['ms_per_step'])"
done
bash tools/profile.sh r3zzn 20 && echo PROFILE_OK && bash tools/cfg2_profile.sh r3zcfg2 10 && echo CFG2_OK
