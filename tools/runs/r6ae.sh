# round 6: the bench's new default launch shape (4 x 32): driver-shape and
# default bench lines, kernel trace + calibrated traffic of the workload
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6ae_bench20.json 2> gpurun_out/r6ae_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6ae_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6ae_bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_isolated']['frac'], d['config'], d['side']['host_api']['value'], d['side']['host_batch']['value'], d['cpu_baseline']['value'], d['side']['batch4k']['value'])"
timeout -k 10 400 python -u bench.py --cpu-seconds 0 > gpurun_out/r6ae_bench.json 2> gpurun_out/r6ae_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6ae_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6ae_bench.json')); print('bench', d['value'], d['kernel_us'])"
bash tools/profile.sh r6ae 20 && echo PROFILE_OK
