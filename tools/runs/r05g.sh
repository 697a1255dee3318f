set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05g_bench20.json 2> gpurun_out/r05g_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r05g_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05g_bench20.json')); print('bench20', d['value'], d['roofline'], d['cpu_baseline']['value'], d['cpu_baseline']['single_thread']['value'])"
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/r05g_bench.json 2> gpurun_out/r05g_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r05g_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05g_bench.json')); print('bench', d['value'], d['roofline'])"
