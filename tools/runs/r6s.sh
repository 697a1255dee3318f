# round 6: bench line with per-kernel events after the CAP-16 tier's LDS heap
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r6s_bench.json 2> gpurun_out/r6s_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6s_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6s_bench.json')); print(d['value'], d['kernel_us'], d['roofline']['frac'], d.get('roofline_isolated',{}).get('frac'))"
