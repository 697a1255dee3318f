set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04e_tests.log; exit 1; }
tail -2 gpurun_out/r04e_tests.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04e_bench20.json 2> gpurun_out/r04e_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r04e_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04e_bench20.json')); print('bench20', d['value'], d['roofline']['frac'], d['roofline_isolated'], d['roofline_decode_isolated'], d['cpu_baseline'], d['kernel_us'])"
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r04e_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04e_bench.json')); print('bench', d['value'])"
bash tools/profile.sh r04e 20 && echo PROFILE_OK
