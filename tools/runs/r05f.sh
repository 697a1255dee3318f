set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r05f_tests.log; exit 1; }
tail -2 gpurun_out/r05f_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05f_bench20.json 2> gpurun_out/r05f_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r05f_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05f_bench20.json')); print('bench20', d['value'], d['roofline']['frac'], d['cpu_baseline'])"
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/r05f_bench.json 2> gpurun_out/r05f_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r05f_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05f_bench.json')); print('bench', d['value'])"
bash tools/profile.sh r05f 20 && echo PROFILE_OK
