# round 6: the pipelined host-buffer batches (tests + the bench's side.host_batch)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: timeout -k 10 600 python -u -m pytest tests/test_gpu_host_batch.py tests/test_cli.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6b_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/r6b_tests.log; exit 1; }
tail -3 gpurun_out/r6b_tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6b_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6b_bench.json')); print('bench', d['value'], d['side']['host_api'], d['side']['host_batch'])"
