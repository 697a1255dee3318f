set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02d_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02d_tests.log; exit 1; }
tail -3 gpurun_out/r02d_tests.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02d_bench20.json 2> gpurun_out/r02d_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r02d_bench20.err; exit 1; }
cat gpurun_out/r02d_bench20.json
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/r02d_bench.json 2> gpurun_out/r02d_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r02d_bench.err; exit 1; }
cat gpurun_out/r02d_bench.json
