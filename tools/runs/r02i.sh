set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02i_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02i_tests.log; exit 1; }
tail -2 gpurun_out/r02i_tests.log
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/r02i_bench.json 2> gpurun_out/r02i_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r02i_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02i_bench.json')); print(d['value'], d['kernel_us'])"
bash tools/ab_bench.sh default MYYUV_ENCODER=fused
