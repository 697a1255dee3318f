set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02f_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02f_tests.log; exit 1; }
tail -3 gpurun_out/r02f_tests.log
for m in split fused; do
  MYYUV_ENCODER=$m timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/r02f_bench_$m.json 2> gpurun_out/r02f_bench_$m.err || { echo BENCH_FAILED; tail -30 gpurun_out/r02f_bench_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r02f_bench_$m.json')); print('$m', d['value'], d['kernel_us'])"
done
