# round 3: K1 writes an 8-byte nonzero map per block (no row-mask byte), K2
# classifies from it; A/B against the round-2 build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -2 gpurun_out/r3c_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-side --cpu-seconds 0 > gpurun_out/r3c_bench20.json 2> gpurun_out/r3c_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r3c_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3c_bench20.json')); print('bench20', d['value'], d['roofline']['frac'], d['kernel_us'])"
timeout -k 10 900 bash tools/ab_bench.sh default build_var/r2 && cp gpurun_out/ab_bench.txt gpurun_out/r3c_ab.txt
