# round 3: K2 classifies from K1's nonzero maps (one coefficient load per block)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/pcie_copy > gpurun_out/r3b_pcie.txt 2>&1 || { echo PCIE_FAILED; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-side --cpu-seconds 0 > gpurun_out/r3b_bench20.json 2> gpurun_out/r3b_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r3b_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3b_bench20.json')); print('bench20', d['value'], d['roofline']['frac'], d['kernel_us'])"
timeout -k 10 400 python -u bench.py --steps 40 --no-side --cpu-seconds 0 > gpurun_out/r3b_bench40.json 2> gpurun_out/r3b_bench40.err || { echo BENCH_FAILED; tail -30 gpurun_out/r3b_bench40.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3b_bench40.json')); print('bench40', d['value'], d['roofline']['frac'], d['kernel_us'])"
timeout -k 10 300 python -u tools/kskip.py > gpurun_out/r3b_kskip.txt 2>&1 || { echo KSKIP_FAILED; tail -5 gpurun_out/r3b_kskip.txt; exit 1; }
cat gpurun_out/r3b_kskip.txt | grep -v amdgpu.ids
