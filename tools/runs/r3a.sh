# round 3, first run: host probe (CPU quota), PCIe copy strategies, the new
# 512-frame configs[3] GPU test, the whole GPU suite, the default bench (with
# the host_api and batch4k side measurements) and the batch4k workload at N=1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us 2>&1; cat /proc/self/cgroup; env | grep -i -E "OMP|MAX_JOBS|NUM_THREADS"; } > gpurun_out/r3a_host.txt 2>&1
timeout -k 10 120 tools/ubench/pcie_copy > gpurun_out/r3a_pcie.txt 2>&1 || { echo PCIE_FAILED; tail -20 gpurun_out/r3a_pcie.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_known_answers.py -m gpu -x -v -k batch4k --timeout 300 --timeout-method thread > gpurun_out/r3a_t512.log 2>&1 || { echo T512_FAILED; tail -40 gpurun_out/r3a_t512.log; exit 1; }
tail -3 gpurun_out/r3a_t512.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3a_tests.log; exit 1; }
tail -2 gpurun_out/r3a_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a_bench20.json 2> gpurun_out/r3a_bench20.err || { echo BENCH_FAILED; tail -30 gpurun_out/r3a_bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3a_bench20.json')); print('bench20', d['value'], d['roofline']['frac'], d['side']['host_api'], d['side']['batch4k'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 300 python -u bench.py --workload batch4k --steps 10 --warmup 2 --cpu-seconds 0 --no-side > gpurun_out/r3a_b4k.json 2> gpurun_out/r3a_b4k.err || { echo B4K_FAILED; tail -30 gpurun_out/r3a_b4k.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3a_b4k.json')); print('batch4k', d['value'], d['ms_per_step'], d['roofline']['frac'])"
