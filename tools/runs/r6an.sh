# round 6: the backend's machine-scheduler strategy at the device link
# (-mllvm -amdgpu-sched-strategy=...; default / max-ilp / max-memory-clause /
# iterative-minreg): bench A/B, kernels alone per 32-frame launch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_bench.sh default build_var/s_max-ilp build_var/s_max-memory-clause build_var/s_iterative-minreg > gpurun_out/r6an_ab.txt 2>&1 || exit 1
cat gpurun_out/r6an_ab.txt
K1AB_B=32 timeout -k 10 400 python3 tools/k1_ab.py default build_var/s_max-ilp build_var/s_max-memory-clause build_var/s_iterative-minreg > gpurun_out/r6an_alone.txt 2>&1 || exit 1
tail -20 gpurun_out/r6an_alone.txt
