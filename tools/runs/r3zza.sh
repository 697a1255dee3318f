# decoder symbol loop: the table's first entry from a register (fewer distinct LDS addresses per value read)
# against HEAD (prev)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zza_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3zza_tests.log; exit 1; }
tail -1 gpurun_out/r3zza_tests.log
timeout -k 10 300 python3 tools/k1_ab.py build_var/prev default > gpurun_out/r3zza_kernels.txt 2>&1 || { echo KAB_FAILED; tail -20 gpurun_out/r3zza_kernels.txt; exit 1; }
cat gpurun_out/r3zza_kernels.txt
timeout -k 10 500 bash tools/ab_bench.sh build_var/prev default > gpurun_out/r3zza_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zza_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zza_ab.txt
cat gpurun_out/r3zza_ab.txt
