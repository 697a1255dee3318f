# round 3: DPP quad exchange (K1) and DPP scans (K2 dense run, K4, tile scan),
# ballot-descent wave max in K2; tests, repeated-compression determinism, A/B
# against the build without them (allbis = HEAD) and round 2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3m_tests.log; exit 1; }
tail -2 gpurun_out/r3m_tests.log
NRUNS=12 timeout -k 10 300 python -u tools/diag/first_diff.py 90 > gpurun_out/r3m_det.log 2>&1 && grep -v amdgpu.ids gpurun_out/r3m_det.log | head -3
timeout -k 10 300 python3 tools/k1_ab.py default build_var/allbis build_var/r2 > gpurun_out/r3m_kab.txt 2>&1; cat gpurun_out/r3m_kab.txt
timeout -k 10 900 bash tools/ab_bench.sh default build_var/allbis && cp gpurun_out/ab_bench.txt gpurun_out/r3m_ab.txt && cat gpurun_out/r3m_ab.txt
