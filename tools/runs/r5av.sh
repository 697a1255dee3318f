# round 5: K2's classification by one LDS atomic per lane and round (count and
# rank) instead of a ballot per key: GPU tests, K2's window phases (stamp
# build), per-kernel times and the bench A/B against the previous commit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5av_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5av_tests.log; exit 1; }
tail -1 gpurun_out/r5av_tests.log
MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/stamps/libmyyuv_hip.so timeout -k 10 200 python3 tools/k2_phase.py 24 > gpurun_out/r5av_k2_phase.txt 2>&1; cat gpurun_out/r5av_k2_phase.txt
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/base > gpurun_out/r5av_kab.txt 2>&1; cat gpurun_out/r5av_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r5av_ab.txt && cat gpurun_out/r5av_ab.txt
