# round 6: k_scan_chain's sizes per thread (MYYUV_SCAN_PER_THREAD 8 / 32
# against 16: 2,048 / 8,192 / 4,096-block chained tiles): decode-side GPU
# tests on both, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in spt8 spt32; do
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/$v/libmyyuv_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or golden or batch or random_sweep or noise" > gpurun_out/r6ay_tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -30 gpurun_out/r6ay_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r6ay_tests_$v.log)"
done
bash tools/ab_bench.sh default build_var/spt8 build_var/spt32 > gpurun_out/r6ay_ab.txt 2>&1 || { cat gpurun_out/r6ay_ab.txt; exit 1; }
cat gpurun_out/r6ay_ab.txt
