# round 6: which source file the iterative-minreg scheduler breaks (r6ao):
# non-rdc builds with the flag on one file each (tools/diag/build_mixed_sched.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in nr_none nr_k_huff_encode nr_k_transform nr_k_huff_decode nr_k_stream; do
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/$v/libmyyuv_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -q --timeout 120 --timeout-method thread -k "k2_windows or tiled_8192 or golden_big or repeated_compress" > gpurun_out/r6ap_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/r6ap_$v.log)"
  [ $rc -le 1 ] || exit 1
done
