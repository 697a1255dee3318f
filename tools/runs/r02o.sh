set -o pipefail
cd $GRAFT_REPO_ROOT
for v in stb st4 st8; do
  echo "== $v"
  MYYUV_HIP_LIB=$GRAFT_REPO_ROOT/build_var/$v/libmyyuv_hip.so timeout -k 10 200 python3 tools/k2_time.py 2>&1 | grep -v "array\|dtype" | head -8 || exit 1
done > gpurun_out/k2_time_r02o.txt
timeout -k 10 900 bash tools/ab_bench.sh default build_var/s8 build_var/s8w4 build_var/s4w4
