set -o pipefail
cd $GRAFT_REPO_ROOT
for v in default build_var/c8 build_var/c8d build_var/c4d; do
  lib=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so; [ $v != default ] && lib=$GRAFT_REPO_ROOT/$v/libmyyuv_hip.so
  echo "== $v"; MYYUV_HIP_LIB=$lib timeout -k 10 120 python3 tools/host_api_rate.py 2>&1 | grep -v amdgpu.ids || exit 1
done
