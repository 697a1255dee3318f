set -o pipefail
cd $GRAFT_REPO_ROOT
for v in default build_var/k5e1 build_var/k5e2 MYYUV_DECODER=split; do
  lib=$GRAFT_REPO_ROOT/yuv-manipulations-2_amd/libmyyuv_hip.so; envs=""
  case "$v" in default) ;; *=*) envs="$v" ;; *) lib=$GRAFT_REPO_ROOT/$v/libmyyuv_hip.so ;; esac
  echo "== $v"; env $envs MYYUV_HIP_LIB=$lib timeout -k 10 120 python3 tools/dec_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done
