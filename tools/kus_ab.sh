#!/bin/bash
# Isolated per-kernel times (bench breakdown pass, one launch group at a time)
# for library variants:  tools/kus_ab.sh <variant>...   (see ab_bench.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for d in "$@"; do
  lib=$R/yuv-manipulations-2_amd/libmyyuv_hip.so; envs=""
  case "$d" in
    default) ;;
    *=*) envs="$d" ;;
    *) lib=$R/$d/libmyyuv_hip.so ;;
  esac
  env $envs MYYUV_HIP_LIB=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 \
    --no-side > gpurun_out/kus_one.json 2>gpurun_out/kus_one.err || { cat gpurun_out/kus_one.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/kus_one.json')); print('$d', d['value'], {k: round(v, 1) for k, v in d['kernel_us'].items()})"
done
