#!/bin/bash
# Diagnostic builds: tools/variant2.sh <out-dir> [hipcc flags...]: every kernel
# file and the host launch code rebuilt with the extra flags.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/yuv-manipulations-2_amd
OUT=$1; shift
mkdir -p "$OUT"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -I$P/csrc -I$R/include"
OBJS=""
for k in k_transform k_huff_encode k_huff_decode k_stream; do
  /opt/rocm/bin/hipcc $FLAGS "$@" -fgpu-rdc -c "$P/csrc/$k.hip" -o "$OUT/$k.o" &
  OBJS="$OBJS $OUT/$k.o"
done
/opt/rocm/bin/hipcc $FLAGS "$@" -fgpu-rdc -x hip -c "$P/csrc/myyuv_hip.cpp" -o "$OUT/myyuv_hip.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fgpu-rdc --hip-link -shared -o "$OUT/libmyyuv_hip.so" $OBJS "$OUT/myyuv_hip.o"
