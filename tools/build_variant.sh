#!/bin/bash
# Builds libmyyuv_hip.so with extra compiler flags into build_var/<name>/ (for
# tools/ab_bench.sh):  tools/build_variant.sh <name> -DFOO=1 ...
# (ARCH=gfx950:xnack- ... builds for that target id instead of gfx950;
# LINKFLAGS="-mllvm ..." adds code-generation options: with -fgpu-rdc the
# device code is generated at the link)
set -e
R=$(cd $(dirname $0)/.. && pwd)
name=$1; shift
out=$R/build_var/$name; mkdir -p $out
C=$R/yuv-manipulations-2_amd/csrc
F="--offload-arch=${ARCH:-gfx950} -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall -I$C -I$R/include -fgpu-rdc $*"
objs=""
for k in k_transform k_huff_encode k_huff_decode k_stream k_color; do
  /opt/rocm/bin/hipcc $F -c $C/$k.hip -o $out/$k.o & objs="$objs $out/$k.o"
done
/opt/rocm/bin/hipcc $F -x hip -c $C/myyuv_hip.cpp -o $out/myyuv_hip.o & objs="$objs $out/myyuv_hip.o"
wait
/opt/rocm/bin/hipcc --offload-arch=${ARCH:-gfx950} -fgpu-rdc --hip-link -shared -mllvm -vectorize-slp=false ${LINKFLAGS:-} -o $out/libmyyuv_hip.so $objs
rm -f $out/*.o
echo built $out/libmyyuv_hip.so
