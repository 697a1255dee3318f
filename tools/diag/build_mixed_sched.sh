#!/bin/bash
# Diagnostic: a build without -fgpu-rdc (device code generated per file) with
# the iterative-minreg machine scheduler on one source file only, to find
# which file a scheduler change breaks:  build_mixed_sched.sh <name> <file>
set -e
R=$(cd $(dirname $0)/../.. && pwd)
name=$1; ff=$2
out=$R/build_var/$name; mkdir -p $out
C=$R/yuv-manipulations-2_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall -I$C -I$R/include -mllvm -vectorize-slp=false"
objs=""
for k in k_transform k_huff_encode k_huff_decode k_stream k_color; do
  X=""; [ "$k" = "$ff" ] && X="-mllvm -amdgpu-sched-strategy=iterative-minreg"
  /opt/rocm/bin/hipcc $F $X -c $C/$k.hip -o $out/$k.o & objs="$objs $out/$k.o"
done
/opt/rocm/bin/hipcc $F -x hip -c $C/myyuv_hip.cpp -o $out/myyuv_hip.o & objs="$objs $out/myyuv_hip.o"
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libmyyuv_hip.so $objs
rm -f $out/*.o
echo built $out
