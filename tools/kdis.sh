#!/bin/bash
# Disassembles the gfx950 code object of a built libmyyuv_hip.so to stdout:
#   tools/kdis.sh [lib]
lib=${1:-$(dirname $0)/../yuv-manipulations-2_amd/libmyyuv_hip.so}
L=/opt/rocm/lib/llvm/bin
d=$(mktemp -d)
$L/llvm-objcopy -O binary --only-section=.hip_fatbin "$lib" $d/fat.bin
$L/clang-offload-bundler --unbundle --type=o --input=$d/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/k.co
$L/llvm-objdump -d --no-show-raw-insn $d/k.co
rm -rf $d
