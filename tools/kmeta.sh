#!/bin/bash
# Register / LDS / scratch usage per kernel of a built libmyyuv_hip.so (from
# the gfx950 code object's metadata): tools/kmeta.sh [lib]
lib=${1:-$(dirname $0)/../yuv-manipulations-2_amd/libmyyuv_hip.so}
L=/opt/rocm/lib/llvm/bin
d=$(mktemp -d)
$L/llvm-objcopy -O binary --only-section=.hip_fatbin "$lib" $d/fat.bin
$L/clang-offload-bundler --unbundle --type=o --input=$d/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/k.co
$L/llvm-readelf --notes $d/k.co | grep -E "\.name:|\.vgpr_count:|\.agpr_count|\.sgpr_count:|group_segment_fixed_size|private_segment_fixed_size|vgpr_spill_count" | grep -v "\.name:.*\(\.kd\|args\)" | paste - - - - - - - 2>/dev/null | sed 's/  */ /g'
rm -rf $d
