#!/bin/bash
# Per-kernel resources of a built libmyyuv_hip.so (gfx950 code object notes):
#   tools/kres.sh [lib] [name-filter]
lib=${1:-$(dirname $0)/../yuv-manipulations-2_amd/libmyyuv_hip.so}
filt=${2:-.}
L=/opt/rocm/lib/llvm/bin
d=$(mktemp -d)
$L/llvm-objcopy -O binary --only-section=.hip_fatbin "$lib" $d/fat.bin
$L/clang-offload-bundler --unbundle --type=o --input=$d/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/k.co
$L/llvm-readelf --notes $d/k.co | python3 -c '
import sys, re
rec = {}
rows = []
for l in sys.stdin:
    m = re.match(r"\s+\.(\w+):\s+(\S+)", l)
    if not m: continue
    k, v = m.groups()
    if k in ("group_segment_fixed_size", "private_segment_fixed_size", "sgpr_count", "vgpr_count", "vgpr_spill_count", "name"):
        rec[k] = v
    if k == "vgpr_spill_count" or (k == "name" and len(rec) == 6):
        pass
    if len(rec) == 6:
        rows.append(rec); rec = {}
for r in rows:
    n = re.sub(r"^_ZN9myyuv_gpu\d+", "", r["name"])[:28]
    if re.search(sys.argv[1], n):
        print("%-28s vgpr %4s spill %3s scratch %4s lds %6s sgpr %s" % (n, r["vgpr_count"], r["vgpr_spill_count"], r["private_segment_fixed_size"], r["group_segment_fixed_size"], r["sgpr_count"]))
' "$filt"
rm -rf $d
