#!/usr/bin/env python3
"""Audit of K2's cross-lane operations in the gfx950 ISA (round 4, VERDICT r3
item 3: the round-3 DPP wrong-output episode, profiles/r3h_dpp_bisect.txt).

Compiles csrc/k_huff_encode.hip for gfx950 to assembly (device only, the
product's flags) twice:
  shipped  the source as it is (ds_bpermute wave max / scans);
  dpp      wave_max_ln replaced by the round-3 DPP form as the commit message
           describes it (row_shr 1/2/4/8, row_bcast 15/31, readlane 63): the
           round-3 source itself was never committed, so this is a
           reconstruction;
and reports, inside k_huff_encode's run loop, every cross-lane instruction
(ds_bpermute, DPP, readlane) with the net count of EXEC narrowings still open
since the loop header (0 = the loop's own EXEC, the full wave: the loop's
control is scalar) and, for DPP, the wait states between the last VALU write
of its source register and the DPP read (the gfx9 VALU -> DPP hazard needs 2).
Usage: python3 tools/diag/k2_crosslane_audit.py > profiles/<tag>_k2_crosslane_audit.txt
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "yuv-manipulations-2_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
         "-I" + CSRC, "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S"]
SHIPPED_MAX = '''__device__ __forceinline__ int wave_max_ln(int v, uint32_t ln) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v = max(v, __builtin_amdgcn_ds_bpermute((int)((ln ^ (uint32_t)d) << 2), v));
  return v;
}'''
DPP_MAX = '''__device__ __forceinline__ int wave_max_ln(int v, uint32_t ln) {
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false));
  return __builtin_amdgcn_readlane(v, 63);
}'''


def compile_k2(src_text, d):
    src = os.path.join(d, "k_huff_encode.hip")
    with open(src, "w") as f:
        f.write(src_text)
    out = os.path.join(d, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-I" + CSRC, src, "-o", out], check=True,
                   stderr=subprocess.DEVNULL)
    lines = open(out).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN9myyuv_gpu13k_huff_encodeE.*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def audit(name, L):
    hdr = next(i for i, l in enumerate(L) if "Inner Loop Header" in l and "run" not in l)
    print(f"== {name}: k_huff_encode, {len(L)} lines, run loop header at line {hdr + 1}")
    depth = 0
    lastw = {}  # vgpr -> index of the last VALU write
    waits = 0
    for i in range(hdr, len(L)):
        l = L[i].strip()
        if not l or l.startswith(";") or l.startswith("."):
            continue
        if re.match(r"s_and_saveexec_b64|s_andn2_saveexec_b64|s_and_b64 exec, exec|s_xor_b64 exec", l):
            depth += 1
        elif re.match(r"s_or_b64 exec, exec|s_mov_b64 exec,", l):
            depth -= 1
        m = re.match(r"s_nop (\d+)", l)
        cross = re.match(r"(ds_bpermute_b32|v_\w+_dpp|v_readlane_b32|v_readfirstlane_b32)\s+(\S+)", l)
        if cross:
            op = cross.group(1)
            note = ""
            if "dpp" in op:
                srcs = re.findall(r"v(\d+)", l.split(",", 1)[1].split(" row_")[0])
                src = srcs[0] if srcs else None
                ws = None
                if src in lastw:
                    ws = sum(1 if not re.match(r"s_nop", L[k].strip()) else int(re.match(r"s_nop (\d+)", L[k].strip()).group(1)) + 1
                             for k in range(lastw[src] + 1, i)
                             if L[k].strip() and not L[k].strip().startswith((";", ".")))
                note = f"  src v{src}: {ws} wait states since its last VALU write" if ws is not None else ""
            print(f"  line {i + 1:6d}  exec-depth {depth:+d}  {l[:90]}{note}")
        if l.startswith("v_"):
            d0 = re.match(r"v_\w+\s+v\[?(\d+)", l)
            if d0:
                lastw[d0.group(1)] = i
        if l.startswith("s_endpgm"):
            break


def main():
    text = open(os.path.join(CSRC, "k_huff_encode.hip")).read()
    assert SHIPPED_MAX in text, "wave_max_ln changed: update the audit"
    with tempfile.TemporaryDirectory() as d:
        audit("shipped (ds_bpermute)", compile_k2(text, d))
        audit("reconstructed round-3 DPP max", compile_k2(text.replace(SHIPPED_MAX, DPP_MAX), d))


if __name__ == "__main__":
    sys.exit(main())
