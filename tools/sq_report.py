#!/usr/bin/env python3
"""Summarise tools/sq_counters.sh output: per kernel, the mean of each counter
per launch, and derived ratios (VALU issue share, waits, IPC)."""
import collections
import csv
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def kname(n):
    """Short kernel name: no namespace, return type or template arguments (k_huff_encode<8u> -> huff_encode)."""
    return re.sub(r"<[^>]*>$", "", n.split("(")[0].replace("void ", "").replace("myyuv_gpu::k_", ""))

def main(tag):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(ROOT, "gpurun_out", f"sq_{tag}", "g*", "run_counter_collection.csv")):
        per = collections.defaultdict(float)
        with open(path) as f:
            for r in csv.DictReader(f):
                k = kname(r["Kernel_Name"])
                per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            vals[k][c].append(v)
    for k in sorted(vals):
        d = {c: sum(v) / len(v) for c, v in vals[k].items()}
        print(f"== {k}")
        for c in sorted(d):
            print(f"   {c:22s} {d[c]:16.0f}")
        w = d.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                if c in d:
                    print(f"   {c + '/wave':22s} {d[c] / w:16.1f}")
        if "SQ_WAVE_CYCLES" in d and "SQ_BUSY_CYCLES" in d:
            print(f"   waves resident (avg)   {d['SQ_WAVE_CYCLES'] / max(1, d['SQ_BUSY_CYCLES']):16.2f}")
        if "SQ_ACTIVE_INST_VALU" in d and "SQ_WAVE_CYCLES" in d:
            print(f"   valu-active/wave-cyc   {d['SQ_ACTIVE_INST_VALU'] / d['SQ_WAVE_CYCLES']:16.3f}")
        if "SQ_WAIT_INST_ANY" in d and "SQ_WAVE_CYCLES" in d:
            print(f"   wait-inst/wave-cyc     {d['SQ_WAIT_INST_ANY'] / d['SQ_WAVE_CYCLES']:16.3f}")
        if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d:
            print(f"   wait-any/wave-cyc      {d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES']:16.3f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "x")
