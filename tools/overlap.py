#!/usr/bin/env python3
"""Diagnostic: concurrency of the bench's timed region from a rocprofv3 kernel
trace (tools/profile.sh -> gpurun_out/prof_<tag>/trace/run_kernel_trace.csv):
per kernel the summed busy time, and over the densest window of codec
launches the time with k kernels running at once (k = 0, 1, 2, ...)."""
import collections
import csv
import re
import sys



def kname(n):
    """Short kernel name: no namespace, return type or template arguments (k_huff_encode<8u> -> huff_encode)."""
    return re.sub(r"<[^>]*>$", "", n.split("(")[0].replace("void ", "").replace("myyuv_gpu::k_", ""))

def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            if "myyuv_gpu::" not in n:
                continue
            k = kname(n)
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    # the timed region: the longest run of launches with gaps < 200 us
    best, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(x[1] for x in cur[-50:]) > 200_000:
            if len(cur) > len(best):
                best = cur
            cur = [r]
        else:
            cur.append(r)
    if len(cur) > len(best):
        best = cur
    t0, t1 = best[0][0], max(r[1] for r in best)
    busy = collections.Counter()
    for s, e, k in best:
        busy[k] += e - s
    ev = sorted([(s, 1) for s, _, _ in best] + [(e, -1) for _, e, _ in best])
    hist = collections.Counter()
    lvl, last = 0, t0
    for t, d in ev:
        hist[lvl] += t - last
        lvl += d
        last = t
    wall = t1 - t0
    print(f"window {wall / 1e3:.1f} us, {len(best)} launches")
    for k, v in busy.most_common():
        print(f"  {k:20s} busy {v / 1e3:9.1f} us  ({v / wall:5.2f} of the window)")
    for lv in sorted(hist):
        print(f"  {lv} running: {hist[lv] / wall:6.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
