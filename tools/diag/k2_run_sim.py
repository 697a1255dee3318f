#!/usr/bin/env python3
"""Diagnostic: K2's window sort simulated on the bench frame (chef-big q50,
oracle transform): blocks classed as class_of does (codec_common.hpp), sorted
per 2,048-block window by key (class, message-length bucket), cut into runs
of 64; prints, per length-bucket scheme, the sum over runs of the longest
message among the blocks K2 builds (its per-position loops run that long).

  python3 tools/diag/k2_run_sim.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
import myyuv_file  # noqa: E402
from oracle import oracle as O  # noqa: E402

ZZ = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,
               7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
               39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
OVF_NUB = 16


def blocks():
    g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv"))
    w, h = g.width, g.height
    raw = np.frombuffer(O.decompress(g.data, w, h, tuple(g.params)), np.uint8)
    planes = [(raw[:w * h].reshape(h, w), 0), (raw[w * h:w * h * 5 // 4].reshape(h // 2, w // 2), 1),
              (raw[w * h * 5 // 4:].reshape(h // 2, w // 2), 1)]
    rows = []
    for P, ch in planes:
        Q = O.qtable(50, ch)
        hh, ww = P.shape
        B = P[:hh // 8 * 8, :ww // 8 * 8].reshape(hh // 8, 8, ww // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        for b in B:
            c = np.asarray(O.fdct_block(b, Q)).reshape(64)[ZZ]
            nz = np.nonzero(c)[0]
            rows.append((nz[-1] + 1 if len(nz) else 0, len(nz)))
    return np.array(rows)


def cost(m, cls, bounds):
    tot = 0
    for s in range(0, len(m), 2048):
        mm, cc = m[s:s + 2048], cls[s:s + 2048]
        b = np.searchsorted(np.array(bounds), mm, side="left")
        key = np.where(cc == 0, 0, np.where(cc == 4, 100, 1 + (cc - 1) * 10 + b))
        o = np.argsort(key, kind="stable")
        ms, cs = mm[o], cc[o]
        for r in range(0, len(ms), 64):
            bl = (cs[r:r + 64] >= 1) & (cs[r:r + 64] <= 3)
            if bl.any():
                tot += int(ms[r:r + 64][bl].max())
    return tot


def main():
    d = blocks()
    m, nnz = d[:, 0], d[:, 1]
    nub = nnz + (m > nnz)
    cls = np.where(m <= 1, 0, np.where(nub <= 4, 1, np.where(nub <= 8, 2, np.where(nub < OVF_NUB, 3, 4))))
    for bounds in ([8, 16], [6, 12, 20], [8, 12, 16], [8, 16, 24]):
        print("buckets <=", bounds, "sum of run maxima", cost(m, cls, bounds))


if __name__ == "__main__":
    main()
