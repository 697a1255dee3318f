"""Diagnostic (CPU, oracle only): transform steps of the fused decoder's unit
forms on the bench frame.  The decoder compacts each 64-block group's blocks
that are not DC-only into units; a unit's stage-1 step k is needed when
coefficient row k is nonzero in any of its blocks, stage-2 step k when column
k is (the first A steps of each stage run without the test).  Prints units
and steps per group for 16-, 8- and 4-block units.

  python tools/diag/idct_units.py [quality]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
from oracle import oracle  # noqa: E402
import myyuv_file  # noqa: E402


def plane_blocks(q):
    g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests/golden/chef-with-trumpet-big-DCT-50.myyuv"))
    w, h = g.width, g.height
    raw = np.frombuffer(oracle.decompress(g.data, w, h, tuple(g.params)), np.uint8)
    planes = [(raw[:w * h].reshape(h, w), 0), (raw[w * h:w * h * 5 // 4].reshape(h // 2, w // 2), 1),
              (raw[w * h * 5 // 4:].reshape(h // 2, w // 2), 1)]
    for pl, chroma in planes:
        Q = oracle.qtable(q, chroma)
        H, W = pl.shape
        blks = pl.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        yield np.stack([oracle.fdct_block(np.ascontiguousarray(b), Q) for b in blks]).reshape(-1, 8, 8)


def main():
    q = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    groups = []
    for C in plane_blocks(q):
        n = len(C) // 64 * 64  # (whole groups of each plane)
        groups.append(C[:n].reshape(-1, 64, 8, 8) != 0)
    nz = np.concatenate(groups)
    rest = nz.reshape(len(nz), 64, 64)[:, :, 1:].any(axis=2)  # not DC-only
    G = len(nz)
    for U, A in ((16, 3), (8, 2), (4, 1)):
        s1 = s2 = units = 0
        for gi in range(G):
            B = nz[gi, np.nonzero(rest[gi])[0]]
            for u0 in range(0, len(B), U):
                b = B[u0:u0 + U]
                r, c = b.any(axis=(0, 2)), b.any(axis=(0, 1))
                r[:A] = True
                c[:A] = True
                s1 += int(r.sum())
                s2 += int(c.sum())
                units += 1
        print(f"q{q} {U:2d}-block units (first {A} steps always): {units / G:.2f} units per group, "
              f"stage-1 steps {s1 / G:.2f}, stage-2 steps {s2 / G:.2f} per group")


if __name__ == "__main__":
    main()
