"""Diagnostic (CPU, oracle only): how many of K6's transform steps the
zero-row / zero-column skip removes on the bench frame.  K6 works on units
of 16 consecutive blocks of a plane; stage 1 step k is needed when coefficient
row k is nonzero in any block of the unit, stage 2 step k when column k is.

  python tools/k6_skip_stats.py [quality]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
from oracle import oracle  # noqa: E402
import myyuv_file  # noqa: E402


def main():
    q = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests/golden/chef-with-trumpet-big-DCT-50.myyuv"))
    w, h = g.width, g.height
    raw = np.frombuffer(oracle.decompress(g.data, w, h, tuple(g.params)), np.uint8)
    planes = [(raw[:w * h].reshape(h, w), 0), (raw[w * h:w * h * 5 // 4].reshape(h // 2, w // 2), 1),
              (raw[w * h * 5 // 4:].reshape(h // 2, w // 2), 1)]
    rows = cols = units = 0
    for pl, chroma in planes:
        Q = oracle.qtable(q, chroma)
        H, W = pl.shape
        blks = pl.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        C = np.stack([oracle.fdct_block(np.ascontiguousarray(b), Q) for b in blks]).reshape(-1, 8, 8)
        n = len(C) - len(C) % 16
        U = C[:n].reshape(-1, 16, 8, 8)  # [unit][block][row][col], natural order
        rows += (U != 0).any(axis=(1, 3)).sum()
        cols += (U != 0).any(axis=(1, 2)).sum()
        units += len(U)
    print(f"q{q}: {units} units; stage-1 steps needed {rows / (units * 8):.3f}, "
          f"stage-2 steps needed {cols / (units * 8):.3f}")


if __name__ == "__main__":
    main()
