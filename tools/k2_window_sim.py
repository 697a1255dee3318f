"""Diagnostic: K2's run composition for a window sort over 1, 2, 4, 8 tiles
(chef-big q50, the bench frame).  Decodes every chunk of the oracle's stream
back to its coefficients, classifies the blocks as K2 does (block_class,
huff_common.hpp), sorts each window's blocks by class, cuts 64-block runs and
counts them by their heaviest class; the cost column weighs each run by the
class's mean wave cycles measured with the stamp build in round 2 (single
4.3k, <= 4 18.4k, <= 8 32.9k, rest 41.1k)."""
import os
import struct
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'yuv-manipulations-2_amd')]
import myyuv_file  # noqa: E402
from oracle import oracle as O  # noqa: E402

ZZ = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
      21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60,
      61, 54, 47, 55, 62, 63]
COST = np.array([4.3, 18.4, 32.9, 41.1])


def blocks():
    g = myyuv_file.YUVFile.load(os.path.join(R, 'tests/golden/chef-with-trumpet-big-DCT-50.myyuv'))
    raw = O.decompress(g.data, g.width, g.height, tuple(g.params))
    p = O.compress(raw, g.width, g.height, (50, 50, 50))
    off, coefs, plane = 12, [], []
    for pl in range(3):
        nb, cs = struct.unpack_from('<2I', p, off)
        off += 8
        sizes = np.frombuffer(p, np.uint8, nb, off)
        off += nb
        o = off
        for s in sizes:
            coefs.append(O.huff_decode_block(p[o:o + int(s)]))
            plane.append(pl)
            o += int(s)
        off += cs
    return np.array(coefs), np.array(plane)


def main():
    B, P = blocks()
    Z = B[:, ZZ]
    nz = Z != 0
    msz = np.where(nz.any(1), 64 - np.argmax(nz[:, ::-1], 1), 0)
    nnz = nz.sum(1)
    nub = nnz + (msz > nnz)
    cls = np.where(msz <= 1, 0, np.where(nub <= 4, 1, np.where(nub <= 8, 2, 3)))
    print(f"blocks {len(B)}; class shares " + " / ".join(f"{(cls == k).mean():.3f}" for k in range(4)))
    tiles = []  # per plane, 256-block tiles (the batch tile order)
    for pl in range(3):
        idx = np.where(P == pl)[0]
        tiles += [idx[t:t + 256] for t in range(0, len(idx), 256)]
    for win in (1, 2, 4, 8):
        runs = np.zeros(4, int)
        for w in range(0, len(tiles), win):
            c = np.sort(np.concatenate([cls[t] for t in tiles[w:w + win]]))
            for r in range(0, len(c), 64):
                runs[c[r:r + 64].max()] += 1
        print(f"window {win} tiles: runs single / <=4 / <=8 / rest = {' / '.join(map(str, runs))}; "
              f"cost {float((runs * COST).sum()):.0f}k wave cycles")


if __name__ == '__main__':
    main()
