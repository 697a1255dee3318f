"""Generates tests/golden/block_kats.npz: per-block known answers (zig-zag
coefficients -> chunk bytes) over the edge classes of tests/blockgen.py, from
the CPU restatement, which is itself pinned byte-exact to the reference's
golden files and to the reference library (tests/test_oracle.py).
Run from the repo root: python tests/golden/make_kats.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import blockgen  # noqa: E402
from oracle import oracle as O  # noqa: E402

ZZ = np.array(O.lib().oracle_zigzag and [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
              41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
              30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
blocks = blockgen.edge_blocks()
coef = np.stack([b for _, b in blocks]).astype(np.int16)
chunks, sizes = [], []
for b in coef:
    nat = np.zeros(64, np.int16)
    nat[ZZ] = b
    ch = O.huff_encode_block(nat)
    chunks.append(np.frombuffer(ch, np.uint8))
    sizes.append(len(ch))
np.savez_compressed(os.path.join(HERE, "block_kats.npz"), coef_zz=coef,
                    sizes=np.array(sizes, np.uint16), chunks=np.concatenate(chunks))
print(len(coef), "blocks,", sum(sizes), "chunk bytes")
