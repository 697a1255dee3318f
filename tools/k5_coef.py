#!/usr/bin/env python3
"""Diagnostic: decode chef-big q50 on the GPU (MYYUV_HIP_LIB build), dump the
coefficient image (myyuv_debug_coef) and compare per block with the oracle's
Huffman decode of each chunk; print the differing positions."""
import ctypes
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
ZZ = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
      20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58,
      59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]


def main():
    import myyuv_file
    import myyuv_hip
    from oracle import oracle as O
    g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv"))
    w, h, q = g.width, g.height, tuple(g.params)
    d = g.data
    ps = struct.unpack_from("<3I", d, 0)
    off = 12
    chunks = []
    for p in range(3):
        hn = struct.unpack_from("<I", d, off)[0]
        sizes = d[off + 8:off + 8 + hn]
        pos = off + 8 + hn
        for s in sizes:
            chunks.append(d[pos:pos + s])
            pos += s
        off += ps[p]
    n = len(chunks)
    ref = np.stack([np.asarray(O.huff_decode_block(c), np.int16).reshape(64) for c in chunks])
    codec = myyuv_hip.Codec(0)
    L = myyuv_hip.load()
    L.myyuv_debug_coef.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    for it in range(2):
        codec.decompress(d, w, h, q)
        got = np.empty((n, 64), np.int16)
        rc = L.myyuv_debug_coef(codec._h, got.ctypes.data, n)
        assert rc == 0, rc
        bad = np.nonzero((got != ref).any(1))[0]
        print(f"iter {it}: {len(bad)} bad blocks")
        for b in bad[:12]:
            zpos = [j for j in range(64) if got[b, ZZ[j]] != ref[b, ZZ[j]]]
            nsym = max([j + 1 for j in range(64) if ref[b, ZZ[j]] != 0] or [1])
            print(f"  block {b} lane {b % 64} size {len(chunks[b])} nsym~{nsym} bad scan pos {zpos[:10]}"
                  f" got {[int(got[b, ZZ[j]]) for j in zpos[:6]]} exp {[int(ref[b, ZZ[j]]) for j in zpos[:6]]}")
    codec.close()


if __name__ == "__main__":
    main()
