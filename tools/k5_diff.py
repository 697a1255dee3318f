#!/usr/bin/env python3
"""Diagnostic: decode chef-big q50 golden on the GPU (MYYUV_HIP_LIB build),
compare with the oracle per 8x8 block, print the mismatching blocks with
their lane, chunk size and symbol count."""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]


def main():
    import myyuv_file
    import myyuv_hip
    from oracle import oracle as O
    g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv"))
    w, h, q = g.width, g.height, tuple(g.params)
    ref = np.frombuffer(O.decompress(g.data, w, h, q), np.uint8)
    codec = myyuv_hip.Codec(0)
    bad_total = 0
    for it in range(3):
        got = np.frombuffer(codec.decompress(g.data, w, h, q), np.uint8)
        planes = [(0, w, h), (w * h, w // 2, h // 2), (w * h * 5 // 4, w // 2, h // 2)]
        bad = []
        gbase = 0
        for p, (off, pw, ph) in enumerate(planes):
            a = ref[off:off + pw * ph].reshape(ph // 8, 8, pw // 8, 8)
            b = got[off:off + pw * ph].reshape(ph // 8, 8, pw // 8, 8)
            d = (a != b).any(axis=(1, 3))
            for by, bx in zip(*np.nonzero(d)):
                k = by * (pw // 8) + bx
                bad.append((p, int(k), int(gbase + k)))
            gbase += (pw // 8) * (ph // 8)
        bad_total += len(bad)
        print(f"iter {it}: {len(bad)} bad blocks")
        # chunk sizes of the bad blocks
        d = g.data
        off = 12
        sizes_all = []
        ps = struct.unpack_from("<3I", d, 0)
        for p in range(3):
            hn = struct.unpack_from("<I", d, off)[0]
            sizes_all.append(list(d[off + 8:off + 8 + hn]))
            off += ps[p]
        for p, k, gg in bad[:20]:
            print(f"  plane {p} block {k} (global {gg}, lane {gg % 64 if p == 0 else (k % 64)}) size {sizes_all[p][k]}")
    codec.close()
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
