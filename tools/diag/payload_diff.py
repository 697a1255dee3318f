"""Diagnostic (CPU): compare two payloads of the same frame block by block
(layout: u32 plane sizes x 3, then per plane u32 blocks, u32 content bytes,
the u8 chunk sizes, the chunks) and describe the differing blocks with the
oracle's decode of the first payload's chunk (message length, distinct
symbols, nonzeros):  python3 tools/diag/payload_diff.py a.bin b.bin"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


# zig-zag order: natural index of zig-zag position i
ZZ = np.array(sorted(range(64), key=lambda n: (n // 8 + n % 8, (n // 8) if (n // 8 + n % 8) % 2 else (n % 8))))


def planes(p):
    off, out = 12, []
    for _ in range(3):
        n, content = struct.unpack_from("<II", p, off)
        sizes = np.frombuffer(p, np.uint8, n, off + 8)
        starts = np.concatenate([[0], np.cumsum(sizes, dtype=np.int64)]) + off + 8 + n
        out.append((sizes, starts))
        off += 8 + n + content
    return out


a, b = (open(x, "rb").read() for x in sys.argv[1:3])
O.lib()
ndiff = 0
for pl, ((sa, oa), (sb, ob)) in enumerate(zip(planes(a), planes(b))):
    for k in range(len(sa)):
        ca, cb = a[oa[k]:oa[k + 1]], b[ob[k]:ob[k + 1]]
        if ca == cb:
            continue
        ndiff += 1
        if ndiff <= 25:
            coef = np.asarray(O.huff_decode_block(ca), np.int16).reshape(64)
            msg = coef[ZZ]
            nz = np.nonzero(msg)[0]
            m = nz[-1] + 1 if len(nz) else 1
            print(f"plane {pl} block {k}: sizes {len(ca)} / {len(cb)}, msz {m}, distinct {len(set(msg[:m].tolist()))}, "
                  f"nnz {len(nz)}, tile {k // 256} pos {k % 256}")
            print("   a", ca.hex())
            print("   b", cb.hex())
print("differing blocks:", ndiff)

# where the second payload's differing chunks decode to: the same block's
# coefficients (a different code for the same message) or another block's
if ndiff:
    pa, pb = planes(a), planes(b)
    for pl in range(3):
        (sa, oa), (sb, ob) = pa[pl], pb[pl]
        coefs = None
        for k in range(len(sa)):
            ca, cb = a[oa[k]:oa[k + 1]], b[ob[k]:ob[k + 1]]
            if ca == cb:
                continue
            if coefs is None:  # every block of the plane, decoded from the first payload
                coefs = {bytes(a[oa[j]:oa[j + 1]]): j for j in range(len(sa))}
                dec = [np.asarray(O.huff_decode_block(a[oa[j]:oa[j + 1]]), np.int16).tobytes() for j in range(len(sa))]
                where = {}
                for j, d in enumerate(dec):
                    where.setdefault(d, []).append(j)
            try:
                db = np.asarray(O.huff_decode_block(cb), np.int16).tobytes()
            except Exception as e:  # noqa: BLE001
                print(f"plane {pl} block {k}: b undecodable ({e})")
                continue
            same = db == dec[k]
            print(f"plane {pl} block {k}: b decodes to {'its own message' if same else 'blocks ' + str(where.get(db, [])[:6])}")
