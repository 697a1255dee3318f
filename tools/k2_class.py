"""Diagnostic: per-wave class, max msz and encode cycles of K2's fast pass
(stamp build), chef-big q50."""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'yuv-manipulations-2_amd')]
os.environ.setdefault('MYYUV_HIP_LIB', os.path.join(R, 'yuv-manipulations-2_amd/build/stamps/libmyyuv_hip.so'))
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402
from oracle import oracle as O  # noqa: E402

g = myyuv_file.YUVFile.load(os.path.join(R, 'tests/golden/chef-with-trumpet-big-DCT-50.myyuv'))
w, h = g.width, g.height
raw = O.decompress(g.data, w, h, tuple(g.params))
c = myyuv_hip.Codec(0)
L = myyuv_hip.load()
for _ in range(3):
    c.compress(raw, w, h, (50, 50, 50))
fs = np.zeros(8192 * 8, np.uint32)
L.myyuv_debug_k2_fstamps(fs.ctypes.data_as(ctypes.c_void_p), 8192)
fs = fs.reshape(-1, 8)
used = fs[:, 7] > 0
fs = fs[used]
cls = fs[:, 0] & 0xFF
wmsz = fs[:, 0] >> 8
tot = fs[:, 7]
names = ['single', 'r4', 'r8', 'r8x']
print(f"waves {len(fs)}; encode cycles: max {tot.max()}")
for k in range(4):
    s = cls == k
    if s.any():
        ph = {f'p{j}': int(fs[s, j].mean()) for j in range(1, 6)}
        print(f"  {names[k]:6s} waves {s.sum():5d}  wmsz mean {wmsz[s].mean():5.1f}  cycles mean {tot[s].mean():8.0f} max {tot[s].max():8d}  phases {ph}")
