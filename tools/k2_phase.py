#!/usr/bin/env python3
"""Diagnostic: K2's per-wave window phases (stamp build,
`tools/build_variant.sh stamps -DMYYUV_STAMPS`; k_huff_encode.hip g_k2_win):
prologue (tiles, classification, sort), runs' fetch + coefficient load +
build, runs' emission and overflow lists, and the last fetch + epilogue, one
24-frame launch group of the bench frame compressed alone:
  MYYUV_HIP_LIB=build_var/stamps/libmyyuv_hip.so python3 tools/k2_phase.py [frames]"""
import ctypes
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'yuv-manipulations-2_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402
from oracle import oracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 24
g = myyuv_file.YUVFile.load(os.path.join(R, 'tests', 'golden', 'chef-with-trumpet-big-DCT-50.myyuv'))
w, h = g.width, g.height
raw = O.decompress(g.data, w, h, tuple(g.params))
q = (50, 50, 50)
c = myyuv_hip.Codec(0)
L = myyuv_hip.load()
dev = torch.device('cuda', 0)
st = torch.cuda.Stream(dev)
sp = st.cuda_stream
cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
d_in = torch.frombuffer(bytearray(raw * B), dtype=torch.uint8).to(dev)
d_pay = torch.empty(B * cap, dtype=torch.uint8, device=dev)
d_sz = torch.zeros(B, dtype=torch.int32, device=dev)
c.reserve_batch(w, h, B)
for _ in range(3):
    c.compress_batch_device(d_in.data_ptr(), B, w, h, q, d_pay.data_ptr(), cap, d_sz.data_ptr(), sp)
c.sync_status(sp)
NW = 65536
buf = (ctypes.c_uint32 * (NW * 8))()
L.myyuv_debug_k2_win(buf, NW)
c.profile(True, kernels=["huff_encode"])
c.compress_batch_device(d_in.data_ptr(), B, w, h, q, d_pay.data_ptr(), cap, d_sz.data_ptr(), sp)
c.sync_status(sp)
kms, kn = c.kernel_stats()["huff_encode"]
rc = L.myyuv_debug_k2_win(buf, NW)
a = np.frombuffer(buf, np.uint32).reshape(NW, 8).astype(np.float64)
a = a[a[:, 7] > 0]
names = {6: "tiles+block words", 5: "classify", 0: "scan+sort+barriers", 1: "fetch+load+build", 2: "emit+lists", 4: "last fetch+epilogue"}
tot = a[:, [0, 1, 2, 4, 5, 6]].sum()
print(f"rc={rc} K2 {kms / kn * 1e3:.1f} us per {B}-frame launch; waves stamped {len(a)} (of the first {NW}), "
      f"runs/wave {a[:, 3].mean():.2f}")
for i, nm in names.items():
    print(f"  {nm:20s} {a[:, i].mean():9.0f} cycles/wave (p90 {np.percentile(a[:, i], 90):8.0f})  {a[:, i].sum() / tot:6.1%}")
print(f"  total                {a[:, [0, 1, 2, 4, 5, 6]].sum(1).mean():9.0f} cycles/wave")
