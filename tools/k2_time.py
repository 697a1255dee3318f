"""Diagnostic: K2 per-stage cycles (stamp build, `make -C yuv-manipulations-2_amd stamps`)
on the bench frame: fast pass summed per wave, wide pass mean and max per wave."""
import ctypes
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'yuv-manipulations-2_amd')]
os.environ.setdefault('MYYUV_HIP_LIB', os.path.join(R, 'yuv-manipulations-2_amd/build/stamps/libmyyuv_hip.so'))
import torch  # noqa: E402
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402
import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

c = myyuv_hip.Codec(0)
L = myyuv_hip.load()
names = ['', 'symbols', 'map', 'heap+len', 'canon', 'emit']


def run(raw, w, h, q, label, iters=10):
    d_in = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    cap = myyuv_hip.payload_bound(w, h)
    d_pay = torch.empty(cap, dtype=torch.uint8, device='cuda')
    d_size = torch.zeros(1, dtype=torch.int32, device='cuda')
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        c.compress_device(d_in.data_ptr(), w, h, (q, q, q), d_pay.data_ptr(), cap, d_size.data_ptr(), sp)
    c.sync_status(sp)
    st = (ctypes.c_ulonglong * 40)()
    L.myyuv_debug_k2_stamps(st)
    c.profile(True)
    for _ in range(iters):
        c.compress_device(d_in.data_ptr(), w, h, (q, q, q), d_pay.data_ptr(), cap, d_size.data_ptr(), sp)
    c.sync_status(sp)
    L.myyuv_debug_k2_stamps(st)
    ks = c.kernel_stats()
    c.profile(False)
    import numpy as np
    fs = np.zeros(8192 * 8, np.uint32)
    L.myyuv_debug_k2_fstamps(fs.ctypes.data_as(ctypes.c_void_p), 8192)
    fs8 = fs.reshape(-1, 8)
    cls_names = {0: 'single', 1: 'r4', 2: 'r8', 3: 'r8x'}
    used = fs8[:, 7] > 0
    for cl in (0, 1, 2, 3):
        sel = used & ((fs8[:, 0] & 0xFF) == cl)
        if sel.any():
            st = fs8[sel]
            stages = {names[k]: int(st[:, k].mean()) for k in range(1, 5)}
            print(f"   class {cls_names[cl]:6s}: {sel.sum():5d} waves, wave msz mean {(st[:, 0] >> 8).mean():5.1f}, "
                  f"total cycles mean {st[:, 7].mean():8.0f}, build stages {stages}", flush=True)
    fs = fs8[:, 1:6]
    fs = fs[fs.sum(1) > 0]
    fast = {names[k + 1]: int(fs[:, k].mean()) for k in range(5)}
    fast_max = {names[k + 1]: int(fs[:, k].max()) for k in range(5)}
    wide_sum = {names[k]: st[k + 8] for k in range(1, 6)}
    wide_max = {names[k]: st[k + 16] for k in range(1, 6)}
    us = lambda k: round(ks[k][0] / max(ks[k][1], 1) * 1e3, 1)
    print(f"{label}: fast {us('huff_encode')} us, wide {us('huff_encode_wide')} us", flush=True)
    print("   fast cycles/wave mean", fast, flush=True)
    print("   fast cycles/wave max", fast_max, "total mean", int(fs.sum(1).mean()), "max", int(fs.sum(1).max()), flush=True)
    print("   wide cycles summed", wide_sum, flush=True)
    print("   wide cycles max/wave", wide_max, flush=True)
    wn = ['', 'load', 'distinct', 'map', 'heap', 'len', 'canon', 'emit']
    import numpy as np
    ws = np.zeros(65536 * 8, np.uint32)
    L.myyuv_debug_k2_wstamps(ws.ctypes.data_as(ctypes.c_void_p), 65536)
    ws = ws.reshape(-1, 8)[:, 1:]
    used = ws.sum(1) > 0
    if used.any():
        ws = ws[used]
        tot = ws.sum(1)
        print(f"   wave encoder {us('huff_encode_wave')} us; {used.sum()} blocks; cycles per block: "
              f"mean {tot.mean():.0f} p50 {np.median(tot):.0f} p99 {np.percentile(tot, 99):.0f} max {tot.max()}", flush=True)
        print("   mean per phase", {wn[k + 1]: int(ws[:, k].mean()) for k in range(7)}, flush=True)
        print("   max per phase", {wn[k + 1]: int(ws[:, k].max()) for k in range(7)}, flush=True)


g = myyuv_file.YUVFile.load(os.path.join(R, 'tests/golden/chef-with-trumpet-big-DCT-50.myyuv'))
w, h = g.width, g.height
raw = O.decompress(g.data, w, h, tuple(g.params))
run(raw, w, h, 50, 'chef-big q50')
run(synth.noise_frame(2048, 1024).tobytes(), 2048, 1024, 50, 'noise q50')
