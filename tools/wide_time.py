"""Diagnostic: the overflow pass k_huff_encode_wide on the bench's 6-frame
launch group (stamp build, `make -C yuv-manipulations-2_amd stamps`): its
per-stage cycles summed over waves and the slowest wave's, against the
kernel's duration."""
import ctypes
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'yuv-manipulations-2_amd')]
os.environ.setdefault('MYYUV_HIP_LIB', os.path.join(R, 'yuv-manipulations-2_amd/build/stamps/libmyyuv_hip.so'))
import torch  # noqa: E402
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402

B = 6
names = ['', 'symbols', 'map', 'heap+len', 'canon', 'emit']
g = myyuv_file.YUVFile.load(os.path.join(R, 'tests/golden/chef-with-trumpet-big-DCT-50.myyuv'))
w, h, q = g.width, g.height, tuple(g.params)
c = myyuv_hip.Codec(0)
L = myyuv_hip.load()
raw = c.decompress(g.data, w, h, q)
cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
dev = torch.device('cuda', 0)
d_in = torch.frombuffer(bytearray(raw * B), dtype=torch.uint8).to(dev)
d_pay = torch.empty(B * cap, dtype=torch.uint8, device=dev)
d_sz = torch.zeros(B, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
for _ in range(3):
    c.compress_batch_device(d_in.data_ptr(), B, w, h, q, d_pay.data_ptr(), cap, d_sz.data_ptr(), s)
torch.cuda.synchronize()
st0 = (ctypes.c_ulonglong * 40)()
L.myyuv_debug_k2_stamps(st0)
iters = 10
c.profile(True)
for _ in range(iters):
    c.compress_batch_device(d_in.data_ptr(), B, w, h, q, d_pay.data_ptr(), cap, d_sz.data_ptr(), s)
torch.cuda.synchronize()
st = (ctypes.c_ulonglong * 40)()
L.myyuv_debug_k2_stamps(st)
ks = c.kernel_stats()
c.profile(False)
us = {k: round(ms / n * 1e3, 1) for k, (ms, n) in ks.items() if n}
print('kernel us per launch', us)
for k in range(1, 6):
    tot = (st[k + 8] - st0[k + 8]) / iters
    print(f"  {names[k]:9s} summed over waves per launch {tot / 1e6:8.2f} Mcycles, slowest wave {st[k + 16]} cycles")
