"""PCIe-inclusive rate of the host-buffer API: the 4032x3008 q50
frame through myyuv_gpu_dct_compress + myyuv_gpu_dct_decompress (H2D copy,
kernels, D2H copy, one sync per call; pageable numpy buffers), and through
the batch compress entry point.  MP = W*H luma pixels; time = t_compress +
t_decompress.  Not the bench's `value` (HBM-resident)."""
import os
import statistics
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "yuv-manipulations-2_amd")]
import torch  # noqa: E402,F401  (one HIP runtime with the library)
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402

g = myyuv_file.YUVFile.load(os.path.join(R, "tests/golden/chef-with-trumpet-big-DCT-50.myyuv"))
w, h, q = g.width, g.height, tuple(g.params)
c = myyuv_hip.Codec(0)
raw = c.decompress(g.data, w, h, q)
mp = w * h / 1e6
tc, td = [], []
for i in range(25):
    t0 = time.perf_counter()
    pay = c.compress(raw, w, h, q)
    t1 = time.perf_counter()
    out = c.decompress(pay, w, h, q)
    t2 = time.perf_counter()
    if i >= 5:
        tc.append(t1 - t0)
        td.append(t2 - t1)
assert len(out) == len(raw)  # (bytes checked by the tests; here only timed)
mc, md = statistics.median(tc), statistics.median(td)
print(f"single frame: compress {mc * 1e3:.2f} ms, decompress {md * 1e3:.2f} ms, {mp / (mc + md):.1f} MP/s", flush=True)
B = 12
frames = [raw] * B
tb = []
for i in range(8):
    t0 = time.perf_counter()
    pays = c.compress_batch(frames, w, h, q)
    tb.append(time.perf_counter() - t0)
assert all(p == pay for p in pays)
mb = statistics.median(tb[2:])
print(f"batch of {B}: compress {mb * 1e3:.2f} ms = {B * mp / mb:.1f} MP/s (compress only)", flush=True)
