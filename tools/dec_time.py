"""Diagnostic: the decoder's time per 6-frame launch alone on the GPU (kernel
events), with no output check (for the MYYUV_K5_EXP ablation builds)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "yuv-manipulations-2_amd")]
import torch  # noqa: E402
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402

B = 6
g = myyuv_file.YUVFile.load(os.path.join(R, "tests/golden/chef-with-trumpet-big-DCT-50.myyuv"))
w, h, q = g.width, g.height, tuple(g.params)
c = myyuv_hip.Codec(0)
raw = c.decompress(g.data, w, h, q)
fb = w * h * 3 // 2
cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
dev = torch.device("cuda", 0)
d_in = torch.frombuffer(bytearray(raw * B), dtype=torch.uint8).to(dev)
d_pay = torch.empty(B * cap, dtype=torch.uint8, device=dev)
d_sz = torch.zeros(B, dtype=torch.int32, device=dev)
d_out = torch.empty(B * fb, dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
c.compress_batch_device(d_in.data_ptr(), B, w, h, q, d_pay.data_ptr(), cap, d_sz.data_ptr(), s)
for _ in range(3):
    c.decompress_batch_device(d_pay.data_ptr(), d_sz.data_ptr(), cap, B, w, h, q, d_out.data_ptr(), s)
torch.cuda.synchronize()
c.profile(True)
for _ in range(20):
    c.decompress_batch_device(d_pay.data_ptr(), d_sz.data_ptr(), cap, B, w, h, q, d_out.data_ptr(), s)
torch.cuda.synchronize()
print({k: round(ms / n * 1e3, 1) for k, (ms, n) in c.kernel_stats().items() if n})
c.profile(False)
