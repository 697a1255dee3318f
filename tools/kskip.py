"""Diagnostic: each kernel's share of the pipelined bench configuration
(KSKIP_NF streams x KSKIP_B-frame launches, default the bench's 3 x 24,
chef-big q50): throughput with that kernel's launches skipped
(myyuv_debug_skip_kernels; identical frames, so the buffers still hold what
the last real launch wrote)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
import torch  # noqa: E402
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402

NF = int(os.environ.get("KSKIP_NF", "3"))
B = int(os.environ.get("KSKIP_B", "24"))
GROUPS = int(os.environ.get("KSKIP_GROUPS", "30"))
g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests/golden/chef-with-trumpet-big-DCT-50.myyuv"))
w, h = g.width, g.height
L = myyuv_hip.load()
L.myyuv_debug_skip_kernels.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
cs = [myyuv_hip.Codec(0) for _ in range(NF)]
raw = cs[0].decompress(g.data, w, h, tuple(g.params))
dev = torch.device("cuda", 0)
# explicit streams (the null stream's handle 0 means "the context's own stream" to the C ABI)
sts = [torch.cuda.Stream(dev) for _ in range(NF)]
cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
fb = w * h * 3 // 2
d_in = torch.frombuffer(bytearray(raw * B), dtype=torch.uint8).to(dev)
d_out = torch.empty((NF, B * fb), dtype=torch.uint8, device=dev)
d_pay = torch.empty((NF, B * cap), dtype=torch.uint8, device=dev)
d_sz = torch.zeros((NF, B), dtype=torch.int32, device=dev)
for c in cs:
    c.reserve_batch(w, h, B)
q = (50, 50, 50)


def group(j):
    k = j % NF
    sp = sts[k].cuda_stream
    cs[k].compress_batch_device(d_in.data_ptr(), B, w, h, q, d_pay[k].data_ptr(), cap, d_sz[k].data_ptr(), sp)
    cs[k].decompress_batch_device(d_pay[k].data_ptr(), d_sz[k].data_ptr(), cap, B, w, h, q,
                                  d_out[k].data_ptr(), sp)


def run(mask):
    for c in cs:
        L.myyuv_debug_skip_kernels(c._h, mask)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(GROUPS):
        group(j)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    return GROUPS * B * w * h / 1e6 / t


for j in range(6):
    group(j)
torch.cuda.synchronize()
base = max(run(0), run(0))
print(f"all kernels: {base:9.0f} MP/s")
for kid, name in enumerate(myyuv_hip.KERNELS):
    if name in ("parse",):
        continue
    v = max(run(1 << kid), run(1 << kid))
    print(f"skip {name:16s}: {v:9.0f} MP/s  ({(1 / base - 1 / v) * B * w * h / 1e6 * 1e6 / B:7.1f} us/frame)")
base2 = run(0)
# expected: the host-API round trip of the same (already decoded) frame
want = cs[0].decompress(cs[0].compress(raw, w, h, q), w, h, q)
ok = bytes(d_out[0, :fb].cpu().numpy()) == want
print(f"all kernels again: {base2:9.0f} MP/s; output intact: {ok}")
