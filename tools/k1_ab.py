#!/usr/bin/env python3
"""Diagnostic: per-kernel times of one 7-frame (K1AB_B) launch group (chef-big q50,
batch entry points, kernels alone on the GPU, HIP events, no correctness
checks) for the library builds given as arguments (directories holding a
libmyyuv_hip.so, "default", or VAR=value: the in-tree build with that
environment), three alternating rounds:
  python3 tools/k1_ab.py default build_var/x ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "yuv-manipulations-2_amd")

CHILD = r'''
import os, sys
sys.path[:0] = [%r, %r]
import torch, myyuv_file, myyuv_hip
from oracle import oracle as O
g = myyuv_file.YUVFile.load(os.path.join(%r, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv"))
w, h, B = g.width, g.height, int(os.environ.get("K1AB_B", "7"))
raw = O.decompress(g.data, w, h, tuple(g.params))
dev = torch.device("cuda", 0)
c = myyuv_hip.Codec(0)
st = torch.cuda.Stream(dev); sp = st.cuda_stream
fb = w * h * 3 // 2
cap = (myyuv_hip.payload_bound(w, h) + 3) & ~3
d_in = torch.frombuffer(bytearray(raw * B), dtype=torch.uint8).to(dev)
d_pay = torch.empty(B * cap, dtype=torch.uint8, device=dev)
d_sz = torch.zeros(B, dtype=torch.int32, device=dev)
d_out = torch.empty(B * fb, dtype=torch.uint8, device=dev)
st.wait_stream(torch.cuda.current_stream(dev))
c.reserve_batch(w, h, B)
q = (50, 50, 50)
for it in range(2):
    c.profile(it == 1)
    for _ in range(20 if it else 3):
        c.compress_batch_device(d_in.data_ptr(), B, w, h, q, d_pay.data_ptr(), cap, d_sz.data_ptr(), sp)
        c.decompress_batch_device(d_pay.data_ptr(), d_sz.data_ptr(), cap, B, w, h, q, d_out.data_ptr(), sp)
    c.sync_status(sp)
print(" ".join(f"{k}={ms / n * 1e3:.1f}" for k, (ms, n) in c.kernel_stats().items() if n))
'''


def main():
    libs = sys.argv[1:] or ["default"]
    for rnd in range(3):
        for lib in libs:
            env = dict(os.environ)
            if "=" in lib:
                k, v = lib.split("=", 1)
                env[k] = v
            elif lib != "default":
                env["MYYUV_HIP_LIB"] = os.path.join(ROOT, lib, "libmyyuv_hip.so")
            r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, PKG, ROOT)], env=env, capture_output=True,
                               text=True, timeout=300)
            print(lib, r.stdout.strip() or r.stderr[-300:], flush=True)


if __name__ == "__main__":
    main()
