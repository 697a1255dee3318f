"""Diagnostic: the pipelined host batches on the big frame, frame by frame
(which calls and which frames differ from the pinned decode, and where)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402


def diff(a, b):
    x = np.frombuffer(a, np.uint8)
    y = np.frombuffer(b, np.uint8)
    if x.size != y.size:
        return f"size {x.size} vs {y.size}"
    d = np.nonzero(x != y)[0]
    if d.size == 0:
        return "equal"
    return f"{d.size} bytes differ, first {d[0]}, last {d[-1]}"


f = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv"))
w, h, q = f.width, f.height, (50, 50, 50)
c = myyuv_hip.Codec(0)
raw = c.decompress(f.data, w, h, q)
pay = c.compress(raw, w, h, q)
print("single roundtrip:", diff(c.decompress(pay, w, h, q), raw), flush=True)
for name, call in (("decompress_batch", c.decompress_batch), ("decompress_frames", c.decompress_frames)):
    for n in (1, 2, 3):
        outs = call([pay] * n, w, h, q)
        print(name, n, [diff(o, raw) for o in outs], flush=True)
for n in (1, 3):
    pays = c.compress_frames([raw] * n, w, h, q)
    print("compress_frames", n, [diff(p, pay) for p in pays], flush=True)
    pays = c.compress_batch([raw] * n, w, h, q)
    print("compress_batch", n, [diff(p, pay) for p in pays], flush=True)
c.close()
