"""Diagnostic (test infrastructure): compress the tiled 8192^2 frame at q90 with
the library named by MYYUV_HIP_LIB (split encoder), compare with the oracle and
report where the payload first differs (plane, block), and whether two
compressions of the same input agree."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."),
                os.path.join(os.path.dirname(__file__), "..", "..", "yuv-manipulations-2_amd")]
import numpy as np
os.environ["MYYUV_ENCODER"] = "split"
import myyuv_hip, myyuv_file, synth
from oracle import oracle as O
O.lib()
here = os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden")
f = myyuv_file.YUVFile.load(os.path.join(here, "chef-with-trumpet-big-DCT-50.myyuv"))
raw = O.decompress(f.data, f.width, f.height, tuple(f.params))
q = int(sys.argv[1]) if len(sys.argv) > 1 else 90
W = H = 8192
img = synth.tiled_frame(raw, f.width, f.height, W, H).tobytes()
c = myyuv_hip.Codec()
ref = O.compress(img, W, H, (q, q, q))
runs = [c.compress(img, W, H, (q, q, q)) for _ in range(int(os.environ.get("NRUNS", "6")))]
print("sizes", [len(x) for x in runs], "ref", len(ref), "equal to ref", [x == ref for x in runs])
bad = [x for x in runs if x != ref]
a = bad[0] if bad else runs[0]
A = np.frombuffer(a, np.uint8); R = np.frombuffer(ref, np.uint8)
n = min(len(A), len(R))
d = np.nonzero(A[:n] != R[:n])[0]
print("differing bytes", d.size, "first", d[:8].tolist(), "last", d[-4:].tolist() if d.size else [])
if d.size:
    # layout: 12-byte header (3 x u32 plane sizes), then per plane: u32 nb, u32 content, nb chunk_size bytes, content
    pos = 12
    for p in range(3):
        nb, content = np.frombuffer(ref[pos:pos + 8], np.uint32)
        s0, c0, end = pos + 8, pos + 8 + nb, pos + 8 + nb + content
        sel = d[(d >= pos) & (d < end)]
        if sel.size:
            sizes = R[s0:c0].astype(np.int64)
            offs = np.concatenate([[0], np.cumsum(sizes)])
            first = sel[0]
            if first < c0:
                print(f"plane {p}: first diff in chunk_size array, block {first - s0}")
            else:
                blk = int(np.searchsorted(offs, first - c0, side="right") - 1)
                bad = np.unique(np.searchsorted(offs, sel[sel >= c0] - c0, side="right") - 1)
                print(f"plane {p}: nb {nb} first diff block {blk} (tile {blk // 256}, lane {blk % 256}) size {sizes[blk]}; "
                      f"{bad.size} blocks differ, first ones {bad[:10].tolist()} sizes {sizes[bad[:10]].tolist()}")
                print("  gpu", A[c0 + offs[blk]: c0 + offs[blk] + sizes[blk]].tolist())
                print("  ref", R[c0 + offs[blk]: c0 + offs[blk] + sizes[blk]].tolist())
        pos = end
