"""Generates tests/golden/batch4k_512.json: the known answers of BASELINE.json
configs[3]/[4] — 512 synthetic 3840x2160 IYUV frames, q=50, frame f the tiled
chef-big frame with origin (f*8 mod 4032, f*8 mod 3008) (SURVEY.md §8d item 4,
yuv-manipulations-2_amd/synth.py) — from the CPU restatement, which is pinned
byte-exact to the reference's goldens and to the reference library itself
(tests/test_oracle.py).  Per frame: the input's sha256, the DCTYUV payload's
size and sha256 (DCT.cpp:371-430) and the sha256 of its decode (DCT.cpp:432-488).
Frames 0, 1, 255 and 511 are cross-checked against the reference library
compiled from /root/reference (oracle/_ref) when it is built.
Run from the repo root: python tests/golden/make_batch4k.py"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
import myyuv_file  # noqa: E402
import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import ref as R  # noqa: E402

W, H, Q, N = 3840, 2160, 50, 512


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    g = myyuv_file.YUVFile.load(os.path.join(HERE, "chef-with-trumpet-big-DCT-50.myyuv"))
    raw = O.decompress(g.data, g.width, g.height, tuple(g.params))
    assert sha(g.decompressed(raw).dumps()) == "5e7769191188285cc127c6b4da900b3420f064191f707383c82128c14e497e5c"
    q3 = (Q, Q, Q)
    frames = []
    t0 = time.time()
    for f in range(N):
        ox, oy = synth.batch_origin(f, g.width, g.height)
        px = synth.tiled_frame(raw, g.width, g.height, W, H, ox, oy).tobytes()
        pay = O.compress(px, W, H, q3)
        dec = O.decompress(pay, W, H, q3)
        if f in (0, 1, 255, 511) and R.available("omp"):
            assert R.compress(px, W, H, q3) == pay, f
            assert R.decompress(pay, W, H, q3) == dec, f
        frames.append({"f": f, "origin": [ox, oy], "input_sha": sha(px), "payload_size": len(pay),
                       "payload_sha": sha(pay), "decoded_sha": sha(dec)})
        if f % 64 == 63:
            print(f"{f + 1}/{N} frames, {time.time() - t0:.0f} s", flush=True)
    # SURVEY.md §8d pins frame 0: the origin-0 tiled frame and its q50 file
    f0 = frames[0]
    assert f0["payload_size"] == 2155708
    out = {"width": W, "height": H, "quality": Q, "frames_total": N,
           "generator": "synth.tiled_frame(chef-big decoded, 3840, 2160, *synth.batch_origin(f, 4032, 3008))",
           "made_by": "tests/golden/make_batch4k.py (oracle/myyuv_oracle.c; frames 0, 1, 255, 511 "
                      "also through oracle/_ref, the reference library)",
           "sum_payload_bytes": sum(x["payload_size"] for x in frames), "frames": frames}
    write(out, os.path.join(HERE, "batch4k_512.json"))


def write(out, path):
    """One frame record per line."""
    head = {k: v for k, v in out.items() if k != "frames"}
    with open(path, "w") as fh:
        fh.write(json.dumps(head)[:-1] + ', "frames": [\n')
        fh.write(",\n".join(json.dumps(x) for x in out["frames"]))
        fh.write("\n]}\n")


if __name__ == "__main__":
    main()
