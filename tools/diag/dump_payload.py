"""Diagnostic (GPU): decompress a golden file with the HIP decoder, compress
the pixels again at the file's qualities and write the payload, for
tools/diag/payload_diff.py to compare two builds' payloads block by block
(MYYUV_HIP_LIB picks the build):
  python3 tools/diag/dump_payload.py <golden-name> <out.bin>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
import myyuv_file  # noqa: E402
import myyuv_hip  # noqa: E402

f = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests", "golden", sys.argv[1]))
c = myyuv_hip.Codec(0)
raw = c.decompress(f.data, f.width, f.height, tuple(f.params))
pay = c.compress(raw, f.width, f.height, tuple(f.params))
open(sys.argv[2], "wb").write(pay)
print(sys.argv[2], len(pay))
