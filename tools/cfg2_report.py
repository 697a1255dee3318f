#!/usr/bin/env python3
"""BASELINE configs[2] summary (tools/cfg2_profile.sh -> tools/traffic.py):
the 8192x8192 tiled frame at q50 and q90, one frame per launch.  Writes
profiles/<tag>_summary.json: per kernel the rocprofv3 average duration, the
calibrated HBM bytes and GB/s; K1's roofline on the algorithmic 3 B/sample
(DESIGN.md §4); the summed kernel time per frame for compress and decompress.

  python3 tools/cfg2_report.py r05cfg2
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK_GBS = 8000.0
W = H = 8192
SAMPLES = W * H * 3 // 2
ENC = ("fdct_quant", "huff_encode", "huff_encode_r16", "huff_encode_wave", "huff_encode_wide", "tile_scan", "stream_out")
DEC = ("scan_chain", "decode_idct")


def main(tag):
    out = {"_note": "8192x8192 tiled frame (SURVEY.md §8d generator), one frame per launch, kernels "
                    "alone on the GPU (tools/kbench.py under rocprofv3); bytes per launch from FETCH_SIZE / "
                    "WRITE_SIZE passes with the calibrated factors (tools/traffic.py); K1 roofline on "
                    "3 B/sample algorithmic bytes, 8 TB/s peak"}
    for q in (50, 90):
        with open(os.path.join(ROOT, "profiles", f"{tag}_q{q}_traffic.json")) as f:
            t = json.load(f)
        ks = {k: v for k, v in t.items() if not k.startswith("_")}
        row = {k: {"avg_us": round(v["avg_ns"] / 1e3, 2), "hbm_mb": round(v["hbm_bytes_per_launch"] / 1e6, 2),
                   "hbm_gb_per_s": v.get("hbm_gb_per_s")} for k, v in ks.items() if v.get("avg_ns")}
        k1 = ks["fdct_quant"]["avg_ns"]
        alg = 3 * SAMPLES
        row["k1_roofline"] = {"algorithmic_bytes": alg, "achieved_gb_per_s": round(alg / k1, 1),
                              "frac": round(alg / k1 / PEAK_GBS, 4)}
        enc = sum(ks[k]["avg_ns"] for k in ENC if k in ks and ks[k].get("avg_ns"))
        dec = sum(ks[k]["avg_ns"] for k in DEC if k in ks and ks[k].get("avg_ns"))
        row["frame_us"] = {"compress": round(enc / 1e3, 1), "decompress": round(dec / 1e3, 1),
                           "round_trip_mp_per_s": round(W * H / 1e6 / ((enc + dec) / 1e9), 1)}
        out[f"q{q}"] = row
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r05cfg2")
