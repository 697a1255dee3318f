#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_*.

Reads gpurun_out/prof_<tag>/{trace,fetch,write}/run_*.csv and writes
  profiles/<tag>_kernel_stats.csv   (rocprofv3 --kernel-trace --stats summary)
  profiles/<tag>_traffic.json       per-kernel HBM bytes per launch
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced stream, so read bytes = 2 * FETCH_SIZE * 1024 for kernels whose
reads are 16-B-per-lane streams, write bytes = WRITE_SIZE * 1024.  K1's 8-B
row loads / 16-B quad stores, K6's quad loads / 8-B row stores, K2's
scattered row loads and K4's gathers have their own factors, measured on known byte counts with the same addressing
(tools/ubench/calib.hip -> profiles/<tag>_calib.json, newest one used).
"""
import collections
import csv
import json
import os
import shutil
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def kname(n):
    """Short kernel name: no namespace, return type or template arguments (k_huff_encode<8u> -> huff_encode)."""
    return re.sub(r"<[^>]*>$", "", n.split("(")[0].replace("void ", "").replace("myyuv_gpu::k_", ""))

def per_kernel(path):
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            d[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


# codec kernel -> (read shape, write shape) of tools/ubench/calib.hip.  K2's
# reads are dominated by its scattered per-lane 16-B row loads (runs of
# blocks), whose FETCH_SIZE counts the bytes once (factor ~1, not 2,
# profiles/r4b_calib.json); its classify pass's coalesced rmask/DC reads
# (factor 2) are ~5 % of the bytes, so the K2 figures are a lower bound
# within that.  K4 gathers 16-B words coalesced (factor 2).
CALIB_SHAPES = {"fdct_quant": ("k1_read", "k1_write"), "dequant_idct": ("k6_read", "k6_write"),
                "huff_encode": ("k2_scatter_read", None), "huff_encode_r16": ("k2_scatter_read", None),
                "huff_encode_wide": ("k2_scatter_read", None), "stream_out": ("k4_gather_read", None)}


def calib_factors():
    pdir = os.path.join(ROOT, "profiles")
    names = sorted(n for n in os.listdir(pdir) if n.endswith("_calib.json"))
    if not names:
        return {}, None
    with open(os.path.join(pdir, names[-1])) as f:
        d = json.load(f)
    return {k: v["factor"] for k, v in d.items() if isinstance(v, dict)}, names[-1]


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats.csv"))
    durations = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            durations[kname(r["Name"])] = float(r["AverageNs"])
    fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"))
    cf, cname = calib_factors()
    out = {"_note": "bytes per launch; read = 2 x FETCH_SIZE (gfx950 wide-stream correction), "
                    "write = WRITE_SIZE; both KiB x 1024; fdct_quant / dequant_idct / huff_encode* / "
                    f"stream_out use the factors measured for their own access shapes ({cname}: "
                    "K2's scattered row loads count once, factor ~1); avg_ns from the kernel-trace pass"}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd") or "at::native" in k:
            continue
        rs, ws = CALIB_SHAPES.get(k, (None, None))
        rf, wf = cf.get(rs, 2.0), cf.get(ws, 1.0)
        rd = rf * fetch.get(k, 0.0) * 1024
        wr = wf * write.get(k, 0.0) * 1024
        out[k] = {"fetch_kib": round(fetch.get(k, 0.0), 1), "write_kib": round(write.get(k, 0.0), 1),
                  "hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
                  "read_factor": rf, "write_factor": wf,
                  "hbm_bytes_per_launch": int(rd + wr), "avg_ns": durations.get(k)}
        if durations.get(k):
            out[k]["hbm_gb_per_s"] = round((rd + wr) / durations[k], 1)
    # the bench run profiled (tools/profile.sh): its frame and launch-group
    # size, so bench.py can scale the per-launch bytes to its own groups
    bj = os.path.join(src, "bench_trace.json")
    if os.path.exists(bj):
        with open(bj) as f:
            cfg = json.loads(f.read().strip().splitlines()[-1])["config"]
        out["_bench"] = {"frame": cfg["frame"], "frames_per_launch": cfg["frames_per_launch"]}
    with open(os.path.join(dst, f"{tag}_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
