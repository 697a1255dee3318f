#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_*.

Reads gpurun_out/prof_<tag>/{trace,fetch,write}/run_*.csv and writes
  profiles/<tag>_kernel_stats.csv   (rocprofv3 --kernel-trace --stats summary)
  profiles/<tag>_traffic.json       per-kernel HBM bytes per launch
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced stream, so read bytes = 2 * FETCH_SIZE * 1024 for kernels whose
reads are 16-B-per-lane streams, write bytes = WRITE_SIZE * 1024.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path):
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            d[r["Kernel_Name"].split("(")[0].replace("myyuv_gpu::k_", "")].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats.csv"))
    durations = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            durations[r["Name"].split("(")[0].replace("myyuv_gpu::k_", "")] = float(r["AverageNs"])
    fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"))
    out = {"_note": "bytes per launch; read = 2 x FETCH_SIZE (gfx950 wide-stream correction), "
                    "write = WRITE_SIZE; both KiB x 1024; avg_ns from the kernel-trace pass"}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd") or "at::native" in k:
            continue
        rd = 2.0 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        out[k] = {"fetch_kib": round(fetch.get(k, 0.0), 1), "write_kib": round(write.get(k, 0.0), 1),
                  "hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
                  "hbm_bytes_per_launch": int(rd + wr), "avg_ns": durations.get(k)}
    with open(os.path.join(dst, f"{tag}_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
