#!/usr/bin/env python3
"""Summarise the FETCH_SIZE / WRITE_SIZE calibration (tools/ubench/calib.hip
run under rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, tools/runs/r02c.sh) into
profiles/<tag>_calib.json: per access shape, the known bytes per launch and
bytes / (counter KiB x 1024) — the factor tools/traffic.py applies to the
codec kernel with that shape."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            d[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]].append(float(r["Counter_Value"]))
    return d


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"calib_{tag}")
    known = {}
    with open(os.path.join(src, "calib.json")) as f:
        for line in f:
            if line.startswith("{"):
                d = json.loads(line)
                known[d["kernel"]] = d
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"))
    out = {"_note": "factor = known bytes per launch / (counter KiB x 1024), mean over the launches; "
                    "read shapes use FETCH_SIZE, write shapes WRITE_SIZE; buffers exceed the 256 MiB Infinity Cache"}
    for k, d in known.items():
        ctr = fetch if k.endswith("read") else write
        vals = ctr.get(k, [])
        if not vals:
            continue
        kib = sum(vals) / len(vals)
        out[k] = {"counter": "FETCH_SIZE" if k.endswith("read") else "WRITE_SIZE",
                  "bytes_per_launch": d["bytes_per_launch"], "counter_kib": round(kib, 1),
                  "factor": round(d["bytes_per_launch"] / (kib * 1024), 4), "TBps": d["TBps"]}
    dst = os.path.join(ROOT, "profiles", f"{tag}_calib.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
