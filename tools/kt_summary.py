#!/usr/bin/env python3
"""Summarises a rocprofv3 --kernel-trace --stats run of bench.py into the JSON
bench.py quotes as ``kernels_rocprof`` (per pass: calls and average duration),
stamped with the build it profiled (zenith_amd/buildinfo.py).

  python tools/kt_summary.py DIR/run_kernel_stats.csv --config c2 -o profiles/r06_v1_kt_c2.json
"""
import argparse
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zenith_amd.buildinfo import source_hash  # noqa: E402

KERNELS = {"k_setup_bin": "setup_bin", "k_tile": "tile", "k_clear": "clear", "k_route": "route"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("stats")
    p.add_argument("--config", default="c2")
    p.add_argument("-o", "--output", required=True)
    a = p.parse_args()
    out = {"config": a.config, "build": source_hash(), "source": "rocprofv3 --kernel-trace --stats", "kernels": {}}
    with open(a.stats) as fh:
        for row in csv.DictReader(fh):
            m = re.search(r"zr::(k_\w+)", row["Name"])
            if not m or m.group(1) not in KERNELS:
                continue
            k = out["kernels"].setdefault(KERNELS[m.group(1)], {"calls": 0, "total_ns": 0, "instances": []})
            k["calls"] += int(row["Calls"])
            k["total_ns"] += int(float(row["TotalDurationNs"]))
            k["instances"].append(row["Name"])
    for k in out["kernels"].values():
        k["avg_us"] = round(k["total_ns"] / max(k["calls"], 1) / 1e3, 2)
    with open(a.output, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
