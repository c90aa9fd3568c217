#!/usr/bin/env python3
"""Per-kernel averages of the counter passes written by tools/pmc_probe.sh.

  python3 tools/pmc_table.py gpurun_out/pmc_<tag>

Every pass directory pN/ holds rocprofv3's run_counter_collection.csv; values of
one (dispatch, counter) are summed over rows, then averaged over the dispatches
of each kernel (k_setup_bin, k_tile, k_route).  SQ cycle counters count
quad-cycles (MI355X_MICROARCH.md, cycle constants), so the derived shares are
ratios of counters of one unit.
"""
import collections
import csv
import glob
import os
import sys

KERNELS = ("k_setup_bin", "k_tile", "k_route")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def main(root):
    acc = collections.defaultdict(float)  # (kernel, dispatch, counter) -> value
    for path in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(path)):
            k = short(row.get("Kernel_Name", ""))
            if k:
                acc[(k, path, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    per = collections.defaultdict(list)
    for (k, _, _, c), v in acc.items():
        per[(k, c)].append(v)
    kernels = sorted({k for k, _ in per})
    counters = sorted({c for _, c in per})
    for k in kernels:
        print(f"== {k}")
        vals = {}
        for c in counters:
            v = per.get((k, c))
            if v:
                vals[c] = sum(v) / len(v)
                print(f"  {c:36s} {vals[c]:16.1f}   (n={len(v)})")
        w = vals.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
                if c in vals:
                    print(f"  share {c:30s} {vals[c] / w:8.3f} of SQ_WAVE_CYCLES")
        if "TCC_HIT_sum" in vals and "TCC_MISS_sum" in vals:
            h, m = vals["TCC_HIT_sum"], vals["TCC_MISS_sum"]
            print(f"  L2 hit rate {h / max(h + m, 1):.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
