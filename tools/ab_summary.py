"""Summarises tools/ab.sh output: per (config, variant) the median ms/step and kernel averages."""
import collections
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    v, c, _ = os.path.basename(f)[:-5].rsplit("_", 2)
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    rows[(c, v)].append(j)
for js in rows.values():  # --emulate-shard lines: the slowest rank's frame and kernels
    for j in js:
        if "max_rank_ms" in j:
            j["ms_per_step"] = j["max_rank_ms"]
            j["kernels"] = {k: {"avg_us": u} for k, u in j["ranks"][j["max_rank"]]["kernels_us"].items()}
for (c, v), js in sorted(rows.items()):
    ms = statistics.median(j["ms_per_step"] for j in js) * 1e3
    ks = {k: statistics.median(j["kernels"][k]["avg_us"] for j in js) for k in js[0]["kernels"]}
    print(f"{c:9s} {v:8s} frame {ms:7.1f} us  " + "  ".join(f"{k} {u:6.1f}" for k, u in ks.items())
          + f"  (n={len(js)}, {' '.join('%.1f' % (j['ms_per_step'] * 1e3) for j in js)})")
