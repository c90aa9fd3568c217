#!/usr/bin/env python3
"""Summarises rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into the JSON
bench.py reads for ``roofline.traffic``.

  python tools/pmc_summary.py --fetch DIR/run_counter_collection.csv \
      --write DIR2/run_counter_collection.csv --calib CALIB_FETCH.csv CALIB_WRITE.csv \
      --config c2 -o profiles/r02_pmc_c2.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md §HBM: on
gfx950 FETCH_SIZE reports half the bytes of 16-B/lane streaming reads; other
widths are uncalibrated there, so tools/pmc_calib.hip measures the factor for the
draw path's own access shapes and this script records them next to the totals.
The draw kernels mix shapes (64-B record gathers, 12-B vertex gathers, 4-B
coalesced lists), so ``hbm_bytes_per_launch`` applies the calibrated factor of
the dominant read shape of each kernel (``READ_SHAPE``) and says so.
"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zenith_amd.buildinfo import source_hash  # noqa: E402  (the build the passes profiled)

KERNELS = {"k_setup_bin": "setup_bin", "k_tile": "tile", "k_clear": "clear"}
# setup_bin reads indices and positions of consecutive vertices: dense, coalesced
# (the ½-count case).  tile reads are 64-B record gathers (counted at face value).
# A narrow gather's calibration factor (gather12) measures line over-fetch, which is
# real traffic, so it is recorded but never applied.
READ_SHAPE = {"setup_bin": "stream4", "tile": "gather64", "clear": "stream4"}
WRITE_SHAPE = {"setup_bin": "store64", "tile": "store4", "clear": "store4"}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"]
        for key, short in KERNELS.items():
            if key in name:
                acc[(short, row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    out = collections.defaultdict(list)
    for (short, _), vals in acc.items():
        out[short].append(sum(vals))  # one value per dispatch (summed over instances)
    return {k: sum(v) / len(v) for k, v in out.items()}, {k: len(v) for k, v in out.items()}


def calib(path, counter, known):
    vals, _ = per_kernel_raw(path, counter)
    return {k: known[k] / (v * 1024.0) for k, v in vals.items() if k in known and v > 0}


def per_kernel_raw(path, counter):
    acc = collections.defaultdict(float)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter:
            acc[(row["Kernel_Name"].split("(")[0], row["Dispatch_Id"])] += float(row["Counter_Value"])
    out = collections.defaultdict(list)
    for (name, _), v in acc.items():
        out[name].append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}, None


def tile_classes(paths, tile):
    """The tile pass's read bytes per request class, from FETCH_SIZE passes of the
    ZR_TILE_DEBUG variant: each ZR_DEBUG switch removes one class of reads
    (pmc_classes.sh), so a class is the drop it causes; "lists_records" (the
    raster's bin-list and record reads) is what remains above the no-raster pass.
    Bytes per launch at the tile pass's fetch factor; stores are WRITE_SIZE."""
    kib = [per_kernel(p, "FETCH_SIZE")[0].get("tile", 0.0) for p in paths]
    dbg0, ids, attrs, recs, noraster = kib
    f = tile["fetch_factor"] * 1024
    c = {"winner_ids": max(dbg0 - ids, 0.0) * f, "winner_attributes": max(dbg0 - attrs, 0.0) * f,
         "resolve_records": max(dbg0 - recs, 0.0) * f}
    c["lists_records"] = max(dbg0 - noraster, 0.0) * f - sum(c.values())
    c["rest"] = noraster * f
    c = {k: int(v) for k, v in c.items()}
    c["stores"] = int(tile["write_kib_per_launch"] * 1024 * tile["write_factor"])
    c["debug_variant_fetch_kib"] = round(dbg0, 1)
    return c


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--fetch", required=True)
    p.add_argument("--write", required=True)
    p.add_argument("--calib", nargs=2, metavar=("FETCH_CSV", "WRITE_CSV"))
    p.add_argument("--calib-known", help="JSON line printed by pmc_calib (bytes moved per kernel)")
    p.add_argument("--config", default="c2")
    p.add_argument("--classes", nargs=5, metavar=("DBG0", "IDS", "ATTRS", "RECS", "NORASTER"),
                   help="FETCH_SIZE csvs of the tile-debug variant (tools/pmc_classes.sh): the tile pass's "
                        "reads split by request class")
    p.add_argument("-o", "--output", required=True)
    a = p.parse_args()
    fetch, nf = per_kernel(a.fetch, "FETCH_SIZE")
    write, nw = per_kernel(a.write, "WRITE_SIZE")
    rf = wf = {}
    if a.calib:
        known = json.loads(open(a.calib_known).read().strip().splitlines()[-1])
        rf = calib(a.calib[0], "FETCH_SIZE", known)
        wf = calib(a.calib[1], "WRITE_SIZE", known)
    out = {"config": a.config, "build": source_hash(),
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)",
           "calibration": {"fetch_factor": rf, "write_factor": wf,
                           "note": "bytes moved / (counter KiB * 1024) on 1 GiB buffers (tools/pmc_calib.hip)"},
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fkb, wkb = fetch.get(k, 0.0), write.get(k, 0.0)
        ff = rf.get(READ_SHAPE[k], 2.0 if not rf else 1.0)
        wfac = wf.get(WRITE_SHAPE[k], 1.0)
        out["kernels"][k] = {
            "fetch_kib_per_launch": round(fkb, 1), "write_kib_per_launch": round(wkb, 1),
            "launches": [nf.get(k, 0), nw.get(k, 0)],
            "read_shape": READ_SHAPE[k], "fetch_factor": round(ff, 3),
            "write_shape": WRITE_SHAPE[k], "write_factor": round(wfac, 3),
            "hbm_bytes_per_launch": int(fkb * 1024 * ff + wkb * 1024 * wfac),
        }
    if a.classes and "tile" in out["kernels"]:
        out["kernels"]["tile"]["classes"] = tile_classes(a.classes, out["kernels"]["tile"])
    with open(a.output, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
