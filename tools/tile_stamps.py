#!/usr/bin/env python3
"""Per-tile phase stamps of one frame (ZR_TILE_DEBUG variant, ZR_DEBUG=128):
where a tile's time goes (init, sort, raster, resolve) and how the tiles of the
pass spread over time.

  ZR_LIB_PATH=zenith_amd/variants/dbg/libzenith_raster.so \\
      python tools/tile_stamps.py --config c3 --shard 0 8 --out gpurun_out/stamps_c3s0
"""
import argparse
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c2")
    p.add_argument("--shard", nargs=2, type=int, default=None)
    p.add_argument("--frames", type=int, default=3)
    p.add_argument("--out", required=True)
    p.add_argument("--from-csv", action="store_true", help="report an existing <out>.tiles.csv (no GPU)")
    a = p.parse_args()
    if a.from_csv:
        return report(a, os.path.abspath(a.out))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    ts = os.path.abspath(a.out)
    for f in (ts, ts + ".tiles.csv"):
        if os.path.exists(f):
            os.remove(f)
    os.environ["ZR_DEBUG"] = "128"
    os.environ["ZR_DEBUG_TS"] = ts
    import torch  # noqa: F401  (the HIP runtime torch binds, as bench.py)
    from zenith_amd import renderer, rhi, scenes
    scene = scenes.config_scene(a.config)
    dev = rhi.RenderDevice(0)
    sh = tuple(a.shard) if a.shard else None
    # a first frame sizes the scratch (a tile list longer than its slab takes the
    # slow all-records scan until the runtime grows the bins at a sync point)
    renderer.render_scene(dev, scene, shard=sh, frames=1)
    renderer.render_scene(dev, scene, shard=sh, frames=a.frames)
    dev.close()
    report(a, ts)


def report(a, ts):
    rows = list(csv.reader(open(ts + ".tiles.csv")))
    # the csv holds one block per sync point, each starting with a header: keep the last
    starts = [i for i, r in enumerate(rows) if r and r[0] == "tile"]
    last = rows[starts[-1] + 1:]
    t = np.array([[float(x) for x in r[1:7]] for r in last])  # t0 start, t1 init, t2 sorted, t3 raster, t4 resolve, t5 chunks
    cnt = np.array([int(r[8]) for r in last])
    nbig = np.array([int(r[7]) for r in last])
    dur = t[:, 4] - t[:, 0]
    print(f"{a.config} shard {a.shard}: {len(t)} tiles, pass span {t[:, 4].max() - t[:, 0].min():.1f} us, "
          f"tile {dur.mean():.1f} us avg (p10 {np.percentile(dur, 10):.1f}, p90 {np.percentile(dur, 90):.1f}, "
          f"max {dur.max():.1f})")
    # (a tile with no segment leaves some of its slots from an earlier draw in
    # 256-thread builds: phase figures over the tiles whose stamps are in order)
    ok = np.all(np.diff(t[:, :5], axis=1) >= 0, axis=1)
    print(f"  phases over {ok.sum()} tiles with ordered stamps:")
    for name, i, j in (("init", 0, 1), ("sort", 1, 2), ("raster", 2, 3), ("resolve", 3, 4)):
        d = (t[:, j] - t[:, i])[ok]
        print(f"  {name:8s} avg {d.mean():6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")
    print(f"  starts: first {t[:, 0].min():.1f}, last {t[:, 0].max():.1f}; ends: first {t[:, 4].min():.1f}, "
          f"last {t[:, 4].max():.1f} us; list length avg {cnt[ok].mean():.0f} max {cnt[ok].max()}")
    heavy = np.argsort(-dur)[:8]
    steps = np.array([int(r[9]) for r in last])   # ZR_TILE_WORK_STATS builds: longest lane walks of the chunks
    sweeps = np.array([int(r[10]) for r in last])  # and wave-path sweeps
    print("  slowest tiles:")
    for k in heavy:
        ph = " ".join(f"{n} {t[k, j] - t[k, i]:.1f}" for n, i, j in (("init", 0, 1), ("sort", 1, 2), ("raster", 2, 3),
                                                                       ("resolve", 3, 4)))
        print(f"    #{k} {dur[k]:.1f} us, {cnt[k]} entries ({nbig[k]} wave-path), lane steps {steps[k]}, "
              f"wave sweeps {sweeps[k]}, start {t[k, 0]:.1f}: {ph}, chunks end {t[k, 5] - t[k, 2]:.1f} after sort")


if __name__ == "__main__":
    main()
