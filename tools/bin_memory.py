"""Bin buffer size and first / steady frame times per config.

Each config renders on a fresh RenderDevice: frame 1 (bin buffer of
bin_default_capacity, slabs of a third of it, everything past them in pool
runs), frame 2 (slabs of the target frame 1 measured, buffer resized at the sync
point between them), then W warm-up and K timed frames.  For each: the kernels'
times (HIP events), the bin buffer (entries = slabs + pool), the pairs, the
pool pairs and runs, and whether any tile fell back to the record scan.

    python tools/bin_memory.py --configs c2 c2x c3 c3x --steps 20 > gpurun_out/bin_memory.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from zenith_amd import renderer, rhi, scenes  # noqa: E402

RUN_CAP = 256  # kMaxRunsPerTile: the run table's entries per tile (uint2 each)


def one_frame(dev, enc):
    dev.kernel_times(reset=True)
    dev.set_profiling(True)
    t0 = time.perf_counter()
    dev.submit_and_wait(enc)
    wall = time.perf_counter() - t0
    dev.set_profiling(False)
    kt = {k: round(ms * 1e3 / max(n, 1), 1) for k, (ms, n) in dev.kernel_times().items()}
    st = dev.last_draw_stats()
    return {"wall_us": round(wall * 1e6, 1), "kernels_us": kt,
            **{k: st[k] for k in ("bin_pairs", "bin_capacity", "bin_pool_pairs", "bin_pool_runs", "overflowed_draws")}}


def measure(cfg, steps, warmup):
    s = scenes.config_scene(cfg)
    ntiles = -(-s.width // 32) * -(-s.height // 32)
    dev = rhi.RenderDevice(0)
    color = rhi.Texture(dev, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
    depth = rhi.Texture(dev, rhi.TextureDesc.new_depth("ds", s.width, s.height))
    rend = renderer.SceneRenderer(dev, s)
    enc = rend.record(color, depth)
    first = one_frame(dev, enc)
    second = one_frame(dev, enc)
    for _ in range(warmup):
        dev.submit(enc)
    dev.wait_idle()
    t0 = time.perf_counter()
    for _ in range(steps):
        dev.submit(enc)
    dev.wait_idle()
    steady_ms = (time.perf_counter() - t0) / steps * 1e3
    steady = one_frame(dev, enc)
    pairs, cap = steady["bin_pairs"], steady["bin_capacity"]
    out = {"config": cfg, "triangles": s.triangles, "target": f"{s.width}x{s.height}", "tiles": ntiles,
           "first": first, "second": second, "steady": steady, "steady_frame_ms": round(steady_ms, 4),
           "bin_mib": round(cap * 4 / 2**20, 2), "run_table_mib": round(ntiles * RUN_CAP * 8 / 2**20, 2),
           "capacity_over_pairs": round(cap / max(pairs, 1), 3),
           "bound_2x_pairs_plus_512_per_tile": 2 * pairs + 512 * ntiles,
           "spilled": steady["overflowed_draws"] > 0}
    enc.destroy()
    color.destroy()
    depth.destroy()
    dev.close()
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", nargs="+", default=["c2", "c2x", "c3", "c3x"])
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    a = p.parse_args()
    for cfg in a.configs:
        print(json.dumps(measure(cfg, a.steps, a.warmup)), flush=True)


if __name__ == "__main__":
    main()
