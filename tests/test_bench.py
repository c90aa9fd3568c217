"""bench.py's contract: the per-pass algorithmic bytes of SURVEY.md §8d and, on
the GPU, the one JSON line the driver parses (keys, roofline and CPU-baseline
objects, the cold-cache pass over rotated input copies)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bytes_per_triangle_match_survey():
    from zenith_amd import scenes
    # 84 B (24-B stride) and 120 B (36-B stride) per triangle
    assert scenes.config_bytes_per_triangle("c1") == 84
    assert scenes.config_bytes_per_triangle("c2") == 120
    assert scenes.config_bytes_per_triangle("c3") == 120
    assert scenes.config_bytes_per_triangle("c4") == 84


def test_algorithmic_bytes():
    import bench
    n, pairs, px = 1_000_000, 1_315_362, 1920 * 1080
    # setup: inputs once + one 32-B compact record per triangle + a 4-B bin entry per pair
    assert bench.algorithmic_bytes("setup_bin", n, 120, pairs, px) == n * (120 + 32) + pairs * 4
    # partitioned setup: a received 48-B route entry in, its 32-B record out
    assert bench.algorithmic_bytes("setup_bin", n, 120, pairs, px, n_route=10) == n * (48 + 32) + pairs * 4
    # tile: bin entry + record per pair, colour + depth texel per owned pixel
    assert bench.algorithmic_bytes("tile", n, 120, pairs, px) == pairs * 36 + px * 8
    assert bench.algorithmic_bytes("route", n, 120, pairs, px, n_route=1000) == 48_000
    assert bench.algorithmic_bytes("exchange", n, 120, pairs, px) == 0
    # C2's frame = 120 MB of input + 16.6 MB of colour + depth
    assert n * 120 + px * 8 == 136_588_800


@pytest.mark.gpu
def test_bench_json_line():
    """One short C1 run with a two-copy cold pass, as a child process: stdout holds
    exactly one JSON line with the contract's keys (SURVEY.md §8d extras included)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c1", "--steps", "4", "--warmup", "2",
           "--cold-copies", "2", "--cpu-seconds", "0.5"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "kernels"):
        assert k in d, k
    assert d["unit"] == "Mtri/s" and d["n_gpus"] == 1 and d["steps"] == 4 and d["value"] > 0
    assert d["config"]["input_copies"] == 1 and d["config"]["triangles"] == 100_000
    assert d["cold_copies"] == 2 and d["value_cold"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 6290.0 and r["peak_spec"] == 8000.0
    assert r["kernel"] in d["kernels"] and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["survey_bytes_per_pair"] == 68 and r["achieved_survey"] > d["kernels"]["tile"]["gbps"]
    assert r["traffic"] is None  # the committed PMC summary is C2's, not C1's
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0
    assert cb["nproc"] == cb["cores"] and cb["nproc_all"] >= cb["nproc"] and cb["cpu_model"]
    assert set(d["kernels"]) >= {"setup_bin", "tile"}


@pytest.mark.gpu
@pytest.mark.parametrize("setup", ["replicated", "partitioned"])
def test_bench_emulate_shard(setup):
    """--emulate-shard G: every rank of the shard timed in turn beside T1; the
    speed-up is T1 / the slowest rank's frame, and partitioned ranks receive the
    records the others really routed (no block overflow at the measured capacity)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c1", "--steps", "4", "--warmup", "2",
           "--emulate-shard", "4", "--setup", setup, "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.strip()][-1])
    assert len(d["rank_ms"]) == 4 and d["max_rank_ms"] == max(d["rank_ms"])
    assert abs(d["speedup"] - d["t1_ms"] / d["max_rank_ms"]) < 1e-2
    assert d["ranks"][d["max_rank"]]["ms"] == d["max_rank_ms"]
    if setup == "partitioned":
        assert d["route_capacity"] > 0 and all(r["route_fallback_draws"] == 0 for r in d["ranks"])
        assert sum(r["triangles_setup"] for r in d["ranks"]) >= 100_000 * 0.9
