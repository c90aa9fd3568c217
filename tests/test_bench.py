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
    # setup is credited with what it loads: 3 u32 indices + 3 float3 positions
    assert bench.SETUP_IN_BYTES == 48


def test_design_bytes_by_request_class():
    import bench
    from zenith_amd import scenes
    # per winner: 12-B vertex ids + the program's attributes of its 3 vertices
    assert bench.winner_bytes(scenes.PROGRAM_BLINN_PHONG) == 12 + 3 * 24
    assert bench.winner_bytes(scenes.PROGRAM_FLAT_COLOR) == 12 + 12
    assert bench.winner_bytes(scenes.PROGRAM_TRIANGLE, 2) == 6 + 36
    assert bench.winner_bytes(scenes.PROGRAM_MESH) == 12 + 60 + 48
    d = bench.design_tile_bytes(1_000, 300, 84, 2_000)
    assert d == {"bins": 4_000, "records": 32_000, "winner_gathers": 25_200, "stores": 16_000}


def test_quoted_profiles_name_this_build():
    """The PMC and kernel-trace summaries bench.py quotes by default (roofline.traffic,
    kernels_rocprof) profiled the library built from this tree: their build stamp
    is the hash of the current sources (zenith_amd/buildinfo.py), and a profile of
    another build is never quoted (build_profile)."""
    import bench
    from zenith_amd import buildinfo
    for name in ("pmc", "kt"):
        path = os.path.join(ROOT, "profiles", f"{bench.PROFILE_TAG}_{name}_c2.json")
        prof, src = bench.build_profile(path, "c2")
        assert prof is not None, src
        assert prof["build"] == buildinfo.source_hash()
    pmc, _ = bench.build_profile(os.path.join(ROOT, "profiles", f"{bench.PROFILE_TAG}_pmc_c2.json"), "c2")
    assert pmc["kernels"]["tile"]["hbm_bytes_per_launch"] > 0
    stale = dict(pmc, build="0" * 16)
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as fh:
        json.dump(stale, fh)
    try:
        prof, src = bench.build_profile(fh.name, "c2")
        assert prof is None and "not this tree's" in src
    finally:
        os.unlink(fh.name)


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
    dz = r["design"]  # winner census: distinct winners <= primitives, > 0 on a soup
    assert 0 < dz["winners"] <= 100_000 and dz["bytes_per_winner"] == 24
    assert dz["bytes"] == sum(dz["classes"].values()) and dz["achieved"] > r["achieved"]
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


def test_setup_auto():
    """--setup auto (the default): partitioned for dense draws (256+ triangles
    per 32x32 tile) at 8+ ranks -- C2 at 8 -- replicated otherwise (C2 at 2/4, C3
    and C1 at 8, any single GPU); an explicit choice is kept."""
    import bench
    assert bench.setup_mode("auto", 8, 1_000_000, 1920, 1080) == "partitioned"
    for g in (1, 2, 4):
        assert bench.setup_mode("auto", g, 1_000_000, 1920, 1080) == "replicated"
    assert bench.setup_mode("auto", 8, 1_000_000, 3840, 2160) == "replicated"
    assert bench.setup_mode("auto", 8, 100_000, 1920, 1080) == "replicated"
    assert bench.setup_mode("replicated", 8, 1_000_000, 1920, 1080) == "replicated"
    assert bench.setup_mode("partitioned", 2, 100_000, 1920, 1080) == "partitioned"


# ------------------------------------------------ launcher-less multi-GPU runs
def test_worker_commands():
    """bench.py --gpus N without a launcher: N children of the same script with the
    same arguments, ranks / device ids / a 127.0.0.1 rendezvous in their env."""
    import bench
    argv = ["--gpus", "4", "--steps", "5", "--config", "c3"]
    cmds = bench.worker_commands(4, argv, 29777, base_env={"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert len(cmds) == 4
    for r, (cmd, env) in enumerate(cmds):
        assert cmd[0] == sys.executable and cmd[-len(argv):] == argv
        assert os.path.basename(cmd[-len(argv) - 1]) == "bench.py"
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29777"
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/usr/bin"  # inherited


def _py(code):
    return ([sys.executable, "-c", code], dict(os.environ))


def test_run_workers_relays_rank0_line():
    import io
    import bench
    buf = io.StringIO()
    rc = bench.run_workers([_py("print('{\"value\": 1}')"), _py("print('rank1 noise')")], out=buf)
    assert rc == 0 and buf.getvalue().strip() == '{"value": 1}'  # rank 1's stdout is not relayed


def test_run_workers_propagates_failure_and_stops_the_rest():
    """A failing worker ends the run with its exit status; the others (which would
    wait in a collective for it) are stopped instead of waited for."""
    import io
    import time
    import bench
    t0 = time.monotonic()
    rc = bench.run_workers([_py("import time; time.sleep(60)"), _py("import sys; sys.exit(3)"),
                            _py("import time; time.sleep(60)")], out=io.StringIO())
    assert rc == 3 and time.monotonic() - t0 < 30
    rc = bench.run_workers([_py("import os, signal; os.kill(os.getpid(), signal.SIGKILL)")], out=io.StringIO())
    assert rc == 128 + 9
    t0 = time.monotonic()
    rc = bench.run_workers([_py("import time; time.sleep(60)")], out=io.StringIO(), timeout=1.0)
    assert rc == 124 and time.monotonic() - t0 < 30


def test_launcherless_parent_never_touches_the_gpu(monkeypatch):
    """The launcher path returns before any HIP call: main() with WORLD_SIZE unset
    and --gpus 2 only builds worker commands (here intercepted)."""
    import bench
    seen = {}

    def fake_launch(a, argv):
        seen["gpus"], seen["argv"] = a.gpus, argv
        return 0
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_workers", fake_launch)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    monkeypatch.setattr(bench.torch.cuda, "set_device", lambda *x: (_ for _ in ()).throw(AssertionError("GPU")))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and seen == {"gpus": 2, "argv": ["--gpus", "2", "--steps", "3"]}


@pytest.mark.gpu
def test_bench_force_dist_worker_path():
    """bench.py --gpus 1 --force-dist without a launcher runs through the worker
    launcher (one RCCL rank, the runtime's exchange + row gather) and prints one
    JSON line."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-dist", "--config", "c1",
           "--steps", "4", "--warmup", "2", "--cold-copies", "0", "--setup", "partitioned", "--worker-timeout", "100"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=115, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and "RCCL" in d["config"]["parallelism"]
