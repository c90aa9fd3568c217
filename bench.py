#!/usr/bin/env python3
"""Draw-path benchmark (BASELINE.json metric): Mtri/s + frames/s at 1080p on the
1M-triangle scene (config C2), 1..N GPUs of one node.

A step is one frame of the hot path: vertex/setup -> bin -> tile raster+resolve
(-> tile-row gather to rank 0 when N > 1).  Inputs (vertex/index buffers) are
uploaded once and resident in HBM before timing; the attachment CLEAR is fused
into the tile pass.  `value` is whole-job throughput: triangles of all frames /
max-over-ranks wall time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
  torchrun --nproc-per-node N bench.py --gpus N ...      (N > 1, RCCL gather)

Without a launcher (WORLD_SIZE unset) and N > 1 (or --force-dist), this process
touches no GPU: it starts N worker processes of itself (one per GPU, ranks and a
127.0.0.1 rendezvous in their environment), relays rank 0's JSON line and exits
non-zero when any worker fails (launch_workers).
"""
import argparse
import json
import os
import sys
import time

import torch  # first: libzenith_raster then binds to the same HIP runtime
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from zenith_amd import buildinfo, renderer, rhi, scenes, shard, zr  # noqa: E402

PROFILE_TAG = "r06_final"        # profiles/<tag>_{pmc,kt}_c2.json: the round's profiles of the final tree

HBM_PEAK_GBPS = 6290.0           # MI355X_MICROARCH.md: HBM3E measured (float4 copy), the peak SURVEY.md §8d fixes
HBM_SPEC_GBPS = 8000.0           # same table: 8.0 TB/s spec
METRIC = BASELINE_METRIC = "Mtriangles/s + frames/s at 1080p (1M-tri scene), 1/2/4/8 GPU; HBM GB/s vs roofline"
RECORD_BYTES = 32                # TriCompact, the per-primitive record k_tile reads per pair (zr_internal.h)
BIN_ENTRY_BYTES = 4
SURVEY_PAIR_BYTES = 68           # SURVEY.md §8d fragment pass: 4-B bin entry + 64-B setup record per pair


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="c2", choices=sorted(scenes.CONFIGS))
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cold-copies", type=int, default=3, metavar="K",
                   help="value_cold: a second timed pass cycling K uploaded copies of the geometry frame to "
                        "frame (K=3 puts C2's 360 MB of input past the 256 MiB Infinity Cache: the HBM-honest "
                        "rate, SURVEY.md §8d); 0 skips it")
    p.add_argument("--emulate-shard", type=int, default=0, metavar="G",
                   help="diagnostic (1 GPU): every rank of a G-way tile-row shard in turn, beside the unsharded "
                        "frame; reports the max-over-ranks frame time and T1 / that (no gather; partitioned "
                        "setup: each rank receives the records the other ranks really route to it)")
    p.add_argument("--setup", choices=["auto", "partitioned", "replicated"], default="auto",
                   help="tile-row shards: set up every primitive on every rank (binning only its own rows), "
                        "or route 1/G of the primitives per rank through an RCCL all-to-all (DESIGN.md §7); "
                        "auto (default): partitioned for dense draws at 8+ ranks, replicated otherwise "
                        "(setup_mode: the 1-GPU emulation's slowest rank, round 4)")
    p.add_argument("--comm", choices=["runtime", "torch"], default="runtime",
                   help="multi-GPU collectives: the runtime's own RCCL communicators (exchange + row gather "
                        "enqueued from C++), or torch.distributed's (Python callbacks)")
    p.add_argument("--force-dist", action="store_true",
                   help="run the multi-GPU code path (RCCL process group, exchange, gather) even at 1 GPU")
    p.add_argument("--worker-timeout", type=float, default=0.0,
                   help="launcher-less N>1 run: stop the workers after this many seconds (0: no limit)")
    p.add_argument("--no-census", action="store_true",
                   help="skip the untimed winner-census frame (its instrumented k_tile would enter a rocprofv3 "
                        "kernel trace beside the timed launches; roofline.design then counts no winners)")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", PROFILE_TAG + "_pmc_c2.json"),
                   help="rocprofv3 PMC summary for roofline.traffic (tools/pmc_summary.py); quoted only when it "
                        "profiled this build (zenith_amd/buildinfo.py)")
    p.add_argument("--rocprof", default=os.path.join(ROOT, "profiles", PROFILE_TAG + "_kt_c2.json"),
                   help="rocprofv3 kernel-trace summary for kernels_rocprof (tools/kt_summary.py); same rule")
    return p.parse_args()


def build_profile(path, config):
    """A profile summary (PMC or kernel trace) of this build and config, or None
    with the reason (a profile of another build is stale: never quoted)."""
    if not os.path.exists(path):
        return None, f"{os.path.basename(path)}: missing"
    with open(path) as fh:
        prof = json.load(fh)
    if prof.get("config") != config:
        return None, f"{os.path.basename(path)}: config {prof.get('config')}"
    if prof.get("build") != buildinfo.source_hash():
        return None, f"{os.path.basename(path)}: build {prof.get('build')} is not this tree's {buildinfo.source_hash()}"
    return prof, os.path.basename(path)


SETUP_IN_BYTES = 12 + 3 * 12    # what k_setup_bin loads per triangle: 3 u32 indices + 3 float3 positions


def setup_mode(requested, world, triangles, width, height):
    """--setup auto: which setup a G-way tile-row shard uses.
    Partitioned setup ships 1/G of the set-up records per rank through an
    all-to-all, replicated setup repeats the whole setup on every rank; the
    1-GPU emulation of the slowest rank (profiles/r04_v3_bench_*shard8*) has
    partitioned ahead where setup dominates the rank -- dense draws, 256+
    triangles per 32x32 tile, at 8 ranks (C2: 35.8 vs 47.7 us) -- and replicated
    ahead elsewhere (C3, 122 per tile: 51.7 vs 54.3 us at 8 ranks; at 2 and 4
    ranks the route and exchange stages cost more than the setup they split)."""
    if requested != "auto":
        return requested
    tiles = ((width + shard.TILE - 1) // shard.TILE) * ((height + shard.TILE - 1) // shard.TILE)
    # (a quarter triangle per pixel of the tiled target)
    return "partitioned" if world >= 8 and 4 * triangles >= tiles * shard.TILE ** 2 else "replicated"


def winner_bytes(program, index_size=4):
    """Bytes the resolve gathers per winning primitive: its vertex
    ids, then the fragment program's attributes of its three vertices -- flat: the
    provoking colour; triangle: 3 colours; Blinn-Phong: 3 x (normal + colour), 24
    contiguous bytes per vertex; mesh: 3 x (normal + uv) plus the 48-B barycentric
    planes setup stored."""
    attrs = {scenes.PROGRAM_FLAT_COLOR: 12, scenes.PROGRAM_TRIANGLE: 36, scenes.PROGRAM_BLINN_PHONG: 72,
             scenes.PROGRAM_MESH: 3 * 20 + 48}[program]
    return 3 * index_size + attrs


def algorithmic_bytes(kernel, n_tris, b_in, pairs, pixels, n_route=0):
    """Per-launch algorithmic bytes of each pass.

    setup_bin: read what setup loads once (b_in per triangle: indices + positions,
               SETUP_IN_BYTES; the interleaved vertex lines also carry the other
               attributes, which the tile pass reads again for its winners),
               write one 32-B record per triangle and one 4-B bin entry per
               (tile, triangle) pair.
               With a partitioned setup n_tris is the rank's received records:
               read each 48-B route entry, write its 32-B record.
    route:     (partitioned setup) read indices + positions of the rank's range
               (12 + 3 * 12 B per triangle; the 48-B entries it writes are the
               receivers' reads).
    tile:      read each pair's bin entry + record once, write the colour + depth
               texel of every owned pixel (4 + 4 B).  (The winners' gathers are
               added by design_tile_bytes.)
    """
    if kernel == "setup_bin":
        if n_route:
            return n_tris * (shard.ENTRY_BYTES + RECORD_BYTES) + pairs * BIN_ENTRY_BYTES
        return n_tris * (b_in + RECORD_BYTES) + pairs * BIN_ENTRY_BYTES
    if kernel == "route":
        return n_route * 48
    if kernel == "tile":
        return pairs * (BIN_ENTRY_BYTES + RECORD_BYTES) + pixels * 8
    return 0


def design_tile_bytes(pairs, winners, per_winner, pixels):
    """The tile pass's design bytes, by request class: pairs x (4-B bin entry +
    32-B record) + winners x (vertex ids + attributes) + pixels x 8."""
    return {"bins": pairs * BIN_ENTRY_BYTES, "records": pairs * RECORD_BYTES,
            "winner_gathers": winners * per_winner, "stores": pixels * 8}


def host_cpus():
    """(threads, nproc --all, CPU model): SURVEY.md §8d times the baseline on all
    the host cores the process may use, i.e. what `nproc` reports (it honours the
    affinity mask and OMP_NUM_THREADS, 16 on the GPU box's share)."""
    import subprocess

    def run(*cmd):
        try:
            return subprocess.run(cmd, capture_output=True, text=True, timeout=10).stdout
        except (OSError, subprocess.SubprocessError):
            return ""
    try:
        threads = int(run("nproc").strip())
    except ValueError:
        threads = len(os.sched_getaffinity(0))
    try:
        total = int(run("nproc", "--all").strip())
    except ValueError:
        total = os.cpu_count() or threads
    model = next((ln.split(":", 1)[1].strip() for ln in run("lscpu").splitlines()
                  if ln.startswith("Model name")), "unknown")
    return max(1, threads), total, model


def cpu_baseline(scene, seconds, max_frames=500):
    """The CPU oracle (oracle/, OpenMP over tile-row bands) on the same scene:
    1 warm-up frame, then whole frames until ``seconds`` of wall time have passed."""
    from oracle import oracle
    threads, total, model = host_cpus()
    oracle.render(scene, nthreads=threads)  # warm-up
    frames = 0
    t0 = time.perf_counter()
    while frames < max_frames and (frames < 3 or time.perf_counter() - t0 < seconds):
        oracle.render(scene, nthreads=threads)
        frames += 1
    dt = time.perf_counter() - t0
    return {"value": round(scene.triangles * frames / dt / 1e6, 3), "unit": "Mtri/s", "cores": threads,
            "kind": "port", "nproc": threads, "nproc_all": total, "cpu_model": model,
            "sample": f"{frames} full frames of {scene.name} ({scene.triangles} tris, {scene.width}x{scene.height}) "
                      f"after 1 warm-up; {dt:.2f} s wall on {threads} threads (nproc; {total} CPUs online, {model})"}


class CaptureExchange(shard.Exchange):
    """--emulate-shard, partitioned setup: keeps this rank's send blocks (its
    routed records for every destination) and delivers nothing."""

    def __init__(self, device, world):
        super().__init__()
        self.device, self.world, self.sent = device, world, None

    def exchange(self, stream, send, recv, nbytes):
        with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=self.device)):
            self.sent = shard.device_bytes(send, nbytes * self.world, self.device).clone().view(self.world, nbytes)
            shard.device_bytes(recv, nbytes * self.world, self.device).zero_()


class ReplayExchange:
    """--emulate-shard, partitioned setup: delivers the blocks every source rank
    really routed to this rank (assembled from their captured sends), so the
    rank's binning and tile pass see its real received set.  The delivery is a
    device copy of those bytes on the runtime's route stream, enqueued by the
    runtime itself (zr_replay_exchange_fn: no Python callback per frame, which
    would make the emulated frame host-bound); the real all-to-all over xGMI is
    the driver's 8-GPU run to measure."""

    def __init__(self, device, recv_blocks: torch.Tensor):
        self.device, self.src = device, recv_blocks.reshape(-1).contiguous()

    def native(self):
        import ctypes
        desc = zr.zr_replay_exchange(self.src.data_ptr(), self.src.numel())
        return zr.lib().zr_replay_exchange_fn(), ctypes.addressof(desc), (desc, self.src)


def route_totals(sent: torch.Tensor):
    """Per-destination entry totals from a captured send buffer's block headers."""
    hdr = sent[:, :8].contiguous().cpu().view(torch.int32)
    return [int(t) for t in hdr[:, 1]]


def emulate(a, scene, cuda):
    """--emulate-shard G (1 GPU): every rank r of a G-way tile-row shard in turn,
    each timed like the bench's step (W warm-up, K frames between syncs), beside
    the unsharded frame T1 on the same GPU.  Partitioned setup: every source
    rank's route runs first (captured), each rank then receives exactly the
    records the others routed to it.  Reports T1, every rank's frame time, the
    speed-up T1 / max-rank time and the 6x target; the row gather is excluded
    (modelled only) and so is the all-to-all's time on the wire (a device copy
    of the received bytes stands in for it)."""
    G = a.emulate_shard
    W, H, N = scene.width, scene.height, scene.triangles
    a.setup = setup_mode(a.setup, G, N, W, H)
    dev = rhi.RenderDevice(0)
    color_t = torch.zeros((H, W * 4), dtype=torch.uint8, device=cuda)
    depth_t = torch.zeros((H, W), dtype=torch.float32, device=cuda)
    torch.cuda.synchronize()
    color = rhi.Texture(dev, rhi.TextureDesc.new_color("frame.color", W, H, scene.color_format), color_t.data_ptr())
    depth = rhi.Texture(dev, rhi.TextureDesc.new_depth("frame.depth", W, H), depth_t.data_ptr())
    rend = renderer.SceneRenderer(dev, scene)

    def timed(enc):
        for _ in range(a.warmup):
            dev.submit(enc)
            dev.wait_idle()  # (a sync per warm-up frame, as in the bench's timed_pass)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            dev.submit(enc)
        dev.wait_idle()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    def kernels(enc):
        dev.kernel_times(reset=True)
        dev.set_profiling(True)
        for _ in range(a.steps):
            dev.submit(enc)
        dev.wait_idle()
        dev.set_profiling(False)
        return {k: round(ms * 1e3 / max(n, 1), 2) for k, (ms, n) in dev.kernel_times().items()}

    enc1 = rend.record(color, depth, encoder=rhi.CommandEncoder(dev))
    t1 = timed(enc1)
    enc1.destroy()
    part = a.setup == "partitioned"
    cap = 0
    recv = None
    if part:
        _, span, _, _ = shard.route_geometry(N, G)

        def capture(c):
            sends = []
            for s in range(G):
                ex = CaptureExchange(cuda, G)
                enc = rend.record(color, depth, shard=(s, G, ex, c), encoder=rhi.CommandEncoder(dev))
                dev.submit(enc)
                dev.wait_idle()
                sends.append(ex.sent)
                enc.destroy()
            return sends
        # exact block capacity for this static scene: the largest routed total
        sends = capture(span)
        cap = max(max(route_totals(x)) for x in sends) + 64
        sends = capture(cap)
        recv = [torch.stack([sends[s][r] for s in range(G)]) for r in range(G)]
    ranks = []
    for r in range(G):
        sh = (r, G, ReplayExchange(cuda, recv[r]), cap) if part else (r, G)
        enc = rend.record(color, depth, shard=sh, encoder=rhi.CommandEncoder(dev))
        tr = timed(enc)
        kt = kernels(enc)
        st = dev.last_draw_stats()
        pixels = shard.owned_pixels(W, H, r, G)
        ranks.append({"rank": r, "ms": round(tr * 1e3, 4), "kernels_us": kt, "bin_pairs": st["bin_pairs"],
                      "triangles_setup": st["triangles_setup"], "pixels": pixels,
                      "route_fallback_draws": st["route_fallback_draws"]})
        enc.destroy()
    worst = max(ranks, key=lambda x: x["ms"])
    # the tile gather, modelled: the largest peer's pixels into rank 0
    # over one xGMI link at ~153 GB/s, overlapped with the next frame
    peer_px = max((shard.owned_pixels(W, H, r, G) for r in range(1, G)), default=0)
    gather_us = peer_px * 4 / 153e9 * 1e6
    b_in = scenes.config_bytes_per_triangle(a.config)
    n_route = shard.route_range(N, worst["rank"], G)
    rank_bytes = (((n_route[1] - n_route[0]) * b_in + worst["triangles_setup"] * shard.ENTRY_BYTES) if part
                  else N * b_in) + worst["pixels"] * 8
    out = {"metric": METRIC + " [1-GPU emulation of a tile-row shard; diagnostic, not the bench line]",
           "config": {"workload": f"{a.config}: {N} tris, {W}x{H}", "shards": G, "setup": a.setup},
           "t1_ms": round(t1 * 1e3, 4), "rank_ms": [x["ms"] for x in ranks],
           "max_rank": worst["rank"], "max_rank_ms": worst["ms"],
           "speedup": round(t1 / (worst["ms"] * 1e-3), 3), "target_speedup": 6.0 if G == 8 else None,
           "value_emulated": round(N / (worst["ms"] * 1e-3) / 1e6, 2), "unit": "Mtri/s",
           "excluded": "row gather (modelled below, overlapped with the next frame) and the all-to-all's wire "
                       "time (a device copy of the received bytes stands in)",
           "gather_model_us": round(gather_us, 1), "route_capacity": cap or None,
           "rank_alg_bytes": rank_bytes, "rank_gbps": round(rank_bytes / (worst["ms"] * 1e-3) / 1e9, 1),
           "ranks": ranks, "steps": a.steps, "warmup": a.warmup}
    for t in (color, depth):
        t.destroy()
    dev.close()
    return out


# ------------------------------------------------------------ worker launcher
def worker_commands(n, argv, port, base_env=None, script=None):
    """The N worker processes of a launcher-less multi-GPU run: this script with
    the same arguments, one rank per GPU (LOCAL_RANK = RANK = device index) and
    the rendezvous in the environment, as torch.distributed.run would set it."""
    base = dict(os.environ if base_env is None else base_env)
    cmds = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        cmds.append(([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv), env))
    return cmds


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def run_workers(cmds, out=None, timeout=None, poll=0.2):
    """Starts every (cmd, env) as a child process (never exec: the parent may not
    replace itself), rank 0's stdout into a file that is relayed to ``out`` when
    all are done, the others' stdout onto stderr.  When a worker fails (non-zero
    exit) or ``timeout`` seconds pass, the rest are stopped -- their own process
    groups, SIGTERM then SIGKILL -- since they may sit in a collective waiting for
    the failed one.  Returns 0 or the first failure's exit status (124 on timeout)."""
    import signal
    import subprocess
    import tempfile
    out = out or sys.stdout
    procs = []
    with tempfile.TemporaryFile("w+") as rank0_out:
        for i, (cmd, env) in enumerate(cmds):
            procs.append(subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=rank0_out if i == 0 else sys.stderr,
                                          start_new_session=True))
        t0 = time.monotonic()
        rc = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]  # -N: killed by signal N
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                rc = 124
                break
            time.sleep(poll)
        if rc:
            for sig, grace in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 5.0)):
                for p in procs:
                    if p.poll() is None:
                        try:
                            os.killpg(p.pid, sig)
                        except ProcessLookupError:
                            pass
                t1 = time.monotonic()
                while any(p.poll() is None for p in procs) and time.monotonic() - t1 < grace:
                    time.sleep(0.1)
            for p in procs:
                if p.poll() is None:
                    p.wait()
            print(f"bench: worker exit codes {[p.returncode for p in procs]}", file=sys.stderr)
        rank0_out.seek(0)
        text = rank0_out.read()
    if text:
        out.write(text)
        out.flush()
    return rc


def launch_workers(a, argv):
    cmds = worker_commands(a.gpus, argv, free_port())
    return run_workers(cmds, timeout=a.worker_timeout or None)


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus > 1 or a.force_dist):
        # no launcher: this process stays off the GPU and runs one worker per GPU
        raise SystemExit(launch_workers(a, sys.argv[1:]))
    # The JSON line is the only thing on stdout: libraries that print to fd 1
    # (RCCL's version banner) are sent to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    torch.cuda.set_device(local)
    cuda = torch.device("cuda", local)
    distributed = world > 1 or a.force_dist
    if distributed:
        dist.init_process_group("nccl", device_id=cuda)

    scene = scenes.config_scene(a.config)
    W, H, N = scene.width, scene.height, scene.triangles
    if a.emulate_shard <= 1:
        a.setup = setup_mode(a.setup, world, N, W, H)
    if a.emulate_shard > 1:
        if distributed:
            raise SystemExit("--emulate-shard is a 1-GPU diagnostic")
        print(json.dumps(emulate(a, scene, cuda)), file=json_out, flush=True)
        return
    dev = rhi.RenderDevice(local)
    # Multi-GPU frames ping-pong between two colour targets: frame f+1 renders
    # while frame f's rows are gathered on a stream of their own.
    nbuf = 2 if distributed else 1
    color_ts = [torch.zeros((H, W * 4), dtype=torch.uint8, device=cuda) for _ in range(nbuf)]
    color_t = color_ts[0]
    depth_t = torch.zeros((H, W), dtype=torch.float32, device=cuda)
    torch.cuda.synchronize()
    colors = [rhi.Texture(dev, rhi.TextureDesc.new_color(f"frame.color{i}", W, H, scene.color_format), t.data_ptr())
              for i, t in enumerate(color_ts)]
    color = colors[0]
    depth = rhi.Texture(dev, rhi.TextureDesc.new_depth("frame.depth", W, H), depth_t.data_ptr())
    # copy 0 is the warm (value) pass's geometry; copies 0..K-1 cycle in the cold pass
    rs = [renderer.SceneRenderer(dev, scene) for _ in range(max(1, a.cold_copies))]
    shard_g = world
    exchange = None
    runtime_comm = distributed and a.comm == "runtime"
    if runtime_comm:
        # every rank must be able to load RCCL before any joins a communicator
        # (a rank that cannot would leave the others blocked in the init)
        ok = torch.tensor([1 if shard.runtime_rccl_available() else 0], device=cuda)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()):
            shard.init_runtime_rccl(dev, rank, world)
        else:
            runtime_comm = False
            print("bench: the runtime cannot load RCCL on every rank; using torch.distributed's", file=sys.stderr)
    if a.setup == "partitioned" and runtime_comm:
        exchange = "rccl"
    elif a.setup == "partitioned" and distributed:
        # its own communicator (and so its own RCCL stream): the exchange of frame
        # f+1 must not queue behind the row gather of frame f
        exchange = shard.RcclExchange(cuda, group=dist.new_group(list(range(world))))
    cap = 0
    if exchange is not None:
        # exchange block capacity: this static scene's largest routed total over all
        # ranks, from one captured route per rank (nothing delivered), max-reduced so
        # every rank records the same capacity (zr_cmd_set_route_capacity)
        _, span, _, _ = shard.route_geometry(N, shard_g)
        cx = CaptureExchange(cuda, shard_g)
        enc = rs[0].record(color, depth, shard=(rank, shard_g, cx, span), encoder=rhi.CommandEncoder(dev))
        dev.submit(enc)
        dev.wait_idle()
        enc.destroy()
        top = torch.tensor([max(route_totals(cx.sent)) + 64], device=cuda)
        dist.all_reduce(top, op=dist.ReduceOp.MAX)
        cap = int(top.item())
    sh = (rank, shard_g, exchange, cap) if exchange is not None else ((rank, shard_g) if shard_g > 1 else None)
    # encs[copy][target]: frame f draws geometry copy f % K into target f % nbuf
    encs = [[r.record(c, depth, shard=sh, encoder=rhi.CommandEncoder(dev)) for c in colors] for r in rs]
    gather = shard.TileGather(W, H, 4, rank, world, cuda) if distributed and not runtime_comm else None
    # Multi-GPU: torch's current stream is the runtime's main stream, so frames,
    # exchanges and gathers are ordered by streams and events, never a host wait.
    main_stream = torch.cuda.ExternalStream(dev.stream, device=cuda)
    stream_ctx = torch.cuda.stream(main_stream) if distributed else None
    if stream_ctx is not None:
        stream_ctx.__enter__()
    gstream = torch.cuda.Stream(cuda) if gather is not None else None
    gdone = [None] * nbuf
    frame = [0]

    host_t = [0.0, 0.0]  # host seconds in submit / gather (diagnostic)

    def step(copies):
        b = frame[0] % nbuf
        enc = encs[frame[0] % copies][b]
        frame[0] += 1
        if gdone[b] is not None:
            main_stream.wait_event(gdone[b])  # the gather of frame f-2 read this target
        h0 = time.perf_counter()
        dev.submit(enc)
        h1 = time.perf_counter()
        host_t[0] += h1 - h0
        if runtime_comm:
            dev.gather_tile_rows(colors[b], 0)  # RCCL on the runtime's gather stream
            host_t[1] += time.perf_counter() - h1
        if gather is not None:
            ev = torch.cuda.Event()
            ev.record(main_stream)
            gstream.wait_event(ev)
            with torch.cuda.stream(gstream):
                gather.gather(color_ts[b])
            gdone[b] = torch.cuda.Event()
            gdone[b].record(gstream)

    def timed_pass(copies):
        """W untimed frames, then K frames bracketed by barrier + synchronize;
        returns (max-over-ranks seconds, host enqueue seconds of this rank)."""
        frame[0] = 0
        for _ in range(a.warmup):
            step(copies)
            # each warm-up frame ends at a sync point, as a presented frame does: the
            # runtime sizes bins and jobs, and picks the tile edge, from what the
            # draws it has seen measured (a shape that changes its tile edge is
            # measured again at the next sync)
            dev.wait_idle()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        host_t[0] = host_t[1] = 0.0
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(copies)
        t_enq = time.perf_counter()  # host enqueue time of the K frames (diagnostic: host-bound if ~ wall)
        dev.wait_idle()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        t1 = time.perf_counter()
        el = torch.tensor([t1 - t0], dtype=torch.float64, device=cuda)
        if distributed:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()), t_enq - t0

    # warm pass (the headline value): one geometry copy, its 120 MB (C2) stays in
    # the Infinity Cache from frame to frame, as in the reference's static scene
    elapsed, enq = timed_pass(1)
    host_submit, host_gather = host_t[0], host_t[1]
    # cold pass: K copies cycled, so every frame's vertex reads come from HBM
    elapsed_cold = timed_pass(len(rs))[0] if len(rs) > 1 else None

    # Per-kernel durations: the same K steps again with HIP events around every
    # launch on the raster stream (events sit between the kernels, so this pass runs
    # the command list eagerly instead of as one graph; its wall time is reported as
    # ms_per_step_profiled, not used for `value`).
    dev.kernel_times(reset=True)
    dev.set_profiling(True)
    # frame-boundary events on the raster stream: per-frame intervals (median / p90,
    # SURVEY.md §8d) of the queued, steady-state frame stream
    fev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    fev[0].record(main_stream)
    tp0 = time.perf_counter()
    frame[0] = 0
    for i in range(a.steps):
        step(1)
        fev[i + 1].record(main_stream)
    dev.wait_idle()
    tp1 = time.perf_counter()
    torch.cuda.synchronize()
    frame_ms = sorted(fev[i].elapsed_time(fev[i + 1]) for i in range(a.steps))
    dev.set_profiling(False)
    kt = dev.kernel_times()
    stats = dev.last_draw_stats()
    # winner census: one more (untimed) frame whose resolve marks each primitive
    # that wins a pixel, for the tile pass's per-winner gather bytes
    winners = None
    if not a.no_census:
        dev.set_profiling(True, census=True)
        frame[0] = 0
        step(1)
        dev.wait_idle()
        winners = dev.last_draw_stats()["winners"]
        dev.set_profiling(False)
    dev.kernel_times(reset=True)
    pairs = stats["bin_pairs"]
    pixels = shard.owned_pixels(W, H, rank, shard_g)
    b_in = scenes.config_bytes_per_triangle(a.config)
    n_setup, n_route = N, 0
    index_size = 4 if scene.index_type == scenes.INDEX_U32 else (2 if scene.index_type == scenes.INDEX_U16 else 0)
    if exchange is not None:  # this rank's range and the triangles it received
        lo, hi = shard.route_range(N, rank, shard_g)
        n_route = hi - lo
        n_setup = stats["triangles_setup"]
    kernels = {}
    for name, (ms, n) in kt.items():
        avg_us = ms * 1e3 / max(n, 1)
        by = algorithmic_bytes(name, n_setup, SETUP_IN_BYTES, pairs, pixels, n_route)
        kernels[name] = {"avg_us": round(avg_us, 2), "launches": n, "alg_bytes": by,
                         "gbps": round(by / (avg_us * 1e-6) / 1e9, 1) if by and avg_us > 0 else None}
    launches = {k: v for k, v in kt.items() if k != "exchange"}  # "exchange": the all-to-all, not a kernel
    dom = max(launches, key=lambda k: launches[k][0]) if launches else "tile"
    dk = kernels.get(dom, {})
    traffic = None
    traffic_classes = None
    pmc, pmc_src = build_profile(a.pmc, a.config)  # measured on the warm pass's single copy, like `achieved`
    if pmc and dom in pmc.get("kernels", {}):
        traffic = pmc["kernels"][dom]["hbm_bytes_per_launch"]
        traffic_classes = pmc["kernels"][dom].get("classes")
    kt_prof, kt_src = build_profile(a.rocprof, a.config)
    kernels_rocprof = ({k: {"avg_us": v["avg_us"], "calls": v["calls"]} for k, v in kt_prof["kernels"].items()}
                       if kt_prof else None)
    achieved = dk.get("gbps") or 0.0
    # SURVEY.md §8d's own fragment-pass figure (64-B records: 68 B per pair) beside
    # this design's minimum (32-B compact records: 36 B per pair)
    survey_bytes = pairs * SURVEY_PAIR_BYTES + pixels * 8
    tile_us = kernels.get("tile", {}).get("avg_us") or 0.0
    achieved_survey = round(survey_bytes / (tile_us * 1e-6) / 1e9, 1) if tile_us > 0 else None
    # the design's own request classes (bins, records, winners' gathers, stores)
    per_winner = winner_bytes(scene.program, index_size)
    design = design_tile_bytes(pairs, winners or 0, per_winner, pixels)
    design_total = sum(design.values())
    achieved_design = round(design_total / (tile_us * 1e-6) / 1e9, 1) if tile_us > 0 else None

    ms_per_step = elapsed / a.steps * 1e3
    value = N * a.steps / elapsed / 1e6
    frame_bytes = N * b_in + W * H * 8
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mtri/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (SplitMix64 triangle soup, SURVEY.md §8d)",
        **({"value_cold": round(N * a.steps / elapsed_cold / 1e6, 2),
            "ms_per_step_cold": round(elapsed_cold / a.steps * 1e3, 4),
            "cold_copies": len(rs)} if elapsed_cold else {}),
        "config": {"workload": (f"{a.config}: {N} tris (reference asset, mesh.slang camera), {W}x{H}, "
                                f"D32 GREATER (reverse-Z), B8G8R8A8_SRGB" if scene.program == scenes.PROGRAM_MESH else
                                f"{a.config}: {N} tris soup, {W}x{H}, "
                                f"{'Blinn-Phong' if scene.program == scenes.PROGRAM_BLINN_PHONG else 'flat'} "
                                f"+ D32 LESS, B8G8R8A8_SRGB"),
                   "triangles": N, "width": W, "height": H, "tile": shard.TILE, "input_copies": 1,
                   "parallelism": f"tile-rows x{world}" + (
                       f", {a.setup} setup" + (" (RCCL all-to-all)" if exchange is not None else "")
                       + f" + RCCL row gather ({'runtime' if runtime_comm else 'torch'} communicators)"
                       if distributed else "")},
        "fps": round(1e3 / ms_per_step, 2),
        "ms_per_step_profiled": round((tp1 - tp0) / a.steps * 1e3, 4),
        "host_enqueue_ms_per_step": round(enq / a.steps * 1e3, 4),
        "frame_ms_median_profiled": round(frame_ms[len(frame_ms) // 2], 4),
        "frame_ms_p90_profiled": round(frame_ms[min(len(frame_ms) - 1, (9 * len(frame_ms)) // 10)], 4),
        "host_submit_ms_per_step": round(host_submit / a.steps * 1e3, 4),
        "host_gather_ms_per_step": round(host_gather / a.steps * 1e3, 4),
        "frame_alg_bytes": frame_bytes,
        "frame_gbps": round(frame_bytes / (ms_per_step * 1e-3) / 1e9, 1),
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "peak_source": "MI355X_MICROARCH.md measured float4 copy (SURVEY.md §8d)",
                     "peak_spec": HBM_SPEC_GBPS, "frac_spec": round(achieved / HBM_SPEC_GBPS, 4),
                     # (the fragment pass's own figures, whichever kernel is the
                     # dominant one: with setup overlapped, C2's setup spans longer)
                     "tile_fields_note": "tile_*, *_per_pair, *_survey and design: k_tile over its own duration",
                     "tile_achieved": kernels.get("tile", {}).get("gbps"),
                     "tile_frac": (round(kernels["tile"]["gbps"] / HBM_PEAK_GBPS, 4)
                                   if kernels.get("tile", {}).get("gbps") else None),
                     "alg_bytes_per_pair": BIN_ENTRY_BYTES + RECORD_BYTES,
                     "survey_bytes_per_pair": SURVEY_PAIR_BYTES,
                     "achieved_survey": achieved_survey,
                     "frac_survey": round(achieved_survey / HBM_PEAK_GBPS, 4) if achieved_survey else None,
                     "design": {"bytes": design_total, "classes": design, "winners": winners,
                                "bytes_per_winner": per_winner, "achieved": achieved_design,
                                "frac": round(achieved_design / HBM_PEAK_GBPS, 4) if achieved_design else None},
                     "traffic_classes": traffic_classes, "traffic_source": pmc_src},
        "kernels": kernels,
        # the same kernels' rocprofv3 kernel-trace averages for this build (no events
        # between launches), beside the event-timed `kernels` above
        "kernels_rocprof": kernels_rocprof, "kernels_rocprof_source": kt_src,
        "build": buildinfo.source_hash(),
        "bin_pairs": pairs,
        "triangles_setup": stats["triangles_setup"],
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene, a.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if stream_ctx is not None:
        dev.wait_idle()
        stream_ctx.__exit__(None, None, None)
    for row in encs:
        for e in row:
            e.destroy()
    for c in colors:
        c.destroy()
    depth.destroy()
    dev.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
