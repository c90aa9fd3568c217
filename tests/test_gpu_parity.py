"""GPU parity: the HIP draw path (through the C ABI) against the CPU oracle.

Bar (north_star / DESIGN.md §5): coverage, depth bits and 8-bit colour codes are
bit-exact; float colour (R32G32B32A32_SFLOAT targets) is bit-exact as well since
both sides evaluate the same explicitly ordered float arithmetic — the test
tolerance below is 0 ULP, tighter than the north star's 1 ULP.
"""
import numpy as np
import pytest

from oracle import oracle
from zenith_amd import renderer, rhi, scenes, shard, zr

pytestmark = pytest.mark.gpu

FLOAT_ULP_TOL = 0  # north_star allows 1 ULP on shaded float colour; we hold 0


def owned(scene, shard_):
    """[H, W] mask of the pixels a shard owns (shard.owned_mask; all without one)."""
    if shard_ is None:
        return np.ones((scene.height, scene.width), dtype=bool)
    return shard.owned_mask(scene.width, scene.height, shard_[0], shard_[1])


def assert_parity(device, scene, shard=None, **kw):
    gc, gd = renderer.render_scene(device, scene, shard=shard, **kw)
    oc, od = oracle.render(scene, shard=shard or (0, 1), tile_size=zr.tile_size(), **kw)
    rows = owned(scene, shard)
    full_c, full_d = gc, gd
    gc, oc = gc[rows], oc.reshape(scene.height, scene.width, -1)[rows]
    if scene.color_format == zr.FORMAT_R32G32B32A32_SFLOAT:
        g = gc.view(np.float32).reshape(-1)
        o = oc.view(np.float32).reshape(-1)
        ulp = np.abs(g.view(np.int32).astype(np.int64) - o.view(np.int32).astype(np.int64))
        assert ulp.max() <= FLOAT_ULP_TOL, f"max ulp {ulp.max()}"
    else:
        diff = np.argwhere(np.any(gc != oc, axis=-1))
        assert diff.size == 0, f"{len(diff)} pixels differ, first {diff[:5].tolist()}: " \
                               f"gpu {gc[diff[0][0]]} oracle {oc[diff[0][0]]}"
    if scene.depth:
        gdb, odb = gd[rows].view(np.uint32), od[rows].view(np.uint32)
        bad = np.argwhere(gdb != odb)
        assert bad.size == 0, f"{len(bad)} depth values differ, first {bad[:5].tolist()}"
    return full_c, full_d


def test_triangle_reference_scene(device):
    """The reference's only scene (triangle.rs) at T=0 on B8G8R8A8_SRGB."""
    gc, _ = assert_parity(device, scenes.triangle_scene())
    bg = np.all(gc == np.array([89, 89, 89, 255], np.uint8), axis=-1)
    assert int((~bg).sum()) == 38400


def test_triangle_renderer_mirror(device):
    """TriangleRenderer (triangle.rs call sequence) renders the golden image."""
    tr = renderer.TriangleRenderer(device)
    tex = rhi.Texture(device, rhi.TextureDesc.new_color("swapchain", 640, 480, zr.FORMAT_B8G8R8A8_SRGB))
    enc = tr.render_to(tex, 640, 480, elapsed=0.0)
    device.submit_and_wait(enc)
    img = tex.read()
    oc, _ = oracle.render(scenes.triangle_scene())
    assert np.array_equal(img, oc)
    tex.destroy()


@pytest.mark.parametrize("t", [0.0, 1.25, 7.5])
def test_triangle_animated(device, t):
    assert_parity(device, scenes.triangle_scene(time=t))


def test_cube(device):
    assert_parity(device, scenes.cube_scene())


@pytest.mark.parametrize("program", [scenes.PROGRAM_FLAT_COLOR, scenes.PROGRAM_BLINN_PHONG, scenes.PROGRAM_TRIANGLE])
def test_small_soup(device, program):
    s = scenes.soup_scene(11, 2000, 256, 192, 10.0, program)
    assert_parity(device, s)


@pytest.mark.parametrize("op,write", [(scenes.OP_LESS, True), (scenes.OP_LEQUAL, True), (scenes.OP_GREATER, True),
                                      (scenes.OP_GEQUAL, True), (scenes.OP_ALWAYS, True), (scenes.OP_LESS, False),
                                      (scenes.OP_EQUAL, True), (scenes.OP_NEVER, True)])
def test_depth_modes(device, op, write):
    s = scenes.soup_scene(12, 3000, 200, 160, 14.0, scenes.PROGRAM_FLAT_COLOR)
    s.depth_op, s.depth_write = op, write
    if op in (scenes.OP_GREATER, scenes.OP_GEQUAL):
        s.depth_clear = 0.0
    assert_parity(device, s)


def test_c1_scaled(device):
    s = scenes.config_scene("c1", n=20000, width=640, height=360)
    assert_parity(device, s)


# ---------------------------------------------------------- coverage of paths
def test_large_triangles_wave_path(device):
    """Primitives beyond the 64-px "small" bound take the wave-cooperative path."""
    s = scenes.soup_scene(13, 400, 512, 384, 150.0, scenes.PROGRAM_BLINN_PHONG)
    assert_parity(device, s)


@pytest.mark.parametrize("seed", [0, 1])
def test_large_slivers_lane_walk(device, seed):
    """Long thin triangles (20 px to ~20,000 px, most of them past the screen, 0.5-6
    px wide, every orientation, some fanned around a shared vertex): large
    primitives that k_tile's lane walk takes tile by tile when their edge values
    there fit int32 (lane_walk_fits) and the wave path takes elsewhere."""
    g = np.random.default_rng(40 + seed)
    W, H, n = 1024, 768, 2400
    c = g.uniform(-1.2, 1.2, (n, 2))
    ang = g.uniform(0, 2 * np.pi, n)
    length = np.exp(g.uniform(np.log(20.0), np.log(20000.0), n)) / (W / 2)   # NDC units
    width = g.uniform(0.5, 6.0, n) / (H / 2)
    d = np.stack([np.cos(ang), np.sin(ang)], 1)
    nrm = np.stack([-d[:, 1], d[:, 0]], 1)
    p0 = c - d * length[:, None] / 2
    p1 = c + d * length[:, None] / 2
    p2 = c + nrm * width[:, None] * g.choice([-1.0, 1.0], (n, 1))
    fan = g.random(n) < 0.2  # slivers sharing vertex 0 (a cap's spokes)
    p0[fan] = np.array([0.1, -0.05])
    z = g.uniform(0.05, 0.95, (n, 3))
    pos = np.stack([p0, p1, p2], 1)
    verts = np.concatenate([pos, z[..., None], g.uniform(0, 1, (n, 3, 3))], axis=2).reshape(-1, 6)
    s = scenes.Scene(f"slivers_{seed}", W, H, scenes.PROGRAM_FLAT_COLOR, verts.astype(np.float32),
                     np.arange(3 * n, dtype=np.uint32), depth=True)
    assert_parity(device, s)


def test_wave_queue_overflow(device):
    """More large primitives in one tile segment than k_tile's wave-path queue
    holds (kBigQueue = 512): 1100 screen-covering triangles, none a sliver, so
    every tile's batch straddles the queue's end and the waves sweep the rest
    themselves (a straddling batch once left queue slots unfilled)."""
    g = np.random.default_rng(77)
    n = 1100
    pos = g.uniform(-3.0, 3.0, (n, 3, 2))
    z = g.uniform(0.0, 1.0, (n, 3, 1))
    verts = np.concatenate([pos, z, g.uniform(0, 1, (n, 3, 3))], axis=2).reshape(-1, 6)
    s = scenes.Scene("wave_queue_overflow", 256, 192, scenes.PROGRAM_FLAT_COLOR, verts.astype(np.float32),
                     np.arange(3 * n, dtype=np.uint32), depth=True)
    assert_parity(device, s)


def test_mixed_sizes(device):
    a = scenes.soup_scene(14, 1500, 300, 200, 6.0, scenes.PROGRAM_FLAT_COLOR)
    b = scenes.soup_scene(15, 60, 300, 200, 120.0, scenes.PROGRAM_FLAT_COLOR)
    v = np.concatenate([a.vertices[:1500], b.vertices[:60], a.vertices[1500:]])
    s = scenes.Scene("mixed", 300, 200, scenes.PROGRAM_FLAT_COLOR, v, np.arange(v.shape[0], dtype=np.uint32),
                     depth=True)
    assert_parity(device, s)


def test_bin_overflow_spill(monkeypatch):
    """A draw with more (tile, primitive) pairs than the bin buffer holds is
    rasterized exactly by k_tile's all-records scan; the runtime then grows the
    buffer, and the next draw reads tile lists again."""
    monkeypatch.setenv("ZR_BIN_CAPACITY", "1024")
    dev = rhi.RenderDevice(0)
    try:
        s = scenes.soup_scene(16, 3000, 640, 480, 40.0, scenes.PROGRAM_FLAT_COLOR)
        assert_parity(dev, s)
        st = dev.last_draw_stats()
        assert st["overflowed_draws"] == 1 and st["bin_pairs"] > 1024 and st["bin_capacity"] >= st["bin_pairs"]
        assert_parity(dev, s)
        assert dev.last_draw_stats()["overflowed_draws"] == 1
    finally:
        dev.close()
    dev = rhi.RenderDevice(0)
    try:  # the wave path (large primitives) while spilling
        assert_parity(dev, scenes.soup_scene(17, 300, 512, 384, 150.0, scenes.PROGRAM_BLINN_PHONG))
        assert dev.last_draw_stats()["overflowed_draws"] == 1
    finally:
        dev.close()


def crowded_tile_scene():
    """9000 small triangles in the 32x32 tile (5, 7) of a 640x480 target among
    3000 spread ones: one tile list ~60x the mean."""
    w, h = 640, 480
    dense = scenes.soup_arrays(41, 9000, 32, 32, 2.0, False)  # 9000 small triangles, most in one 32x32 tile
    dense[:, 0] = dense[:, 0] * (32.0 / w) + (2 * 32 * 5 + 32) / w - 1.0  # tile (5, 7)
    dense[:, 1] = dense[:, 1] * (32.0 / h) + (2 * 32 * 7 + 32) / h - 1.0
    sparse = scenes.soup_arrays(42, 3000, w, h, 10.0, False)
    v = np.concatenate([sparse[:4500], dense, sparse[4500:]]).astype(np.float32)
    return scenes.Scene("slab_overflow", w, h, scenes.PROGRAM_FLAT_COLOR, v, np.arange(len(v), dtype=np.uint32),
                        depth=True)


def test_slab_overflow_one_tile():
    """A crowded tile whose list outgrows its slab keeps its excess in pool runs
    (DrawParams::runs), read after the slab part, with no record scan: on the
    first draw (slabs of a third of the buffer) and on later ones (slabs of the
    measured target, bin_slab_target)."""
    s = crowded_tile_scene()
    dev = rhi.RenderDevice(0)
    try:
        for _ in range(3):
            assert_parity(dev, s)
            st = dev.last_draw_stats()
            assert st["overflowed_draws"] == 0, st
            assert st["bin_pool_runs"] > 0 and 0 < st["bin_pool_pairs"] < st["bin_pairs"], st
    finally:
        dev.close()


@pytest.mark.parametrize("slab", ["0", "24", "300"])
def test_pool_runs(monkeypatch, slab):
    """Slabs forced small (ZR_BIN_SLAB; 0: every pair in a pool run): every tile
    list is read through its run table -- soups on 256- and 512-thread tiles with
    the record table on and off, a tile-row shard, the camera program's fans, the
    wave path, lists of several 1024-entry segments, records-mode (partitioned)
    setup and repeated frames -- exact, with no record scan."""
    monkeypatch.setenv("ZR_BIN_SLAB", slab)
    for nt, table in (("256", "1"), ("512", "1"), ("512", "0")):
        monkeypatch.setenv("ZR_TILE_NT", nt)
        monkeypatch.setenv("ZR_REC_TABLE", table)
        dev = rhi.RenderDevice(0)
        try:
            assert_parity(dev, scenes.config_scene("c1", n=30000, width=640, height=360))
            assert_parity(dev, scenes.soup_scene(18, 4000, 512, 384, 12.0, scenes.PROGRAM_BLINN_PHONG), shard=(1, 3))
            assert_parity(dev, scenes.soup_scene(17, 300, 512, 384, 150.0, scenes.PROGRAM_FLAT_COLOR))
            assert_parity(dev, crowded_tile_scene())
            assert dev.last_draw_stats()["bin_pool_runs"] > 0
            assert_parity(dev, scenes.cerberus_scene(640, 480))
            assert dev.last_draw_stats()["overflowed_draws"] == 0
        finally:
            dev.close()
    monkeypatch.delenv("ZR_TILE_NT")
    monkeypatch.delenv("ZR_REC_TABLE")
    dev = rhi.RenderDevice(0)
    try:
        # frames back to back: each tile pass resets the run words the next
        # draw's setup fills (a tile resetting its run word before every wave had
        # read it sent the others past its slab)
        s = scenes.config_scene("c2", n=200_000)
        gc, gd = renderer.render_scene(dev, s, frames=8)
        oc, od = oracle.render(s, nthreads=16)
        assert np.array_equal(gc, oc) and np.array_equal(gd.view(np.uint32), od.view(np.uint32))
        assert dev.last_draw_stats()["overflowed_draws"] == 0
    finally:
        dev.close()
    assert_partitioned_parity(scenes.soup_scene(70, 20000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG), 3)


@pytest.mark.parametrize("jobs", ["256", "1000"])
def test_tile_jobs(monkeypatch, jobs):
    """Tile lists split into jobs of ZR_JOBS entries, each its own k_tile block
    that stores its LDS keys to a key buffer of its own; the last job of a tile
    (a ticket) folds the other jobs' buffers into its keys with a min and
    resolves it.
    Exact on 256- and 512-thread tiles with the record table on and off, a
    tile-row shard, the camera program's fans, the wave path, a crowded tile
    (~35 jobs), depth ops without writes (initial-depth tiles), jobs over pool
    runs (slabs forced small), repeated frames and records-mode setup."""
    monkeypatch.setenv("ZR_JOBS", jobs)
    for nt, table, slab in (("256", "1", None), ("512", "1", None), ("512", "0", "24")):
        monkeypatch.setenv("ZR_TILE_NT", nt)
        monkeypatch.setenv("ZR_REC_TABLE", table)
        if slab:
            monkeypatch.setenv("ZR_BIN_SLAB", slab)
        dev = rhi.RenderDevice(0)
        try:
            assert_parity(dev, scenes.config_scene("c1", n=30000, width=640, height=360))
            assert_parity(dev, scenes.soup_scene(18, 4000, 512, 384, 12.0, scenes.PROGRAM_BLINN_PHONG), shard=(1, 3))
            assert_parity(dev, scenes.soup_scene(17, 300, 512, 384, 150.0, scenes.PROGRAM_FLAT_COLOR))
            assert_parity(dev, crowded_tile_scene())
            assert dev.last_draw_stats()["tile_jobs"] >= 4  # (the crowded tile: ~8000 entries)
            assert_parity(dev, scenes.cerberus_scene(640, 480))
            for op, clear in ((scenes.OP_LEQUAL, 1.0), (scenes.OP_GREATER, 0.0)):
                s = scenes.soup_scene(72, 6000, 200, 160, 14.0, scenes.PROGRAM_FLAT_COLOR)
                s.depth_op, s.depth_clear = op, clear
                assert_parity(dev, s)
                s.depth_write = False  # last-wins keys over the loaded depth
                assert_parity(dev, s)
            assert dev.last_draw_stats()["overflowed_draws"] == 0
        finally:
            dev.close()
    for k in ("ZR_TILE_NT", "ZR_REC_TABLE", "ZR_BIN_SLAB"):
        monkeypatch.delenv(k, raising=False)
    dev = rhi.RenderDevice(0)
    try:
        s = scenes.config_scene("c2")  # (645 entries per tile: 2-3 jobs each)
        gc, gd = renderer.render_scene(dev, s, frames=4)
        oc, od = oracle.render(s, nthreads=16)
        assert np.array_equal(gc, oc) and np.array_equal(gd.view(np.uint32), od.view(np.uint32))
        assert (dev.last_draw_stats()["tile_jobs"] > 0) == (jobs == "256")  # (longest C2 list: 741)
    finally:
        dev.close()
    assert_partitioned_parity(scenes.soup_scene(70, 20000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG), 3)


@pytest.mark.parametrize("cfg", ["c2x", "c3x"])
def test_clustered_first_frame(cfg):
    """Gaussian-clustered 1M-triangle scenes (scenes.clustered_scene; c2x at 1080p,
    central tiles ~40x the mean list; c3x at 4K): on a fresh device the first
    frame already holds every pair (the crowded tiles' excess in pool runs, no
    tile takes the record scan), the second frame too (slabs of the measured
    target), both exact; the bin buffer then holds at most 2x the pairs plus 512
    entries per tile.  The tile edge (tile_shift_for): the first
    frame takes the edge by size (c2x 32 px, c3x at 4K 64 px), whose measured
    shape is crowded, so the later frames take 16 px (c2x) or, where 16-px tiles
    would be too many, 32 (c3x)."""
    s = scenes.config_scene(cfg)
    oc, od = oracle.render(s, nthreads=16)
    edges = {"c2x": [32, 16, 16], "c3x": [64, 32, 32]}[cfg]
    dev = rhi.RenderDevice(0)
    try:
        for frame in range(3):
            gc, gd = renderer.render_scene(dev, s)
            st = dev.last_draw_stats()
            assert st["tile_size"] == edges[frame], (frame, st)
            ntiles = -(-s.width // st["tile_size"]) * -(-s.height // st["tile_size"])
            assert st["overflowed_draws"] == 0, (frame, st)
            assert st["bin_pool_runs"] > 0, (frame, st)
            # (its crowded tiles are split into tile jobs, the first frame included:
            # a shape not measured yet builds jobs for whatever lists turn out long)
            assert st["tile_jobs"] > 0, (frame, st)
            assert np.array_equal(gc, oc), frame
            assert np.array_equal(gd.view(np.uint32), od.view(np.uint32)), frame
        assert st["bin_capacity"] <= 2 * st["bin_pairs"] + 512 * ntiles, st
    finally:
        dev.close()


@pytest.mark.parametrize("stage", ["0", "1"])
def test_setup_bin_stage(monkeypatch, stage):
    """k_setup_bin's phase 4 staged in LDS (ZR_BIN_STAGE=1, forced even beside an
    overlapped tile pass) and direct (0), bit-exact on: a soup, a tile shard, the
    camera program's fans, pairs past full slabs (ZR_BIN_CAPACITY), and a draw
    whose workgroups have more pairs than the staging holds (large triangles:
    those workgroups scatter directly)."""
    monkeypatch.setenv("ZR_BIN_STAGE", stage)
    dev = rhi.RenderDevice(0)
    try:
        assert_parity(dev, scenes.config_scene("c1", n=30000, width=640, height=360))
        assert_parity(dev, scenes.soup_scene(18, 4000, 512, 384, 12.0, scenes.PROGRAM_BLINN_PHONG), shard=(1, 3))
        assert_parity(dev, scenes.cerberus_scene(640, 480))
        assert_parity(dev, scenes.soup_scene(17, 300, 512, 384, 150.0, scenes.PROGRAM_FLAT_COLOR))
    finally:
        dev.close()
    monkeypatch.setenv("ZR_BIN_CAPACITY", "1024")
    dev = rhi.RenderDevice(0)
    try:
        assert_parity(dev, scenes.soup_scene(16, 3000, 640, 480, 40.0, scenes.PROGRAM_FLAT_COLOR))
        assert dev.last_draw_stats()["overflowed_draws"] == 1
    finally:
        dev.close()


@pytest.mark.parametrize("table", [0, 1])
def test_record_table(monkeypatch, table):
    """k_tile's 512-thread resolve with its LDS record table forced on or off
    (ZR_REC_TABLE; the runtime enables it from 256 primitives per tile): exact on
    every program and depth op, with large primitives among small ones, a tile-row
    shard, tile lists of several 1024-entry segments (the 2048-slot hash keeps the
    earlier segments' slots; lookups that miss fall back to the gathered record),
    large primitives in the later segments of such lists, and the spill path."""
    monkeypatch.setenv("ZR_REC_TABLE", str(table))
    monkeypatch.setenv("ZR_TILE_NT", "512")
    dev = rhi.RenderDevice(0)
    try:
        for prog in (scenes.PROGRAM_TRIANGLE, scenes.PROGRAM_FLAT_COLOR, scenes.PROGRAM_BLINN_PHONG):
            assert_parity(dev, scenes.soup_scene(80 + prog, 6000, 320, 240, 6.0, prog))
        assert_parity(dev, scenes.soup_scene(84, 400, 512, 384, 150.0, scenes.PROGRAM_BLINN_PHONG))
        for op, write in ((scenes.OP_LEQUAL, True), (scenes.OP_GREATER, True), (scenes.OP_LESS, False)):
            s = scenes.soup_scene(85, 4000, 256, 192, 8.0, scenes.PROGRAM_BLINN_PHONG)
            s.depth_op, s.depth_write = op, write
            if op == scenes.OP_GREATER:
                s.depth_clear = 0.0
            assert_parity(dev, s)
        assert_parity(dev, scenes.soup_scene(86, 6000, 320, 240, 6.0, scenes.PROGRAM_BLINN_PHONG), shard=(2, 3))
        # ~2900 entries per 32x32 tile: three segments, the table full after the first
        dense = scenes.soup_scene(87, 40000, 96, 96, 5.0, scenes.PROGRAM_BLINN_PHONG)
        assert_parity(dev, dense)
        # large primitives in every segment of ~5000-entry tiles: a large entry's
        # sorted position held an earlier segment's small record, and a hash slot
        # that segment inserted for the position must not resolve to it
        small = scenes.soup_arrays(89, 30000, 96, 96, 5.0, True).reshape(-1, 3, 9)
        big = scenes.soup_arrays(90, 1200, 96, 96, 150.0, True).reshape(-1, 3, 9)
        v = np.concatenate([np.concatenate([small[25 * i:25 * i + 25], big[i:i + 1]]) for i in range(1200)])
        mixed = scenes.Scene("segments_with_large", 96, 96, scenes.PROGRAM_BLINN_PHONG, v.reshape(-1, 9),
                             np.arange(3 * len(v), dtype=np.uint32), depth=True)
        assert_parity(dev, mixed)
        for op in (scenes.OP_LEQUAL, scenes.OP_GREATER):
            mixed.depth_op, mixed.depth_clear = op, (0.0 if op == scenes.OP_GREATER else 1.0)
            assert_parity(dev, mixed)
    finally:
        dev.close()
    monkeypatch.setenv("ZR_BIN_CAPACITY", "1024")  # the spill path (records set up again, not read)
    dev = rhi.RenderDevice(0)
    try:
        assert_parity(dev, scenes.soup_scene(88, 6000, 320, 240, 12.0, scenes.PROGRAM_BLINN_PHONG))
    finally:
        dev.close()


@pytest.mark.parametrize("nt", [256, 512])
def test_tile_workgroup_sizes(monkeypatch, nt):
    """k_tile at each workgroup size (4 or 8 waves per tile; the runtime picks by
    tiles per CU, ZR_TILE_NT forces one): exact on every program, the wave path,
    depth ops and a tile-row shard."""
    monkeypatch.setenv("ZR_TILE_NT", str(nt))
    dev = rhi.RenderDevice(0)
    try:
        for prog in (scenes.PROGRAM_TRIANGLE, scenes.PROGRAM_FLAT_COLOR, scenes.PROGRAM_BLINN_PHONG):
            assert_parity(dev, scenes.soup_scene(60 + prog, 4000, 320, 240, 9.0, prog))
        assert_parity(dev, scenes.soup_scene(63, 300, 512, 384, 150.0, scenes.PROGRAM_BLINN_PHONG))
        for op, write in ((scenes.OP_LEQUAL, True), (scenes.OP_GREATER, True), (scenes.OP_LESS, False)):
            s = scenes.soup_scene(64, 3000, 256, 192, 10.0, scenes.PROGRAM_FLAT_COLOR)
            s.depth_op, s.depth_write = op, write
            if op == scenes.OP_GREATER:
                s.depth_clear = 0.0
            assert_parity(dev, s)
        assert_parity(dev, scenes.soup_scene(65, 3000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG), shard=(1, 3))
    finally:
        dev.close()


@pytest.mark.parametrize("edge", [16, 32, 64])
def test_tile_edges(monkeypatch, edge):
    """Every path of k_tile at each tile edge (ZR_TILE forces it; the runtime
    picks per draw, tile_shift_for): the flat and Blinn-Phong programs under the
    depth-writing modes take 16- and 64-px tiles (256 / 1024 threads), the other
    draws (triangle and camera programs, last-wins modes) and tile-row shards stay
    on 32.  Exact on soups, large primitives (wave path and lane walk), lists of
    several segments with the record table on and off, a crowded tile in pool
    runs, tile jobs, the record-scan spill, and frames back to back."""
    monkeypatch.setenv("ZR_TILE", str(edge))
    dev = rhi.RenderDevice(0)
    try:
        def check(scene, want, shard=None):
            assert_parity(dev, scene, shard=shard)
            assert dev.last_draw_stats()["tile_size"] == want, (scene.name, dev.last_draw_stats())
        for prog in (scenes.PROGRAM_FLAT_COLOR, scenes.PROGRAM_BLINN_PHONG):
            check(scenes.soup_scene(160 + prog, 5000, 330, 250, 9.0, prog), edge)
        check(scenes.soup_scene(163, 400, 512, 384, 150.0, scenes.PROGRAM_BLINN_PHONG), edge)
        for op, clear in ((scenes.OP_LEQUAL, 1.0), (scenes.OP_GREATER, 0.0), (scenes.OP_GEQUAL, 0.0)):
            s = scenes.soup_scene(164, 3000, 256, 192, 10.0, scenes.PROGRAM_FLAT_COLOR)
            s.depth_op, s.depth_clear = op, clear
            check(s, edge)
        s.depth_write = False  # last-wins keys: 32-px tiles
        check(s, 32)
        check(scenes.soup_scene(165, 2000, 256, 192, 10.0, scenes.PROGRAM_TRIANGLE), 32)
        check(scenes.cerberus_scene(640, 480), 32)
        check(scenes.soup_scene(166, 3000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG), 32, shard=(1, 3))
        check(scenes.soup_scene(66, 3000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG), edge)
        for table in ("0", "1"):  # several 1024-entry segments per tile (the record table's reuse)
            monkeypatch.setenv("ZR_REC_TABLE", table)
            d2 = rhi.RenderDevice(0)
            try:
                assert_parity(d2, scenes.soup_scene(87, 40000, 96, 96, 5.0, scenes.PROGRAM_BLINN_PHONG))
                assert d2.last_draw_stats()["tile_size"] == edge
            finally:
                d2.close()
        monkeypatch.delenv("ZR_REC_TABLE")
        check(crowded_tile_scene(), edge)
        for _ in range(2):  # the shape measured: later draws take its slab / pool / jobs sizing
            s = scenes.config_scene("c2", n=200_000)
            gc, gd = renderer.render_scene(dev, s, frames=3)
            oc, od = oracle.render(s, nthreads=16)
            assert np.array_equal(gc, oc) and np.array_equal(gd.view(np.uint32), od.view(np.uint32))
            assert dev.last_draw_stats()["tile_size"] == edge
    finally:
        dev.close()
    monkeypatch.setenv("ZR_JOBS", "256")  # tile jobs (key buffers of the edge's pixels)
    dev = rhi.RenderDevice(0)
    try:
        check_jobs = scenes.soup_scene(167, 20000, 160, 128, 10.0, scenes.PROGRAM_BLINN_PHONG)
        for _ in range(2):
            assert_parity(dev, check_jobs)
            st = dev.last_draw_stats()
            assert st["tile_size"] == edge and st["tile_jobs"] > 0, st
    finally:
        dev.close()
    monkeypatch.delenv("ZR_JOBS")
    monkeypatch.setenv("ZR_BIN_CAPACITY", "1024")  # the record-scan spill
    dev = rhi.RenderDevice(0)
    try:
        assert_parity(dev, scenes.soup_scene(16, 3000, 640, 480, 40.0, scenes.PROGRAM_FLAT_COLOR))
        st = dev.last_draw_stats()
        assert st["overflowed_draws"] == 1 and st["tile_size"] == edge, st
    finally:
        dev.close()


@pytest.mark.parametrize("fmt", [zr.FORMAT_R8G8B8A8_UNORM, zr.FORMAT_B8G8R8A8_UNORM, zr.FORMAT_R8G8B8A8_SRGB,
                                 zr.FORMAT_R32G32B32A32_SFLOAT])
def test_color_formats(device, fmt):
    s = scenes.soup_scene(17, 800, 160, 120, 12.0, scenes.PROGRAM_BLINN_PHONG)
    s.color_format = fmt
    assert_parity(device, s)


@pytest.mark.parametrize("mask", [0x1, 0x6, 0x8, 0xB])
def test_write_masks(device, mask):
    s = scenes.soup_scene(18, 600, 128, 96, 10.0, scenes.PROGRAM_FLAT_COLOR)
    s.write_mask = mask
    assert_parity(device, s)


@pytest.mark.parametrize("cull,front", [(scenes.CULL_BACK, scenes.FRONT_CCW), (scenes.CULL_BACK, scenes.FRONT_CW),
                                        (scenes.CULL_FRONT, scenes.FRONT_CCW), (3, scenes.FRONT_CCW)])
def test_cull_modes(device, cull, front):
    s = scenes.soup_scene(19, 1000, 160, 120, 12.0, scenes.PROGRAM_FLAT_COLOR)
    s.cull_mode, s.front_face = cull, front
    assert_parity(device, s)


@pytest.mark.parametrize("vp,sc", [((20.0, 10.0, 200.0, 150.0, 0.0, 1.0), (30, 20, 150, 100)),
                                   ((0.0, 180.0, 256.0, -180.0, 0.0, 1.0), (0, 0, 256, 180)),
                                   ((-40.0, -30.0, 320.0, 240.0, 0.25, 0.75), (5, 7, 240, 160))])
def test_viewport_scissor(device, vp, sc):
    s = scenes.soup_scene(20, 1200, 256, 180, 14.0, scenes.PROGRAM_FLAT_COLOR)
    assert_parity(device, s, viewport=vp, scissor=sc)


def test_draw_arguments(device):
    """u16 indices with first_index / vertex_offset, instancing, non-indexed draws."""
    base = scenes.soup_scene(23, 300, 128, 128, 12.0, scenes.PROGRAM_FLAT_COLOR)
    s = scenes.Scene("args", 128, 128, scenes.PROGRAM_FLAT_COLOR, base.vertices,
                     np.arange(base.vertices.shape[0] - 30, dtype=np.uint16), depth=True,
                     first=12, vertex_offset=30, count=600, instance_count=2)
    assert_parity(device, s)
    s2 = scenes.Scene("nonindexed", 128, 128, scenes.PROGRAM_FLAT_COLOR, base.vertices, None, depth=True,
                      first=9, count=450)
    assert_parity(device, s2)


def test_out_of_range_indices_dropped(device):
    base = scenes.soup_scene(24, 200, 128, 128, 12.0, scenes.PROGRAM_FLAT_COLOR)
    idx = np.arange(600, dtype=np.uint32)
    idx[::7] = 10_000_000  # beyond the vertex buffer: those primitives are discarded
    s = scenes.Scene("oob", 128, 128, scenes.PROGRAM_FLAT_COLOR, base.vertices, idx, depth=True)
    assert_parity(device, s)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tile_row_shards(device, world):
    s = scenes.soup_scene(25, 3000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG)
    for r in range(world):
        assert_parity(device, s, shard=(r, world))


# ------------------------------------------------------- full benchmark sizes
@pytest.mark.parametrize("cfg", ["c1", "c2"])
def test_full_config_parity(device, cfg):
    """C1 (100k tris) and C2 (1M tris) at 1920x1080, bit-exact vs the oracle (both
    on 32-px tiles: tile_shift_for)."""
    s = scenes.config_scene(cfg)
    gc, gd = renderer.render_scene(device, s)
    st = device.last_draw_stats()
    assert st["tile_size"] == 32, st
    oc, od, ost = oracle.render(s, nthreads=16, with_stats=True)
    assert np.array_equal(gc, oc)
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    assert st["triangles_setup"] == ost.triangles_setup


def test_c3_4k_shards_union(device):
    """C3 geometry (1M tris, 3840x2160): the union of 8 shards rendered separately
    equals the oracle frame, colour and depth bits (the multi-GPU partition, on
    one GPU; 1020 tiles per rank: 8 round-robin rows of 120 + a run of 60; shards
    bin 32-px tiles), and the unsharded frame, which tile_shift_for puts on 64-px
    tiles (a 4K target with 122 primitives per 32-px tile)."""
    s = scenes.config_scene("c3")
    oc, od = oracle.render(s, nthreads=16)
    acc = np.zeros_like(oc)
    accd = np.full_like(od, np.nan)
    for r in range(8):
        gc, gd = renderer.render_scene(device, s, shard=(r, 8))
        assert device.last_draw_stats()["tile_size"] == 32
        rows = owned(s, (r, 8))
        acc[rows] = gc[rows]
        accd[rows] = gd[rows]
    assert np.array_equal(acc, oc)
    assert np.array_equal(accd.view(np.uint32), od.view(np.uint32))
    gc, gd = renderer.render_scene(device, s)
    assert device.last_draw_stats()["tile_size"] == 64
    assert np.array_equal(gc, oc)
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))


def test_c4_micro_triangles(device):
    """C4: 10M sub-pixel triangles at 1080p; exact vs the oracle.  4.8 primitives
    per pixel: setup's micro-primitive test is on by default (use_micro_test) and
    drops the ones that miss their sample."""
    s = scenes.config_scene("c4")
    gc, gd = renderer.render_scene(device, s)
    assert device.last_draw_stats()["micro_fragments"] > 100_000
    assert device.last_draw_stats()["tile_size"] == 64  # (>= 1 primitive per pixel: tile_shift_for)
    oc, od = oracle.render(s, nthreads=16)
    assert np.array_equal(gc, oc)
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))


def mixed_micro_scene(seed, n, width, height, program, flat_z=None):
    """Micro primitives (a clipped bbox of one pixel: k_setup_bin tests the one
    sample and drops those that miss it, DrawParams::micro; the covered ones are
    binned and resolved by k_tile like any other) interleaved in API order with
    ordinary 6-px ones: every third primitive is ordinary.  flat_z: every vertex
    at that depth, so every fragment of a pixel ties and only API order decides."""
    normals = program == scenes.PROGRAM_BLINN_PHONG
    micro = scenes.soup_arrays(seed, n, width, height, 0.45, normals).reshape(n, 3, -1)
    big = scenes.soup_arrays(seed + 1000, n, width, height, 6.0, normals).reshape(n, 3, -1)
    pick = (np.arange(n) % 3 == 0)[:, None, None]
    verts = np.where(pick, big, micro)
    if flat_z is not None:
        verts[:, :, 2] = flat_z
    return scenes.Scene(f"mixed_micro_s{seed}", width, height, program, verts.reshape(3 * n, -1),
                        np.arange(3 * n, dtype=np.uint32), depth=True)


@pytest.fixture(scope="module")
def micro_device():
    """A device with setup's micro-primitive test forced on (ZR_MICRO=1, read at
    device creation; by default only draws of >= 1 primitive per pixel get it)."""
    import os
    old = os.environ.get("ZR_MICRO")
    os.environ["ZR_MICRO"] = "1"
    dev = rhi.RenderDevice(0)
    if old is None:
        del os.environ["ZR_MICRO"]
    else:
        os.environ["ZR_MICRO"] = old
    yield dev
    dev.close()


@pytest.mark.parametrize("op,clear,flat", [(scenes.OP_LESS, 1.0, None), (scenes.OP_LEQUAL, 1.0, 0.5),
                                           (scenes.OP_LESS, 1.0, 0.5), (scenes.OP_GREATER, 0.0, None),
                                           (scenes.OP_GEQUAL, 0.0, 0.25)])
def test_micro_primitives_mixed(micro_device, op, clear, flat):
    """Micro primitives (tested for their one sample by setup, dropped there when
    they miss it: DrawParams::micro) beside ordinary ones, API order mixed: depth
    modes, and with every depth equal the order rules (LESS: first wins, LEQUAL /
    GEQUAL: last wins).  The draw stats count the covered micro primitives, so the
    path is known to run."""
    device = micro_device
    s = mixed_micro_scene(83, 60_000, 320, 240, scenes.PROGRAM_BLINN_PHONG, flat)
    s.depth_op, s.depth_clear = op, clear
    assert_parity(device, s)
    assert device.last_draw_stats()["micro_fragments"] > 1000


def test_micro_primitives_modes(micro_device):
    """The micro path under no depth attachment (last wins by API order), depth
    test without writes (last-wins pre-test against the loaded depth), a 3-way
    tile-row shard (only owned tiles' samples), a partial last tile row, the
    triangle program, and a one-pixel scissor."""
    device = micro_device
    s = mixed_micro_scene(84, 40_000, 300, 170, scenes.PROGRAM_FLAT_COLOR)
    s.depth = False
    assert_parity(device, s)
    assert device.last_draw_stats()["micro_fragments"] > 1000
    s = mixed_micro_scene(85, 40_000, 300, 170, scenes.PROGRAM_FLAT_COLOR)
    s.depth_write = False  # (depth test, no writes: last wins among those passing the loaded depth)
    assert_parity(device, s)
    assert device.last_draw_stats()["micro_fragments"] > 1000
    s = mixed_micro_scene(86, 40_000, 300, 170, scenes.PROGRAM_BLINN_PHONG)
    for r in range(3):
        assert_parity(device, s, shard=(r, 3))
    s = mixed_micro_scene(87, 20_000, 300, 170, scenes.PROGRAM_TRIANGLE)
    s.time = 1.25
    assert_parity(device, s)
    # a one-pixel scissor: every primitive's clipped bbox is that pixel, yet the
    # large ones (extents far past 64 px) stay on the ordinary path
    s = scenes.soup_scene(89, 3000, 200, 160, 60.0, scenes.PROGRAM_FLAT_COLOR)
    assert_parity(device, s, scissor=(97, 61, 1, 1))
    s = mixed_micro_scene(90, 30_000, 200, 160, scenes.PROGRAM_BLINN_PHONG)
    assert_parity(device, s, scissor=(33, 21, 1, 1))


def test_micro_primitives_repeat(micro_device):
    """Back-to-back frames of a micro-heavy draw with no host sync in between:
    the last frame equals the oracle's."""
    s = mixed_micro_scene(88, 50_000, 256, 192, scenes.PROGRAM_FLAT_COLOR)
    gc, gd = renderer.render_scene(micro_device, s, frames=3)
    oc, od = oracle.render(s)
    assert np.array_equal(gc, oc) and np.array_equal(gd.view(np.uint32), od.view(np.uint32))


def test_determinism_repeat(device):
    s = scenes.config_scene("c2", n=200_000)
    a = renderer.render_scene(device, s)
    b = renderer.render_scene(device, s)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))


@pytest.fixture(params=["eager", "graph"])
def resubmit_device(request, monkeypatch):
    if request.param == "graph":
        monkeypatch.setenv("ZR_GRAPH", "1")
    dev = rhi.RenderDevice(0)
    yield dev
    dev.close()


def test_resubmit_graph_replay(resubmit_device):
    """One recorded command list submitted repeatedly (with ZR_GRAPH=1: eager, then
    captured into a HIP graph, then replayed).  The Time uniform changes between
    submissions and every frame must match the oracle at that time (the graph
    reads the buffer, not a recorded value)."""
    device = resubmit_device
    s = scenes.triangle_scene()
    color = rhi.Texture(device, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
    r = renderer.SceneRenderer(device, s)
    enc = r.record(color, None)
    for t in (0.0, 1.25, 7.5, 2.0, 0.5):
        r.time_buffer.as_range(0, 4).write(np.float32(t).tobytes())
        device.submit_and_wait(enc)
        ref, _ = oracle.render(scenes.triangle_scene(time=t))
        assert np.array_equal(color.read(), ref), f"t={t}"
    enc.destroy()
    color.destroy()


def test_resubmit_soup_graph_replay(resubmit_device):
    device = resubmit_device
    s = scenes.soup_scene(41, 5000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG)
    color = rhi.Texture(device, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
    depth = rhi.Texture(device, rhi.TextureDesc.new_depth("ds", s.width, s.height))
    r = renderer.SceneRenderer(device, s)
    enc = r.record(color, depth)
    ref, refd = oracle.render(s)
    for _ in range(4):
        device.submit(enc)
    device.wait_idle()
    assert np.array_equal(color.read(), ref)
    assert np.array_equal(depth.read().view(np.uint32), refd.view(np.uint32))
    enc.destroy()
    color.destroy()
    depth.destroy()


# ------------------------------------------- partitioned setup
def render_partitioned(scene, world, capacity=0, frames=1, **kw):
    """All `world` ranks of a partitioned tile-row shard, emulated by threads on
    one GPU (each with its own RenderDevice); returns each rank's (colour, depth,
    stats).  `capacity`: records per exchange block (0: the runtime's default);
    `frames`: frames submitted back to back before the read-back."""
    import threading
    group = shard.ThreadGroupExchange.Group(world, "cuda:0")
    out = [None] * world

    def run(r):
        dev = rhi.RenderDevice(0)
        try:
            sh = (r, world, shard.ThreadGroupExchange(group, r), capacity)
            out[r] = renderer.render_scene(dev, scene, shard=sh, frames=frames, **kw)
            out[r] = out[r] + (dev.last_draw_stats(),)
        except BaseException as e:  # noqa: BLE001 - reported below
            out[r] = e
            group.barrier.abort()
        finally:
            dev.close()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    for r in range(world):
        if isinstance(out[r], BaseException):
            raise out[r]
    return out


def assert_partitioned_parity(scene, world, capacity=0, frames=1, nthreads=16, **kw):
    oc, od = oracle.render(scene, nthreads=nthreads, **kw)
    stats = []
    for r, (gc, gd, st) in enumerate(render_partitioned(scene, world, capacity, frames, **kw)):
        rows = owned(scene, (r, world))
        bad = np.argwhere(np.any(gc[rows] != oc[rows], axis=-1))
        assert bad.size == 0, f"rank {r}/{world}: {len(bad)} pixels differ, first {bad[:5].tolist()}"
        if scene.depth:
            assert np.array_equal(gd[rows].view(np.uint32), od[rows].view(np.uint32)), f"rank {r}/{world} depth"
        stats.append(st)
    return stats


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partitioned_shards(world):
    """Each rank sets up 1/G of the primitives and routes them (k_route) through
    the exchange; every rank's rows equal the oracle frame.  20k primitives give
    several route chunks per rank at G=2 and empty ranges at G=8."""
    assert_partitioned_parity(scenes.soup_scene(70, 20000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG), world)


def test_partitioned_paths():
    """Wave path, mixed sizes, depth ops, instancing and u16 indices under the
    partitioned setup."""
    assert_partitioned_parity(scenes.soup_scene(71, 300, 512, 384, 150.0, scenes.PROGRAM_BLINN_PHONG), 3)
    s = scenes.soup_scene(72, 3000, 200, 160, 14.0, scenes.PROGRAM_FLAT_COLOR)
    s.depth_op = scenes.OP_LEQUAL
    assert_partitioned_parity(s, 2)
    s = scenes.soup_scene(73, 3000, 200, 160, 14.0, scenes.PROGRAM_FLAT_COLOR)
    s.depth_op, s.depth_clear = scenes.OP_GREATER, 0.0
    assert_partitioned_parity(s, 4)
    assert_partitioned_parity(scenes.cube_scene(), 2)
    assert_partitioned_parity(scenes.triangle_scene(time=1.25), 3)


def test_partitioned_ranks_without_rows():
    """G=8 on a 96x64 target has 6 tiles: ranks 3 and 7 own none, yet they still
    route their ranges and join every exchange
    (nobody is left waiting); a 160x120 target (20 tiles, all leftover rows) gives
    every rank a run of 2 or 3 tiles."""
    s = scenes.soup_scene(77, 3000, 96, 64, 8.0, scenes.PROGRAM_BLINN_PHONG)
    assert sum(shard.owned_pixels(96, 64, r, 8) == 0 for r in range(8)) == 2
    assert_partitioned_parity(s, 8)
    assert_partitioned_parity(scenes.soup_scene(77, 4000, 160, 120, 8.0, scenes.PROGRAM_BLINN_PHONG), 8)


def test_partitioned_beside_busy_stream():
    """A partitioned draw while another stream keeps every CU busy (matmuls):
    setup kernel has no grid barrier, so it needs no co-residency and cannot
    time out; the frame is exact."""
    import threading
    import torch
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    stop = threading.Event()

    def busy():
        with torch.cuda.stream(side):
            while not stop.is_set():
                for _ in range(8):
                    a.matmul(a)
                side.synchronize()

    t = threading.Thread(target=busy)
    t.start()
    try:
        assert_partitioned_parity(scenes.soup_scene(78, 300_000, 640, 480, 3.0, scenes.PROGRAM_FLAT_COLOR), 2)
    finally:
        stop.set()
        t.join(timeout=60)


def test_mixed_draw_sizes_no_sync(device):
    """A draw above 2^18 primitives and one per pixel (setup on the main stream,
    scratch set 0) followed by small draws (setup on the setup stream,
    alternating sets) with no host sync in between: every target equals its own
    oracle frame."""
    big = scenes.soup_scene(79, 400_000, 640, 480, 3.0, scenes.PROGRAM_BLINN_PHONG)
    small = [scenes.soup_scene(80 + i, 2000 + 1000 * i, 320, 240, 9.0, scenes.PROGRAM_FLAT_COLOR) for i in range(3)]
    jobs = []
    for s in [big] + small:
        color = rhi.Texture(device, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
        depth = rhi.Texture(device, rhi.TextureDesc.new_depth("ds", s.width, s.height))
        r = renderer.SceneRenderer(device, s)
        enc = r.record(color, depth, encoder=rhi.CommandEncoder(device))
        jobs.append((s, r, enc, color, depth))
    for _ in range(2):
        for _, _, enc, _, _ in jobs:
            device.submit(enc)
    device.wait_idle()
    for s, _, enc, color, depth in jobs:
        oc, od = oracle.render(s)
        assert np.array_equal(color.read(), oc), s.name
        assert np.array_equal(depth.read().view(np.uint32), od.view(np.uint32)), s.name
        enc.destroy()
        color.destroy()
        depth.destroy()


def test_overlapped_large_draws_no_sync(device):
    """Draws above 2^18 primitives but below one per pixel set up beside the
    previous draw's tile pass (use_overlap_setup: the setup stream, alternating
    scratch sets).  Back to back, twice, with no host sync: the clustered c2x
    (tile jobs, pool runs, the schedule workgroup), a uniform soup, a draw above
    one primitive per pixel (main stream) between them -- every target equals its
    own oracle frame."""
    todo = [scenes.config_scene("c2x"),
            scenes.soup_scene(91, 400_000, 1280, 720, 5.0, scenes.PROGRAM_BLINN_PHONG),
            scenes.soup_scene(92, 400_000, 640, 480, 3.0, scenes.PROGRAM_FLAT_COLOR),
            scenes.soup_scene(93, 300_000, 800, 600, 4.0, scenes.PROGRAM_FLAT_COLOR)]
    jobs = []
    for s in todo:
        color = rhi.Texture(device, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
        depth = rhi.Texture(device, rhi.TextureDesc.new_depth("ds", s.width, s.height))
        r = renderer.SceneRenderer(device, s)
        enc = r.record(color, depth, encoder=rhi.CommandEncoder(device))
        jobs.append((s, r, enc, color, depth))
    for _ in range(2):
        for _, _, enc, _, _ in jobs:
            device.submit(enc)
    device.wait_idle()
    for s, _, enc, color, depth in jobs:
        oc, od = oracle.render(s, nthreads=16)
        assert np.array_equal(color.read(), oc), s.name
        assert np.array_equal(depth.read().view(np.uint32), od.view(np.uint32)), s.name
        enc.destroy()
        color.destroy()
        depth.destroy()


def test_partitioned_c2_full():
    """C2 (1M triangles, 1920x1080) as 8 partitioned ranks: union = oracle frame."""
    assert_partitioned_parity(scenes.config_scene("c2"), 8)


def test_partitioned_c3_full():
    """C3 (1M triangles, 3840x2160) as 8 partitioned ranks, two frames back to
    back: each rank's ~1020 tiles take 4-wave tiles (tile_threads_for's
    partitioned branch, >= 3.5 tiles per CU) and the second frame's route,
    exchange and record binning run on the setup stream beside the first frame's
    tile pass.  Union of the ranks' rows = the oracle frame; no block overflowed."""
    stats = assert_partitioned_parity(scenes.config_scene("c3"), 8, frames=2)
    assert all(st["route_fallback_draws"] == 0 for st in stats)
    assert max(st["route_max_entries"] for st in stats) > 0


@pytest.mark.parametrize("capacity", [1, 300])
def test_partitioned_route_overflow(capacity):
    """Exchange blocks far too small for the routed records: the receivers see the
    overflow in the block headers and set up every primitive of the draw
    themselves -- still exact -- and the stats report it."""
    s = scenes.soup_scene(81, 8000, 320, 240, 10.0, scenes.PROGRAM_BLINN_PHONG)
    stats = assert_partitioned_parity(s, 4, capacity=capacity)
    assert all(st["route_fallback_draws"] >= 1 for st in stats)
    assert all(st["route_max_entries"] > capacity for st in stats)


def test_replay_exchange_layout_checked(device):
    """zr_replay_exchange_fn (bench.py --emulate-shard) copies recorded receive
    blocks into the draw's receive buffer: a recording of another layout (here one
    block for a 2-way shard) is refused at submit with VALIDATION_FAILED instead of
    being copied past the buffer's end; the draw's own layout is accepted."""
    import ctypes
    import torch
    s = scenes.soup_scene(82, 2000, 160, 120, 8.0, scenes.PROGRAM_FLAT_COLOR)
    cap, world = 100, 2
    block = 16 + 48 * cap  # route_block_bytes(cap): RouteHeader + cap RouteEntry

    class Replay:
        def __init__(self, nbytes):
            self.src = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")

        def native(self):
            desc = zr.zr_replay_exchange(self.src.data_ptr(), self.src.numel())
            return zr.lib().zr_replay_exchange_fn(), ctypes.addressof(desc), (desc, self.src)

    color = rhi.Texture(device, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
    depth = rhi.Texture(device, rhi.TextureDesc.new_depth("ds", s.width, s.height))
    r = renderer.SceneRenderer(device, s)
    bad = r.record(color, depth, shard=(0, world, Replay(block), cap), encoder=rhi.CommandEncoder(device))
    with pytest.raises(zr.ZrError) as e:
        device.submit(bad)
    assert e.value.code == zr.ERROR_VALIDATION_FAILED
    device.wait_idle()
    good = r.record(color, depth, shard=(0, world, Replay(world * block), cap), encoder=rhi.CommandEncoder(device))
    device.submit(good)
    device.wait_idle()
    for x in (bad, good, color, depth):
        x.destroy()


def test_partitioned_overflow_spill(monkeypatch):
    monkeypatch.setenv("ZR_BIN_CAPACITY", "256")
    assert_partitioned_parity(scenes.soup_scene(74, 3000, 320, 240, 30.0, scenes.PROGRAM_FLAT_COLOR), 2)


def test_partitioned_rccl_exchange():
    """The RCCL exchange itself (torch.distributed "nccl", world size 1: the
    all-to-all is a local copy through RCCL) ordered on torch's stream."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        dev = rhi.RenderDevice(0)
        dev.set_stream(torch.cuda.current_stream().cuda_stream)
        ex = shard.RcclExchange("cuda:0")
        s = scenes.soup_scene(75, 5000, 256, 192, 10.0, scenes.PROGRAM_BLINN_PHONG)
        gc, gd = renderer.render_scene(dev, s, shard=(0, 1, ex))
        oc, od = oracle.render(s)
        assert ex.calls == 1
        assert np.array_equal(gc, oc) and np.array_equal(gd.view(np.uint32), od.view(np.uint32))
        dev.close()
    finally:
        dist.destroy_process_group()


def test_runtime_rccl_world1():
    """The runtime's own RCCL communicators (zr_device_init_rccl) at world size 1:
    partitioned setup through zr_rccl_exchange_fn, and the tile-row gather (no
    peers: nothing moves) ordered before the next pass on the same target."""
    dev = rhi.RenderDevice(0)
    try:
        shard.init_runtime_rccl(dev, 0, 1)
        s = scenes.soup_scene(76, 5000, 256, 192, 10.0, scenes.PROGRAM_BLINN_PHONG)
        color = rhi.Texture(dev, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
        depth = rhi.Texture(dev, rhi.TextureDesc.new_depth("ds", s.width, s.height))
        r = renderer.SceneRenderer(dev, s)
        enc = r.record(color, depth, shard=(0, 1, "rccl"))
        oc, od = oracle.render(s)
        for _ in range(3):
            dev.submit(enc)
            dev.gather_tile_rows(color, 0)
        dev.wait_idle()
        assert np.array_equal(color.read(), oc) and np.array_equal(depth.read().view(np.uint32), od.view(np.uint32))
        enc.destroy()
        color.destroy()
        depth.destroy()
    finally:
        dev.close()


# ------------------------------------------------ mesh program (camera, clip)
@pytest.mark.parametrize("seed,n", [(31, 600), (32, 3000), (33, 20000)])
def test_mesh_soup(device, seed, n):
    """mesh.slang through a reverse-Z camera: near-plane crossings (clipped fans),
    primitives behind the camera and beyond the view edges; bit-exact."""
    assert_parity(device, scenes.mesh_soup_scene(seed, n, 320, 240))


@pytest.mark.parametrize("op,write", [(scenes.OP_GEQUAL, True), (scenes.OP_ALWAYS, True), (scenes.OP_GREATER, False)])
def test_mesh_depth_modes(device, op, write):
    """Last-wins modes resolve depth from the winning fan triangle's record."""
    s = scenes.mesh_soup_scene(34, 2000, 256, 192)
    s.depth_op, s.depth_write = op, write
    assert_parity(device, s)


def test_mesh_cerberus(device):
    """The reference's cerberus asset (33,543 triangles) through the camera."""
    assert_parity(device, scenes.cerberus_scene(640, 480))
    assert_parity(device, scenes.cerberus_scene(1920, 1080))


@pytest.mark.parametrize("scene", ["cerberus", "soup"])
def test_mesh_push_constants(device, scene):
    """View.view_proj recorded with CommandEncoder::push_constants (command.rs:180-185;
    mesh_push.slang) instead of bound as the View uniform: bit-exact with the
    oracle and with the uniform render of the same scene."""
    s = scenes.cerberus_scene(640, 480) if scene == "cerberus" else scenes.mesh_soup_scene(36, 3000, 320, 240)
    uc, ud = renderer.render_scene(device, s)
    s.push_view = True
    pc, pd = assert_parity(device, s)
    assert np.array_equal(pc, uc) and np.array_equal(pd.view(np.uint32), ud.view(np.uint32))


def test_mesh_push_constants_errors(device):
    """A draw whose pipeline reads push constants that were not pushed, or were
    pushed with a layout of other ranges, fails at submit (VALIDATION_FAILED)."""
    s = scenes.mesh_soup_scene(37, 200, 64, 64)
    s.push_view = True
    r = renderer.SceneRenderer(device, s)
    color = rhi.Texture(device, rhi.TextureDesc.new_color("rt", 64, 64, s.color_format))
    depth = rhi.Texture(device, rhi.TextureDesc.new_depth("ds", 64, 64))
    other = rhi.GraphicPipeline(device, r.pipeline.shader, r.pipeline.state, [s.color_format], zr.FORMAT_D32_SFLOAT,
                                push_constant_ranges=[(zr.SHADER_STAGE_VERTEX, 0, 64)])
    try:
        for push in (None, "half", "other_layout"):
            enc = rhi.CommandEncoder(device)

            def job(ctx):
                e = ctx.encoder()
                ctx.begin_rendering((64, 64))
                ctx.bind_pipeline()
                vp = np.asarray(s.view_proj, np.float32)
                if push == "half":
                    e.push_constants(ctx.pipeline.layout(), zr.SHADER_STAGE_ALL_GRAPHICS, 0, vp[:8])
                elif push == "other_layout":
                    e.push_constants(other, zr.SHADER_STAGE_VERTEX, 0, vp)
                e.set_viewport(0, [rhi.Viewport(0.0, 0.0, 64.0, 64.0)])
                e.set_scissor(0, [rhi.Rect2D(0, 0, 64, 64)])
                e.bind_vertex_buffers(0, [r.vertex_buffer], [0])
                e.bind_index_buffer(r.index_buffer, 0, s.index_type)
                e.draw_indexed(s.draw_count, 1, 0, 0, 0)
                ctx.end_rendering()

            rhi.execute_graphic_node(device, enc, r.pipeline, [color], depth, job)
            with pytest.raises(zr.ZrError) as e:
                device.submit_and_wait(enc)
            assert e.value.code == zr.ERROR_VALIDATION_FAILED
            enc.destroy()
    finally:
        other.destroy()
        color.destroy()
        depth.destroy()


def test_mesh_shards_and_spill(monkeypatch, device):
    s = scenes.mesh_soup_scene(35, 3000, 320, 240)
    for r in range(3):
        assert_parity(device, s, shard=(r, 3))
    monkeypatch.setenv("ZR_BIN_CAPACITY", "256")
    dev = rhi.RenderDevice(0)
    try:
        assert_parity(dev, s)
        assert dev.last_draw_stats()["overflowed_draws"] == 1
    finally:
        dev.close()


# ------------------------------------------------- present / clear (§8f row 4)
@pytest.mark.parametrize("fmt", [zr.FORMAT_B8G8R8A8_SRGB, zr.FORMAT_R8G8B8A8_UNORM, zr.FORMAT_R32G32B32A32_SFLOAT])
def test_clear_color_image(device, fmt):
    """zenith-sandbox's SimpleApp frame: cmd_clear_color_image (0.2, 0.3, 0.8, 1)
    over the whole image, encoded like the oracle's clear."""
    W, H = 200, 150
    tex = rhi.Texture(device, rhi.TextureDesc.new_color("swapchain", W, H, fmt))
    app = renderer.SimpleAppRenderer(device)
    device.submit_and_wait(app.render_to(tex))
    img = tex.read()
    s = scenes.Scene("clear", W, H, scenes.PROGRAM_FLAT_COLOR, np.zeros((0, 6), np.float32),
                     np.zeros(0, np.uint32), color_format=fmt, clear_color=renderer.SimpleAppRenderer.CLEAR)
    ref, _ = oracle.render(s)
    assert np.ascontiguousarray(img).tobytes() == ref.tobytes()
    if fmt == zr.FORMAT_B8G8R8A8_SRGB:
        from zenith_amd import present
        back = present.read_png_rgba(present.png_bytes(img, fmt))
        assert tuple(back[0, 0]) == tuple(img[0, 0, [2, 1, 0, 3]])
    tex.destroy()


def test_clear_then_draw_load(device):
    """A clear, then a render pass that LOADs the cleared colour and draws."""
    s = scenes.soup_scene(36, 500, 160, 120, 10.0, scenes.PROGRAM_FLAT_COLOR)
    s.depth = False  # no depth attachment: the last primitive wins, in order
    tex = rhi.Texture(device, rhi.TextureDesc.new_color("rt", s.width, s.height, s.color_format))
    enc = rhi.CommandEncoder(device)
    enc.begin()
    enc.clear_color_image(tex, s.clear_color)
    enc.end()
    device.submit_and_wait(enc)
    r = renderer.SceneRenderer(device, s)
    ref, _ = oracle.render(s)
    enc2 = r.record(tex, None)
    device.submit_and_wait(enc2)
    assert np.array_equal(tex.read(), ref)  # the pass's CLEAR equals the image clear's value
    enc.destroy()
    tex.destroy()


@pytest.mark.parametrize("program", [scenes.PROGRAM_FLAT_COLOR, scenes.PROGRAM_BLINN_PHONG])
def test_depth_range_discard(device, program):
    """Vertex depths spread over [-0.22, 1.22]: fragments outside [0, 1] are
    discarded per fragment, so the lane raster's range test runs
    (its loop without the test serves only waves whose vertices are all inside)."""
    s = scenes.soup_scene(23, 1500, 192, 128, 14.0, program)
    z = s.vertices[:, 2]
    s.vertices[:, 2] = z * np.float32(1.6) - np.float32(0.3)
    assert (s.vertices[:, 2] < 0).any() and (s.vertices[:, 2] > 1).any()
    assert_parity(device, s)


@pytest.mark.parametrize("nt", [256, 512])
def test_winner_census(monkeypatch, nt):
    """zr_device_set_profiling(dev, 2): zr_draw_stats.winners counts the distinct
    primitives that won a pixel (bench.py's per-winner bytes).  Each triangle's
    provoking colour encodes its id in UNORM8, so the frame itself gives the
    exact count; both resolve forms (256 / 512 threads) are checked."""
    monkeypatch.setenv("ZR_TILE_NT", str(nt))
    dev = rhi.RenderDevice(0)
    try:
        s = scenes.soup_scene(38, 3000, 256, 192, 10.0, scenes.PROGRAM_FLAT_COLOR)
        ids = np.arange(1, 3001)
        s.vertices[0::3, 3:6] = np.stack([ids & 255, (ids >> 8) & 255, (ids >> 16) & 255], 1).astype(np.float32) / 255
        s.color_format, s.clear_color = zr.FORMAT_R8G8B8A8_UNORM, (0.0, 0.0, 0.0, 0.0)
        dev.set_profiling(True, census=True)
        gc, _ = assert_parity(dev, s)
        dev.set_profiling(False)
        got = gc[..., 0].astype(np.int64) + (gc[..., 1].astype(np.int64) << 8) + (gc[..., 2].astype(np.int64) << 16)
        expected = len(np.unique(got[got > 0]))
        assert 1000 < expected < 3000
        assert dev.last_draw_stats()["winners"] == expected
    finally:
        dev.close()


@pytest.mark.parametrize("sched", [0, 1])
def test_tile_schedule(monkeypatch, sched):
    """k_tile's heaviest-first tile schedule (built by k_setup_bin's last workgroup
    past phase 2; ZR_TILE_SCHED forces it on or off): exact on every program, a
    tile-row shard, the spill path, partitioned records-mode setup and the mesh
    program, at both workgroup sizes; a list order never changes the image."""
    monkeypatch.setenv("ZR_TILE_SCHED", str(sched))
    for nt in (256, 512):
        monkeypatch.setenv("ZR_TILE_NT", str(nt))
        dev = rhi.RenderDevice(0)
        try:
            for prog in (scenes.PROGRAM_TRIANGLE, scenes.PROGRAM_FLAT_COLOR, scenes.PROGRAM_BLINN_PHONG):
                assert_parity(dev, scenes.soup_scene(90 + prog, 5000, 330, 250, 7.0, prog))
            assert_parity(dev, scenes.soup_scene(93, 4000, 330, 250, 7.0, scenes.PROGRAM_BLINN_PHONG), shard=(1, 3))
            assert_parity(dev, scenes.mesh_soup_scene(94, 3000, 320, 240))
            assert_parity(dev, scenes.cerberus_scene(640, 480))
        finally:
            dev.close()
    monkeypatch.setenv("ZR_BIN_CAPACITY", "1024")
    dev = rhi.RenderDevice(0)
    try:
        assert_parity(dev, scenes.soup_scene(95, 4000, 320, 240, 12.0, scenes.PROGRAM_FLAT_COLOR))
    finally:
        dev.close()
    monkeypatch.delenv("ZR_BIN_CAPACITY")
    assert_partitioned_parity(scenes.soup_scene(96, 6000, 320, 240, 8.0, scenes.PROGRAM_BLINN_PHONG), 3)
