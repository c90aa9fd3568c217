"""GPU parity: the HIP draw path (through the C ABI) against the CPU oracle.

Bar (north_star / DESIGN.md §5): coverage, depth bits and 8-bit colour codes are
bit-exact; float colour (R32G32B32A32_SFLOAT targets) is bit-exact as well since
both sides evaluate the same explicitly ordered float arithmetic — the test
tolerance below is 0 ULP, tighter than the north star's 1 ULP.
"""
import numpy as np
import pytest

from oracle import oracle
from zenith_amd import renderer, rhi, scenes, zr

pytestmark = pytest.mark.gpu

FLOAT_ULP_TOL = 0  # north_star allows 1 ULP on shaded float colour; we hold 0


def owned_rows(h, tile, shard):
    if shard is None:
        return np.ones(h, dtype=bool)
    r, n = shard
    return ((np.arange(h) // tile) % n) == r


def assert_parity(device, scene, shard=None, **kw):
    gc, gd = renderer.render_scene(device, scene, shard=shard, **kw)
    oc, od = oracle.render(scene, shard=shard or (0, 1), **kw)
    rows = owned_rows(scene.height, 32, shard)
    gc, oc = gc[rows], oc[rows]
    if scene.color_format == zr.FORMAT_R32G32B32A32_SFLOAT:
        g = gc.view(np.float32).reshape(-1)
        o = oc.view(np.float32).reshape(-1)
        ulp = np.abs(g.view(np.int32).astype(np.int64) - o.view(np.int32).astype(np.int64))
        assert ulp.max() <= FLOAT_ULP_TOL, f"max ulp {ulp.max()}"
    else:
        diff = np.argwhere(np.any(gc != oc, axis=-1))
        assert diff.size == 0, f"{len(diff)} pixels differ, first {diff[:5].tolist()}: " \
                               f"gpu {gc[tuple(diff[0])]} oracle {oc[tuple(diff[0])]}"
    if scene.depth:
        gdb, odb = gd[rows].view(np.uint32), od[rows].view(np.uint32)
        bad = np.argwhere(gdb != odb)
        assert bad.size == 0, f"{len(bad)} depth values differ, first {bad[:5].tolist()}"
    return gc, gd


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
