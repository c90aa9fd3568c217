"""The oracle against an independent float64 restatement (tests/second_opinion.py).

The oracle and the kernels implement one hand-written float32 contract (DESIGN.md
§3), bit for bit.  These tests check that contract against a second reading of
the Vulkan rules, written separately in float64 numpy, on small soups shaped
like C1 (flat colour, ~12 px triangles) and C2 (Blinn-Phong, ~6 px triangles) and
on the reference's cerberus mesh through the camera program:

  - coverage: the same pixels are covered (exact integer edge tests on both
    sides; a vertex whose float32 and float64 viewport coordinates snap to
    different 1/256 steps may move a boundary pixel: <= 0.05 % of pixels);
  - winners: both pick the same primitive almost everywhere (a different winner
    only where two fragments' depths are within rounding of each other);
  - where the winners agree: colour within 1 code, and depth within 2^-23 (one
    float32 ulp at 1.0) of the float64 value -- within 1 ulp of it for >= 95 %
    of the pixels; the rest are small depths, where the contract's float32
    barycentric evaluation spends a few ulps.

The reference ships no fixtures, so parity stays "unpinned";
this lowers the risk that the oracle and the kernels share a misreading.
"""
import numpy as np
import pytest

from oracle import oracle
from tests import second_opinion as so
from zenith_amd import scenes


def _oracle_winners(scene):
    """The oracle's winning primitive per pixel: the same scene drawn with the
    flat program into R32G32B32A32, each primitive's provoking colour = its id."""
    v = scene.vertices.copy()
    idx = scene.indices.astype(np.int64)
    ids = np.full(v.shape[0], -1.0, np.float32)
    ids[idx[0::3]] = np.arange(idx.size // 3, dtype=np.float32)  # soups: vertex 3t is t's provoking vertex
    v2 = np.zeros((v.shape[0], 6), np.float32)
    v2[:, 0:3] = v[:, 0:3]
    v2[:, 3] = ids
    s = scenes.Scene(scene.name + "_ids", scene.width, scene.height, scenes.PROGRAM_FLAT_COLOR, v2,
                     scene.indices, color_format=scenes.FMT_R32G32B32A32_SFLOAT, clear_color=(-1.0, 0, 0, 1),
                     depth=True, depth_op=scene.depth_op, depth_clear=scene.depth_clear, cull_mode=scene.cull_mode)
    col, _ = oracle.render(s)
    return col.view(np.float32).reshape(scene.height, scene.width, 4)[..., 0].astype(np.int64)


def _compare(scene, ref, max_cov_frac=5e-4, min_same_frac=0.999):
    col, dep = oracle.render(scene)
    rgb = col[..., [2, 1, 0]].astype(np.int64)  # B8G8R8A8_SRGB -> RGB codes
    clear = scene.depth_clear
    cov_o = dep != np.float32(clear)
    cov_s = ref.depth != np.float32(clear)
    n_px = scene.width * scene.height
    assert cov_s.sum() > n_px // 4, "scene too sparse to say anything"
    assert (cov_o != cov_s).sum() <= max(2, int(max_cov_frac * n_px)), (int(cov_o.sum()), int(cov_s.sum()))
    win_o = _oracle_winners(scene)
    both = cov_o & cov_s
    same = both & (win_o == ref.winner)
    assert same.sum() >= min_same_frac * both.sum(), (int(same.sum()), int(both.sum()))
    ulp = so.ulp_distance(dep[same], ref.depth[same])
    err = np.abs(dep[same].astype(np.float64) - ref.depth[same].astype(np.float64))
    assert err.max() <= 2.0 ** -23, f"depth: {int((err > 2.0 ** -23).sum())} pixels beyond 2^-23"
    assert np.mean(ulp <= 1) >= 0.95, f"depth: only {np.mean(ulp <= 1):.4f} within 1 ulp"
    codes = so.codes_rgb(ref)
    d = np.abs(rgb[same] - codes[same])
    assert d.max() <= 1, f"colour: {int((d > 1).sum())} pixels beyond 1 code (max {int(d.max())})"
    return int(same.sum()), float(np.mean(ulp == 0)), float(np.mean(d == 0))


@pytest.mark.parametrize("seed", [101, 102])
def test_flat_soup_c1_shaped(seed):
    """C1-shaped: flat colour (provoking vertex), D32 LESS, ~12 px triangles."""
    s = scenes.soup_scene(seed, 3000, 320, 180, 12.0 * 320 / 1920 * 4, scenes.PROGRAM_FLAT_COLOR)
    n, z_exact, c_exact = _compare(s, so.render_soup(s))
    assert n > 20000 and c_exact > 0.999  # flat colours are exact float32 inputs


@pytest.mark.parametrize("seed", [103, 104])
def test_blinn_soup_c2_shaped(seed):
    """C2-shaped: per-pixel Blinn-Phong from interpolated normals and colours."""
    s = scenes.soup_scene(seed, 12000, 256, 144, 6.0 * 256 / 1920 * 4, scenes.PROGRAM_BLINN_PHONG)
    n, z_exact, c_exact = _compare(s, so.render_soup(s))
    assert n > 15000 and c_exact > 0.95


def test_cerberus_camera_mesh():
    """The reference's cerberus asset (33,543 triangles) through mesh.slang's
    camera at 320x240: perspective-correct shading and reverse-Z depth."""
    s = scenes.cerberus_scene(320, 240)
    ref, n_clip = so.render_mesh(s)
    assert n_clip == 0  # the view needs no near/far clipping: the comparison is complete
    col, dep = oracle.render(s)
    rgb = col[..., [2, 1, 0]].astype(np.int64)
    cov_o, cov_s = dep > 0, ref.depth > 0
    assert cov_s.sum() > 5000
    assert (cov_o != cov_s).sum() <= max(4, int(1e-3 * cov_s.sum()))
    both = cov_o & cov_s & ~ref.near_tie
    assert both.sum() >= 0.99 * cov_s.sum()
    # reverse-Z depth = near / w is small (~3e-4 here): an absolute bound of 2^-23
    # says little, so the relative one -- z / w rounded per vertex, then the
    # float32 screen-space interpolation -- is checked too
    # (the float32 plane evaluation cancels at these small depths: with the camera
    # matrix formed as glam forms it -- f32 products and sums in Mat4::mul_vec4's
    # order, scenes.view_projection -- 6 of ~7800 pixels lie 33-97 ulp from
    # float64, all within 2.9e-9 absolute; the 99th percentile is 4 ulp)
    ulp = so.ulp_distance(dep[both], ref.depth[both])
    err = np.abs(dep[both].astype(np.float64) - ref.depth[both].astype(np.float64))
    assert err.max() <= 2.0 ** -23 and ulp.max() <= 128, (float(err.max()), int(ulp.max()))
    assert np.percentile(ulp, 99) <= 8
    assert np.mean(ulp <= 1) >= 0.95
    codes = so.codes_rgb(ref)
    d = np.abs(rgb[both] - codes[both])
    assert d.max() <= 1, f"colour: {int((d > 1).sum())} pixels beyond 1 code"


def test_zplane_discard_equals_exact_clip_at_w1():
    """at w = 1 the depth planes z = 0 and z = 1 are lines of
    constant interpolated depth in screen space, so discarding samples whose
    depth leaves [0, 1] keeps exactly the samples of the triangle clipped
    against those planes -- Vulkan's clip volume -- without snapping new
    vertices.  Checked against the exact sample set in rationals on triangles
    crossing both planes."""
    from fractions import Fraction as F
    rng = np.random.default_rng(7)
    checked = 0
    for _ in range(6):
        p = rng.uniform(-0.9, 0.9, (3, 2))
        z = np.array([rng.uniform(-0.8, -0.1), rng.uniform(1.1, 1.6), rng.uniform(0.2, 0.8)])
        v = np.zeros((3, 6), np.float32)
        v[:, 0:2], v[:, 2], v[:, 3:6] = p, z, 1.0
        s = scenes.Scene("zclip", 64, 48, scenes.PROGRAM_FLAT_COLOR, v, np.arange(3, dtype=np.uint32),
                         color_format=scenes.FMT_R8G8B8A8_UNORM, depth=True, depth_op=scenes.OP_ALWAYS)
        _, dep = oracle.render(s)
        got = dep != np.float32(1.0)  # ALWAYS + write: every kept sample writes its depth
        # exact: snapped vertices (as the oracle snaps), exact barycentrics, exact z
        X = [int(np.rint(np.float32(np.float32(x) * np.float32(32.0) + np.float32(32.0)) * 256)) for x in v[:, 0]]
        Y = [int(np.rint(np.float32(np.float32(y) * np.float32(24.0) + np.float32(24.0)) * 256)) for y in v[:, 1]]
        zs = [F(float(q)) for q in v[:, 2]]
        A = (X[1] - X[0]) * (Y[2] - Y[0]) - (X[2] - X[0]) * (Y[1] - Y[0])
        order = [0, 1, 2] if A > 0 else [0, 2, 1]
        A = abs(A)
        ref = np.zeros((48, 64), bool)
        for py in range(48):
            for px in range(64):
                sx, sy = px * 256 + 128, py * 256 + 128
                E, inside = [], True
                for i in range(3):
                    a, b = order[(i + 1) % 3], order[(i + 2) % 3]
                    ex, ey = X[b] - X[a], Y[b] - Y[a]
                    e = ex * (sy - Y[a]) - ey * (sx - X[a])
                    tl = ey < 0 or (ey == 0 and ex > 0)
                    inside &= (e >= 0) if tl else (e > 0)
                    E.append(e)
                if not inside:
                    continue
                zz = sum(F(E[i], A) * zs[order[i]] for i in range(3))
                ref[py, px] = 0 <= zz <= 1
        assert ref.sum() > 20
        # only samples whose exact depth lies within float rounding of a plane may differ
        assert (got != ref).sum() <= 2, int((got != ref).sum())
        checked += int(ref.sum())
    assert checked > 500
