"""A second, independent restatement of the draw path in float64 (TEST
INFRASTRUCTURE ONLY): written from the Vulkan 1.3 rasterization rules and the
shader sources, sharing no code or formulas with oracle/zr_oracle.c or the
kernels.  Where those two evaluate an explicitly ordered float32 contract
(DESIGN.md §3), this one evaluates the mathematical definition in float64:

  - viewport transform (Vulkan 1.3 §Controlling the Viewport), snap to
    subPixelPrecisionBits = 8, facing = sign of the signed area, top-left rule
  - depth: z = sum b_i z_i with exact barycentrics b_i = E_i / A (screen-space
    linear), rounded once to the D32_SFLOAT attachment; fragments outside
    [minDepth, maxDepth] do not exist (z-plane clipping at w = 1)
  - the mesh program: clip = view_proj * (p, 1), perspective-correct weights
    b_i / w_i, depth z_ndc interpolated linearly in screen space
  - fragment programs in float64 (flat_color, blinn_phong, mesh .slang), sRGB
    OETF exactly, UNORM8 round to nearest
  - in-order depth test (LESS / GREATER) on the stored float32 depth

tests/test_second_opinion.py compares it with the oracle: coverage must match,
depth within 1 ulp and colour within 1 code wherever both pick the same
winner.  A shared misreading of Vulkan by the oracle and the kernels would show
up here as a systematic difference.
"""
from __future__ import annotations

import numpy as np

from zenith_amd import scenes


def srgb_code(c):
    """Linear [0,1] -> 8-bit sRGB code (KHR Data Format 13.3, round to nearest)."""
    c = np.clip(np.nan_to_num(c, nan=0.0), 0.0, 1.0)
    e = np.where(c <= 0.0031308, 12.92 * c, 1.055 * np.power(c, 1.0 / 2.4) - 0.055)
    return np.floor(e * 255.0 + 0.5).astype(np.int64)


L_DIR = np.array([0.3, 0.5, 0.8]) / np.linalg.norm([0.3, 0.5, 0.8])
H_DIR = (L_DIR + [0.0, 0.0, 1.0]) / np.linalg.norm(L_DIR + [0.0, 0.0, 1.0])


def blinn_phong(n, kd):
    """blinn_phong.slang / mesh.slang lighting: kd (0.05 + max(N.L, 0)) + 0.5 max(N.H, 0)^32."""
    ln = np.linalg.norm(n, axis=-1, keepdims=True)
    N = np.divide(n, ln, out=np.zeros_like(n), where=ln > 0)
    ndl = np.maximum(N @ L_DIR, 0.0)
    ndh = np.maximum(N @ H_DIR, 0.0)
    return kd * (0.05 + ndl)[:, None] + 0.5 * (ndh ** 32)[:, None]


class Frame:
    """Colour (float64 RGB, NaN = clear), depth (float32) and winner id per pixel."""

    def __init__(self, W, H, clear_depth):
        self.rgb = np.full((H, W, 3), np.nan)
        self.depth = np.full((H, W), clear_depth, np.float32)
        self.winner = np.full((H, W), -1, np.int64)
        # pixels where another fragment's depth came within 1 ulp of the winner's:
        # which one wins is up to float rounding, not to the rules
        self.near_tie = np.zeros((H, W), bool)

    def depth_test(self, px, py, z32, greater):
        cur = self.depth[py, px]
        close = np.abs(z32.view(np.int32).astype(np.int64) - cur.view(np.int32).astype(np.int64)) <= 1
        self.near_tie[py[close], px[close]] = True
        return (z32 > cur) if greater else (z32 < cur)


def _snap(xf):
    return np.rint(np.asarray(xf, np.float64) * 256.0).astype(np.int64)


def _edge_setup(X, Y):
    """Signed-area orientation and the three edge functions' coefficients.
    Returns None for a degenerate triangle, else (order, A) with A > 0 after
    ordering the vertices so that the interior is where every E_i >= 0."""
    A = (X[1] - X[0]) * (Y[2] - Y[0]) - (X[2] - X[0]) * (Y[1] - Y[0])
    if A == 0:
        return None
    return ([0, 1, 2] if A > 0 else [0, 2, 1]), abs(int(A))


def _cover(X, Y, order, x0, y0, x1, y1):
    """Samples (pixel centres) of the bbox inside the triangle, top-left rule
    (Vulkan: a sample on an edge belongs to the triangle iff the edge is a top or
    a left edge in the y-down framebuffer).  Returns (px, py, E[3]) with E the
    exact integer edge values, E_i opposite vertex order[i]."""
    px, py = np.meshgrid(np.arange(x0, x1 + 1), np.arange(y0, y1 + 1))
    px, py = px.ravel(), py.ravel()
    sx, sy = px * 256 + 128, py * 256 + 128
    xs = [X[k] for k in order]
    ys = [Y[k] for k in order]
    inside = np.ones(px.shape, bool)
    E = []
    for i in range(3):
        a, b = (i + 1) % 3, (i + 2) % 3
        ex, ey = xs[b] - xs[a], ys[b] - ys[a]
        e = ex * (sy - ys[a]) - ey * (sx - xs[a])
        top_left = ey < 0 or (ey == 0 and ex > 0)
        inside &= (e >= 0) if top_left else (e > 0)
        E.append(e)
    return px[inside], py[inside], [e[inside] for e in E]


def render_soup(scene):
    """Pass-through vertex stage (w = 1): flat_color / blinn_phong soups with a
    depth attachment, cull NONE, full viewport (0, 0, W, H, 0, 1)."""
    assert scene.program in (scenes.PROGRAM_FLAT_COLOR, scenes.PROGRAM_BLINN_PHONG)
    W, H = scene.width, scene.height
    v = scene.vertices.astype(np.float64)
    idx = scene.indices.astype(np.int64)
    f = Frame(W, H, scene.depth_clear)
    less = scene.depth_op == scenes.OP_LESS
    for t in range(idx.size // 3):
        tv = v[idx[3 * t:3 * t + 3]]
        # the viewport transform in float32 as a device evaluates it: one fused
        # multiply-add, i.e. the exact value x (W/2) + W/2 rounded once to float32
        # (exact in float64 for these magnitudes), then snapped
        xf = (tv[:, 0] * (W / 2.0) + W / 2.0).astype(np.float32)
        yf = (tv[:, 1] * (H / 2.0) + H / 2.0).astype(np.float32)
        zf = tv[:, 2]
        X, Y = _snap(xf), _snap(yf)
        es = _edge_setup(X, Y)
        if es is None:
            continue
        order, A = es
        x0 = max(0, int(np.ceil((X.min() - 128) / 256.0)))
        x1 = min(W - 1, int(np.floor((X.max() - 128) / 256.0)))
        y0 = max(0, int(np.ceil((Y.min() - 128) / 256.0)))
        y1 = min(H - 1, int(np.floor((Y.max() - 128) / 256.0)))
        if x0 > x1 or y0 > y1:
            continue
        px, py, E = _cover(X, Y, order, x0, y0, x1, y1)
        if px.size == 0:
            continue
        b = np.stack([E[i].astype(np.float64) / A for i in range(3)], axis=1)  # weight of order[i]
        zo = np.array([zf[k] for k in order])
        z = b @ zo
        keep = (z >= 0.0) & (z <= 1.0)
        z32 = z.astype(np.float32)
        keep &= f.depth_test(px, py, z32, not less)
        px, py, b, z32 = px[keep], py[keep], b[keep], z32[keep]
        if px.size == 0:
            continue
        f.depth[py, px] = z32
        f.winner[py, px] = t
        if scene.program == scenes.PROGRAM_FLAT_COLOR:
            f.rgb[py, px] = tv[0, 3:6]  # provoking vertex = first
        else:
            nrm = b @ tv[order][:, 3:6]
            kd = b @ tv[order][:, 6:9]
            f.rgb[py, px] = blinn_phong(nrm, kd)
    return f


def render_mesh(scene):
    """mesh.slang through scene.view_proj (column-major), depth GREATER / clear 0
    as the scenes use it (reverse-Z).  Returns (frame, n_clip): primitives that
    would need near/far clipping or lie behind the camera are not rendered but
    counted (the cerberus comparison asserts there are none)."""
    assert scene.program == scenes.PROGRAM_MESH
    W, H = scene.width, scene.height
    M = np.array(scene.view_proj, np.float64).reshape(4, 4).T  # row-major: clip = M @ (p, 1)
    v = scene.vertices.astype(np.float64)
    idx = scene.indices.astype(np.int64)
    f = Frame(W, H, scene.depth_clear)
    n_clip = 0
    greater = scene.depth_op == scenes.OP_GREATER
    for t in range(idx.size // 3):
        tv = v[idx[3 * t:3 * t + 3]]
        # the vertex stage's output is float32 (mesh.slang's float4 SV_Position)
        clip = (M @ np.concatenate([tv[:, 0:3], np.ones((3, 1))], axis=1).T).T.astype(np.float32).astype(np.float64)
        w = clip[:, 3]
        if (w <= 0).any() or (clip[:, 2] < 0).any() or (clip[:, 2] > w).any():
            n_clip += 1
            continue
        xf = (clip[:, 0] / w + 1.0) * (W / 2.0)
        yf = (clip[:, 1] / w + 1.0) * (H / 2.0)
        zn = clip[:, 2] / w
        X, Y = _snap(xf), _snap(yf)
        es = _edge_setup(X, Y)
        if es is None:
            continue
        order, A = es
        # cull BACK with CCW front faces: Vulkan's a = -A/2 (y-down), a > 0 is CCW
        A_signed = (X[1] - X[0]) * (Y[2] - Y[0]) - (X[2] - X[0]) * (Y[1] - Y[0])
        ccw = A_signed < 0
        front = ccw if scene.front_face == scenes.FRONT_CCW else not ccw
        if (scene.cull_mode == scenes.CULL_BACK and not front) or (scene.cull_mode == scenes.CULL_FRONT and front):
            continue
        x0 = max(0, int(np.ceil((X.min() - 128) / 256.0)))
        x1 = min(W - 1, int(np.floor((X.max() - 128) / 256.0)))
        y0 = max(0, int(np.ceil((Y.min() - 128) / 256.0)))
        y1 = min(H - 1, int(np.floor((Y.max() - 128) / 256.0)))
        if x0 > x1 or y0 > y1:
            continue
        px, py, E = _cover(X, Y, order, x0, y0, x1, y1)
        if px.size == 0:
            continue
        bs = np.stack([E[i].astype(np.float64) / A for i in range(3)], axis=1)  # screen weights of order[i]
        z = bs @ np.array([zn[k] for k in order])
        keep = (z >= 0.0) & (z <= 1.0)
        z32 = z.astype(np.float32)
        keep &= f.depth_test(px, py, z32, greater)
        px, py, bs, z32 = px[keep], py[keep], bs[keep], z32[keep]
        if px.size == 0:
            continue
        # perspective-correct weights of the unsnapped primitive (the snap decides
        # coverage only; Vulkan leaves the interpolation positions' precision to
        # the implementation): the homogeneous screen vertices h_k, and
        # b_k proportional to p . (h_{k+1} x h_{k+2}) at the sample p
        h = np.stack([(clip[:, 0] + clip[:, 3]) * (W / 2.0), (clip[:, 1] + clip[:, 3]) * (H / 2.0), clip[:, 3]], 1)
        pts = np.stack([px + 0.5, py + 0.5, np.ones(px.size)], axis=1)
        pw = np.stack([pts @ np.cross(h[(k + 1) % 3], h[(k + 2) % 3]) for k in range(3)], axis=1)
        pw /= pw.sum(axis=1, keepdims=True)
        vo = tv
        nrm = pw @ vo[:, 3:6]
        uv = pw @ vo[:, 6:8]
        kd = np.stack([0.35 + 0.3 * uv[:, 0], 0.35 + 0.3 * uv[:, 1], np.full(len(uv), 0.7)], axis=1)
        f.depth[py, px] = z32
        f.winner[py, px] = t
        f.rgb[py, px] = blinn_phong(nrm, kd)
    return f, n_clip


def codes_rgb(frame):
    """8-bit sRGB codes (RGB) of a second-opinion frame; clear pixels = -1."""
    out = np.full(frame.rgb.shape, -1, np.int64)
    m = ~np.isnan(frame.rgb[..., 0])
    out[m] = srgb_code(frame.rgb[m])
    return out


def ulp_distance(a, b):
    """|a - b| in float32 ulps (both non-negative finite float32 arrays)."""
    return np.abs(a.astype(np.float32).view(np.int32).astype(np.int64) -
                  b.astype(np.float32).view(np.int32).astype(np.int64))
