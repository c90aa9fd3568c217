"""Synthetic scenes for the draw path (BASELINE.json ``configs``).

Everything here is host-side workload generation (numpy), shared by the tests, the
bench and the goldens.  Scenes are plain data: interleaved vertex bytes, index
bytes and the pipeline/render-pass parameters that ``triangle.rs`` (or the config
table) would set.  Nothing here rasterizes.

Random soups follow SURVEY.md §8d exactly: a counter-based SplitMix64 stream,
``float = (u >> 40) * 2^-24``, 32 draws per triangle at fixed offsets (so any
triangle can be generated independently and in parallel).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

# VkFormat / Vk enums used in scene descriptions (numeric Vulkan values).
FMT_R8G8B8A8_UNORM = 37
FMT_R8G8B8A8_SRGB = 43
FMT_B8G8R8A8_UNORM = 44
FMT_B8G8R8A8_SRGB = 50
FMT_R32G32B32A32_SFLOAT = 109
FMT_D32_SFLOAT = 126
FMT_R32G32B32_SFLOAT = 106

CULL_NONE, CULL_FRONT, CULL_BACK = 0, 1, 2
FRONT_CCW, FRONT_CW = 0, 1
OP_NEVER, OP_LESS, OP_EQUAL, OP_LEQUAL, OP_GREATER, OP_NOTEQUAL, OP_GEQUAL, OP_ALWAYS = range(8)
INDEX_U16, INDEX_U32 = 0, 1
LOAD_LOAD, LOAD_CLEAR, LOAD_DONT_CARE = 0, 1, 2

PROGRAM_TRIANGLE, PROGRAM_FLAT_COLOR, PROGRAM_BLINN_PHONG, PROGRAM_MESH = 0, 1, 2, 3
PROGRAM_FILES = {
    PROGRAM_TRIANGLE: "content/shaders/triangle.slang",
    PROGRAM_FLAT_COLOR: "content/shaders/flat_color.slang",
    PROGRAM_BLINN_PHONG: "content/shaders/blinn_phong.slang",
    PROGRAM_MESH: "content/shaders/mesh.slang",
}
# float components of each vertex input, location order
PROGRAM_LAYOUT = {PROGRAM_TRIANGLE: (3, 3), PROGRAM_FLAT_COLOR: (3, 3), PROGRAM_BLINN_PHONG: (3, 3, 3),
                  PROGRAM_MESH: (3, 3, 2)}  # mesh: zenith-asset Vertex {position, normal, uv}
PROGRAM_ATTRS = {k: len(v) for k, v in PROGRAM_LAYOUT.items()}


@dataclasses.dataclass
class Scene:
    """One render pass with one draw, as ``TriangleRenderer::render_to`` records it."""

    name: str
    width: int
    height: int
    program: int
    vertices: np.ndarray          # float32 [V, 3*attrs] interleaved, location order
    indices: np.ndarray | None    # uint16/uint32 [I] or None for a non-indexed draw
    color_format: int = FMT_B8G8R8A8_SRGB
    clear_color: tuple = (0.1, 0.1, 0.1, 1.0)       # triangle.rs:110-113
    cull_mode: int = CULL_NONE                       # triangle.rs:116
    front_face: int = FRONT_CCW                      # pipeline.rs:520-533 default
    depth: bool = False                              # DepthStencilDesc present?
    depth_test: bool = True
    depth_write: bool = True
    depth_op: int = OP_LESS                          # pipeline.rs:435-453 default
    depth_clear: float = 1.0
    time: float = 0.0                                # Time.time, pinned for goldens
    write_mask: int = 0xF
    instance_count: int = 1                          # draw_indexed(count, instances, first, offset, 0)
    first: int = 0                                   # first_index / first_vertex
    vertex_offset: int = 0
    count: int | None = None                         # default: all indices / vertices
    view_proj: tuple | None = None                   # mesh program: View.view_proj, 16 floats column-major
    push_view: bool = False                          # mesh program: view_proj as push constants (mesh_push.slang)

    @property
    def layout(self) -> tuple:
        return PROGRAM_LAYOUT[self.program]

    @property
    def stride(self) -> int:
        return 4 * sum(self.layout)

    @property
    def index_type(self) -> int:
        if self.indices is None:
            return -1
        return INDEX_U16 if self.indices.dtype == np.uint16 else INDEX_U32

    @property
    def draw_count(self) -> int:
        if self.count is not None:
            return int(self.count)
        return int(self.indices.size if self.indices is not None else self.vertices.shape[0])

    @property
    def triangles(self) -> int:
        return (self.draw_count // 3) * self.instance_count

    def vertex_bytes(self) -> bytes:
        return np.ascontiguousarray(self.vertices, dtype=np.float32).tobytes()

    def index_bytes(self) -> bytes:
        return b"" if self.indices is None else np.ascontiguousarray(self.indices).tobytes()


# ---------------------------------------------------------------- C0 scenes

def triangle_scene(width: int = 640, height: int = 480, time: float = 0.0) -> Scene:
    """The reference's only scene: zenith-renderer/src/triangle.rs:28-33 (3 verts,
    u16 indices [0,1,2]), clear [.1,.1,.1,1], cull NONE, no depth attachment."""
    verts = np.array(
        [[0.0, 0.5, 0.0, 1.0, 0.0, 0.0],
         [-0.5, -0.5, 0.0, 0.0, 1.0, 0.0],
         [0.5, -0.5, 0.0, 0.0, 0.0, 1.0]], dtype=np.float32)
    idx = np.array([0, 1, 2], dtype=np.uint16)
    return Scene("triangle", width, height, PROGRAM_TRIANGLE, verts, idx, time=time)


def cube_scene(width: int = 640, height: int = 480, angle_deg: float = 30.0) -> Scene:
    """Synthetic 12-triangle cube (content/mesh has no cube).

    The vertex stage is pass-through, so the cube is rotated and projected on the
    host (orthographic, z mapped into [0.2, 0.8]); faces are wound CCW in Vulkan's
    sense and drawn with cull BACK + depth LESS, one flat colour per face."""
    a = math.radians(angle_deg)
    b = math.radians(angle_deg * 0.7)
    ry = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    rx = np.array([[1, 0, 0], [0, math.cos(b), -math.sin(b)], [0, math.sin(b), math.cos(b)]])
    corners = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], dtype=np.float64)
    p = corners @ (rx @ ry).T * 0.45
    aspect = width / height
    ndc = np.stack([p[:, 0] / aspect, p[:, 1], 0.5 + p[:, 2] * 0.35], axis=1)
    # faces as corner quads (outward normals), split into two triangles each
    faces = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    colors = [(1, 0.2, 0.2), (0.2, 1, 0.2), (0.2, 0.2, 1), (1, 1, 0.2), (1, 0.2, 1), (0.2, 1, 1)]
    verts, idx = [], []
    for f, col in zip(faces, colors):
        quad = [f[0], f[1], f[2], f[3]]
        for tri in ((0, 1, 2), (0, 2, 3)):
            for k in tri:
                idx.append(len(verts))
                verts.append([*ndc[quad[k]], *col])
    v = np.array(verts, dtype=np.float32)
    i = np.array(idx, dtype=np.uint16)
    s = Scene("cube", width, height, PROGRAM_FLAT_COLOR, v, i, cull_mode=CULL_BACK, depth=True)
    # pick the winding that leaves the camera-facing faces (|z| smaller = nearer) CCW
    s.front_face = _front_face_for_nearer(v, i, width, height)
    return s


def _front_face_for_nearer(v, i, w, h):
    tri = v[i.astype(np.int64)].reshape(-1, 3, 6)
    xf = (tri[:, :, 0] * 0.5 + 0.5) * w
    yf = (tri[:, :, 1] * 0.5 + 0.5) * h
    a2 = (xf[:, 1] - xf[:, 0]) * (yf[:, 2] - yf[:, 0]) - (xf[:, 2] - xf[:, 0]) * (yf[:, 1] - yf[:, 0])
    zc = tri[:, :, 2].mean(axis=1)
    near = zc < np.median(zc)
    ccw = a2 < 0  # Vulkan: a = -A2/2 > 0 is counter-clockwise
    return FRONT_CCW if (ccw[near].mean() >= 0.5) else FRONT_CW


# ------------------------------------------------------------- random soups

_GOLD = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, counters: np.ndarray) -> np.ndarray:
    """Counter-based SplitMix64: value i = mix(seed + (i+1)*golden)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (counters.astype(np.uint64) + np.uint64(1)) * _GOLD
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform(seed: int, counters: np.ndarray) -> np.ndarray:
    u = splitmix64(seed, counters)
    return (u >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


def soup_arrays(seed: int, n: int, width: int, height: int, L: float, normals: bool,
                first: int = 0) -> np.ndarray:
    """Per-vertex interleaved float32 rows for triangles [first, first+n)."""
    t = np.arange(first, first + n, dtype=np.uint64)
    base = t * np.uint64(32)

    def U(off):
        return _uniform(seed, base + np.uint64(off))

    cx = U(0) * 2.0 - 1.0
    cy = U(1) * 2.0 - 1.0
    ex, ey = 2.0 * L / width, 2.0 * L / height
    cols = 9 if normals else 6
    out = np.empty((n, 3, cols), dtype=np.float32)
    for k in range(3):
        o = 2 + 10 * k
        out[:, k, 0] = cx + (U(o) * 2.0 - 1.0) * ex
        out[:, k, 1] = cy + (U(o + 1) * 2.0 - 1.0) * ey
        out[:, k, 2] = 0.05 + U(o + 2) * 0.9
        ccol = 6 if normals else 3
        out[:, k, ccol] = U(o + 3)
        out[:, k, ccol + 1] = U(o + 4)
        out[:, k, ccol + 2] = U(o + 5)
        if normals:
            u1 = np.maximum(U(o + 6), 2.0 ** -24)
            u2 = U(o + 7)
            u3 = np.maximum(U(o + 8), 2.0 ** -24)
            u4 = U(o + 9)
            r1 = np.sqrt(-2.0 * np.log(u1))
            r2 = np.sqrt(-2.0 * np.log(u3))
            g = np.stack([r1 * np.cos(2 * np.pi * u2), r1 * np.sin(2 * np.pi * u2),
                          r2 * np.cos(2 * np.pi * u4)], axis=1)
            g /= np.maximum(np.linalg.norm(g, axis=1, keepdims=True), 1e-30)
            out[:, k, 3:6] = g
    return out.reshape(n * 3, cols)


def clustered_scene(seed: int, n: int, width: int, height: int, L: float, program: int, sigma: float = 0.12,
                    name: str | None = None) -> Scene:
    """A soup whose triangle centres are Gaussian around the screen centre
    (sigma in NDC units, clipped to [-1, 1]) instead of uniform: a skewed scene
    whose central tiles hold many times the mean list length (the bin layout's
    worst case: DESIGN.md §4).  Same per-vertex stream
    as soup_scene otherwise."""
    verts = soup_arrays(seed, n, width, height, L, program == PROGRAM_BLINN_PHONG).reshape(n, 3, -1)
    t = np.arange(n, dtype=np.uint64) * np.uint64(32)
    u1 = np.maximum(_uniform(seed + 7919, t + np.uint64(30)), 2.0 ** -24)
    u2 = _uniform(seed + 7919, t + np.uint64(31))
    r = np.sqrt(-2.0 * np.log(u1)) * sigma
    c = np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)], axis=1)
    c = np.clip(c, -1.0, 1.0)
    old_c = verts[:, :, :2].mean(axis=1, keepdims=True)
    verts[:, :, :2] += (c[:, None, :] - old_c).astype(np.float32)
    return Scene(name or f"clustered_s{seed}_n{n}", width, height, program, verts.reshape(3 * n, -1),
                 np.arange(3 * n, dtype=np.uint32), depth=True, cull_mode=CULL_NONE)


CONFIGS = {
    # id: (seed, triangles, width, height, L px, program)   SURVEY.md §8d table
    "c1": (1, 100_000, 1920, 1080, 12.0, PROGRAM_FLAT_COLOR),
    "c2": (2, 1_000_000, 1920, 1080, 6.0, PROGRAM_BLINN_PHONG),
    "c3": (3, 1_000_000, 3840, 2160, 12.0, PROGRAM_BLINN_PHONG),
    "c4": (4, 10_000_000, 1920, 1080, 0.5, PROGRAM_FLAT_COLOR),
    # not a BASELINE config: the reference's real asset through the camera program
    # (SURVEY.md §8f rows 2-3), 33,543 triangles at 1080p
    "cerberus": (None, 33_543, 1920, 1080, None, PROGRAM_MESH),
    # not BASELINE configs: C2's and C3's triangles, Gaussian-clustered (clustered_scene)
    "c2x": (12, 1_000_000, 1920, 1080, 6.0, PROGRAM_BLINN_PHONG),
    "c3x": (13, 1_000_000, 3840, 2160, 12.0, PROGRAM_BLINN_PHONG),
}


def soup_scene(seed: int, n: int, width: int, height: int, L: float, program: int,
               name: str | None = None) -> Scene:
    normals = program == PROGRAM_BLINN_PHONG
    verts = soup_arrays(seed, n, width, height, L, normals)
    idx = np.arange(3 * n, dtype=np.uint32)
    return Scene(name or f"soup_s{seed}_n{n}", width, height, program, verts, idx,
                 depth=True, cull_mode=CULL_NONE)


def config_scene(cfg: str, n: int | None = None, width: int | None = None,
                 height: int | None = None) -> Scene:
    seed, tris, w, h, L, prog = CONFIGS[cfg]
    if cfg == "cerberus":
        return cerberus_scene(width or w, height or h)
    if cfg.endswith("x"):
        return clustered_scene(seed, n or tris, width or w, height or h, L, prog, name=cfg)
    return soup_scene(seed, n or tris, width or w, height or h, L, prog, name=cfg)


def config_bytes_per_triangle(cfg: str) -> int:
    """B_in of SURVEY.md §8d: 3 vertices at the stride + 3 u32 indices."""
    prog = CONFIGS[cfg][5]
    return 3 * 4 * sum(PROGRAM_LAYOUT[prog]) + 3 * 4


# ------------------------------------------------------------------ camera
# zenith-core/src/camera.rs: Camera::view_projection = proj * view (:85-87) with
# proj = Mat4::perspective_infinite_reverse_rh(fov_y, aspect, near) (:50, :60) and
# view = Mat4::look_to_rh(position, forward, WORLD_SPACE_UP = +Z) (:121-124), in
# glam 0.30's column-major layout, restated in float32 operation by operation as
# glam's scalar code computes them (Rust does not contract a * b + c into an FMA):
# Vec3::dot = (x x' + y y') + z z', Vec3::cross, Vec3::normalize = v * (1 / length),
# and Mat4 * Mat4 column by column as Mat4::mul_vec4 does,
# ((A.x * b.x + A.y * b.y) + A.z * b.z) + A.w * b.w, every product and sum rounded
# to f32 (tests/test_oracle.py::test_view_projection_f32_bits).
NEAR_PLANE = 0.1          # camera.rs:16
WORLD_UP = (0.0, 0.0, 1.0)
_F = np.float32


def _dot3(a, b):
    return (_F(a[0]) * _F(b[0]) + _F(a[1]) * _F(b[1])) + _F(a[2]) * _F(b[2])


def _cross3(a, b):
    a, b = [_F(x) for x in a], [_F(x) for x in b]
    return (a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1])


def _normalize3(v):
    r = _F(1.0) / _F(np.sqrt(_dot3(v, v)))  # Vec3::length_recip: 1 / sqrt(dot), f32
    return tuple(_F(x) * r for x in v)


def perspective_infinite_reverse_rh(fov_y: float, aspect: float, z_near: float) -> np.ndarray:
    """glam Mat4::perspective_infinite_reverse_rh: columns
    (f/aspect,0,0,0), (0,f,0,0), (0,0,0,-1), (0,0,z_near,0), f = 1/tan(fov_y/2)
    (f32::tan: the float64 tangent of the f32 argument, rounded once)."""
    f = _F(1.0) / _F(math.tan(_F(0.5) * _F(fov_y)))
    m = np.zeros((4, 4), np.float32)  # m[col][row]
    m[0, 0] = f / _F(aspect)
    m[1, 1] = f
    m[2, 3] = -1.0
    m[3, 2] = _F(z_near)
    return m


def look_to_rh(eye, direction, up) -> np.ndarray:
    """glam Mat4::look_to_rh: f = normalize(dir), s = normalize(f x up), u = s x f;
    columns (s.x,u.x,-f.x,0), (s.y,u.y,-f.y,0), (s.z,u.z,-f.z,0),
    (-dot(eye,s), -dot(eye,u), dot(eye,f), 1)."""
    e = tuple(_F(x) for x in eye)
    f = _normalize3(direction)
    s_ = _normalize3(_cross3(f, up))
    u = _cross3(s_, f)
    m = np.zeros((4, 4), np.float32)
    m[0] = (s_[0], u[0], -f[0], 0.0)
    m[1] = (s_[1], u[1], -f[1], 0.0)
    m[2] = (s_[2], u[2], -f[2], 0.0)
    m[3] = (-_dot3(e, s_), -_dot3(e, u), _dot3(e, f), 1.0)
    return m


def mat4_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """glam Mat4 * Mat4 (column-major m[col][row]): column c of the product is
    Mat4::mul_vec4(a, b[c]) = ((a.x * b.x + a.y * b.y) + a.z * b.z) + a.w * b.w,
    componentwise in f32 (products and sums each rounded)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    out = np.zeros((4, 4), np.float32)
    for c in range(4):
        col = a[0] * b[c, 0]
        col = col + a[1] * b[c, 1]
        col = col + a[2] * b[c, 2]
        col = col + a[3] * b[c, 3]
        out[c] = col
    return out


def view_projection(eye, forward, fov_y=math.pi / 6, aspect=1.77777, z_near=NEAR_PLANE) -> tuple:
    """Camera::view_projection = proj * view as 16 column-major floats (the View
    uniform's bytes)."""
    proj = perspective_infinite_reverse_rh(fov_y, aspect, z_near)
    view = look_to_rh(eye, forward, WORLD_UP)
    return tuple(float(x) for x in mat4_mul(proj, view).reshape(-1))


def mesh_soup_scene(seed: int, n: int, width: int, height: int, extent: float = 6.0,
                    eye=(0.0, -3.0, 0.5), forward=(0.0, 1.0, -0.1), name: str | None = None) -> Scene:
    """Camera-space test scene for the mesh program: n triangles with vertices
    scattered in a box in front of (and around) the camera, so primitives cross
    the near plane, lie behind the camera or straddle the view edges.  Reverse-Z:
    depth GREATER, clear 0 (camera.rs:50), cull BACK / CCW front (pipeline.rs
    defaults)."""
    g = np.random.default_rng(seed)
    c = g.uniform((-extent, -4.0, -extent / 2), (extent, 12.0, extent / 2), (n, 1, 3))
    d = g.uniform(-1.5, 1.5, (n, 3, 3))
    pos = (c + d).reshape(-1, 3).astype(np.float32)
    nrm = g.normal(size=(3 * n, 3)).astype(np.float32)
    uv = g.uniform(0.0, 1.0, (3 * n, 2)).astype(np.float32)
    verts = np.concatenate([pos, nrm, uv], axis=1)
    vp = view_projection(eye, forward, aspect=width / height)
    return Scene(name or f"mesh_soup_s{seed}_n{n}", width, height, PROGRAM_MESH, verts,
                 np.arange(3 * n, dtype=np.uint32), depth=True, depth_op=OP_GREATER, depth_clear=0.0,
                 cull_mode=CULL_BACK, view_proj=vp)


CERBERUS_NPZ = "tests/golden/cerberus.mesh.npz"  # relative to the repo root


def mesh_scene(vertices: np.ndarray, indices: np.ndarray, width: int, height: int, eye, forward,
               name: str = "mesh", fov_y: float = math.pi / 6) -> Scene:
    """A baked Mesh<Vertex> (zenith_amd.assets) through a camera: reverse-Z depth
    (GREATER, clear 0), cull BACK with CCW front faces, clear (0.1, 0.1, 0.1, 1)."""
    vp = view_projection(eye, forward, fov_y=fov_y, aspect=width / height)
    return Scene(name, width, height, PROGRAM_MESH, np.ascontiguousarray(vertices, np.float32),
                 np.ascontiguousarray(indices, np.uint32), depth=True, depth_op=OP_GREATER, depth_clear=0.0,
                 cull_mode=CULL_BACK, view_proj=vp)


def cerberus_scene(width: int = 640, height: int = 480, eye=(291.6, -31.5, 111.9), target=(-3.7, -52.2, -14.2),
                   npz: str | None = None) -> Scene:
    """content/mesh/cerberus (33,543 triangles, CC-BY-4.0, tests/golden/CERBERUS.txt)
    baked as gltf_loader.rs does, seen by a camera at `eye` looking at `target`.
    `npz`: the fixture (default) or a baked ``.mesh`` file (assets.bake_gltf)."""
    import os
    path = npz or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), CERBERUS_NPZ)
    if path.endswith(".mesh"):  # zenith-asset's baked file (assets.load_mesh)
        from .assets import load_mesh
        v, i, _ = load_mesh(path)
    else:
        with np.load(path, allow_pickle=False) as z:
            v, i = z["vertices"], z["indices"]
    fwd = tuple(float(t - e) for t, e in zip(target, eye))
    return mesh_scene(v, i, width, height, eye, fwd, name=f"cerberus_{width}x{height}")
