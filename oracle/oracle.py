"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module; the product (zenith_amd/) never does.  See zr_oracle.h for the contract
and the reference citations.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


class _Target(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("color_format", C.c_int32),
                ("color", C.c_void_p), ("depth", C.c_void_p)]


class _VertexInput(C.Structure):
    _fields_ = [("vertex_data", C.c_void_p), ("vertex_bytes", C.c_uint64), ("stride", C.c_uint32),
                ("attr_count", C.c_uint32), ("attr_offset", C.c_uint32 * 4), ("attr_size", C.c_uint32 * 4),
                ("index_data", C.c_void_p), ("index_bytes", C.c_uint64), ("index_type", C.c_int32)]


class _DrawState(C.Structure):
    _fields_ = [("program", C.c_int32), ("time", C.c_float), ("viewport", C.c_float * 6),
                ("scissor", C.c_int32 * 4), ("render_area", C.c_int32 * 4),
                ("cull_mode", C.c_uint32), ("front_face", C.c_int32),
                ("depth_test", C.c_uint32), ("depth_write", C.c_uint32), ("depth_op", C.c_int32),
                ("color_write_mask", C.c_uint32), ("tile_size", C.c_uint32),
                ("shard_rank", C.c_uint32), ("shard_count", C.c_uint32), ("view_proj", C.c_float * 16)]


class _DrawCmd(C.Structure):
    _fields_ = [("count", C.c_uint32), ("instance_count", C.c_uint32), ("first", C.c_uint32),
                ("vertex_offset", C.c_int32), ("first_instance", C.c_uint32), ("indexed", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("triangles_in", C.c_uint64), ("triangles_setup", C.c_uint64),
                ("fragments_covered", C.c_uint64), ("fragments_passed", C.c_uint64),
                ("triangles_dropped_clip", C.c_uint64)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.zro_snap.argtypes = [C.c_float]
        L.zro_snap.restype = C.c_int32
        L.zro_sinf.argtypes = [C.c_float]
        L.zro_sinf.restype = C.c_float
        L.zro_encode_unorm8.argtypes = [C.c_float]
        L.zro_encode_unorm8.restype = C.c_uint32
        L.zro_encode_srgb8.argtypes = [C.c_float]
        L.zro_encode_srgb8.restype = C.c_uint32
        L.zro_srgb_threshold.argtypes = [C.c_uint32]
        L.zro_srgb_threshold.restype = C.c_float
        L.zro_signed_area2.argtypes = [C.POINTER(C.c_float)]
        L.zro_signed_area2.restype = C.c_int64
        L.zro_format_bpp.argtypes = [C.c_int32]
        L.zro_format_bpp.restype = C.c_uint32
        L.zro_clear.argtypes = [C.POINTER(_Target), C.POINTER(C.c_int32 * 4), C.POINTER(C.c_float * 4),
                                C.c_int, C.c_float, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32]
        L.zro_clear.restype = None
        L.zro_draw.argtypes = [C.POINTER(_Target), C.POINTER(_DrawState), C.POINTER(_VertexInput),
                               C.POINTER(_DrawCmd), C.c_int, C.POINTER(Stats)]
        L.zro_draw.restype = C.c_int
        _lib = L
    return _lib


def snap(x: float) -> int:
    return lib().zro_snap(x)


def sinf(x: float) -> float:
    return lib().zro_sinf(x)


def encode_srgb8(c: float) -> int:
    return lib().zro_encode_srgb8(c)


def encode_unorm8(c: float) -> int:
    return lib().zro_encode_unorm8(c)


def srgb_thresholds() -> np.ndarray:
    return np.array([lib().zro_srgb_threshold(k) for k in range(255)], dtype=np.float32)


def signed_area2(xy) -> int:
    arr = (C.c_float * 6)(*xy)
    return lib().zro_signed_area2(arr)


def format_bpp(fmt: int) -> int:
    return lib().zro_format_bpp(fmt)


def render(scene, tile_size: int = 32, shard=(0, 1), nthreads: int = 1, with_stats: bool = False,
           viewport=None, scissor=None, render_area=None):
    """Replays ``TriangleRenderer::render_to``'s node on the CPU: begin_rendering
    (CLEAR), set_viewport {0,0,W,H,0,1}, set_scissor full, bind VB/IB, one
    draw_indexed(count,1,0,0,0), end_rendering.  Returns (color, depth[, stats]).
    Rows not owned by ``shard`` are left zero (colour) / NaN (depth)."""
    L = lib()
    W, H = scene.width, scene.height
    bpp = L.zro_format_bpp(scene.color_format)
    color = np.zeros((H, W * bpp), dtype=np.uint8)
    depth = np.full((H, W), np.nan, dtype=np.float32) if scene.depth else None
    tgt = _Target(W, H, scene.color_format, color.ctypes.data,
                  depth.ctypes.data if depth is not None else None)
    ra = render_area or (0, 0, W, H)
    ra_c = (C.c_int32 * 4)(*ra)
    cc = (C.c_float * 4)(*scene.clear_color)
    L.zro_clear(C.byref(tgt), C.byref(ra_c), C.byref(cc), 1, C.c_float(scene.depth_clear),
                1 if scene.depth else 0, tile_size, shard[0], shard[1])
    vb = np.ascontiguousarray(scene.vertices, dtype=np.float32)
    ib = None if scene.indices is None else np.ascontiguousarray(scene.indices)
    layout = scene.layout
    nat = len(layout)
    offs = (C.c_uint32 * 4)(*[4 * sum(layout[:a]) for a in range(nat)], *([0] * (4 - nat)))
    sizes = (C.c_uint32 * 4)(*[4 * n for n in layout], *([0] * (4 - nat)))
    vi = _VertexInput(vb.ctypes.data, vb.nbytes, vb.shape[1] * 4, nat, offs, sizes,
                      ib.ctypes.data if ib is not None else None, ib.nbytes if ib is not None else 0,
                      scene.index_type)
    vp = viewport or (0.0, 0.0, float(W), float(H), 0.0, 1.0)
    sc = scissor or (0, 0, W, H)
    st = _DrawState(scene.program, scene.time, (C.c_float * 6)(*vp), (C.c_int32 * 4)(*sc), ra_c,
                    scene.cull_mode, scene.front_face, 1 if scene.depth_test else 0,
                    1 if scene.depth_write else 0, scene.depth_op, scene.write_mask, tile_size,
                    shard[0], shard[1], (C.c_float * 16)(*(scene.view_proj or (0.0,) * 16)))
    cmd = _DrawCmd(scene.draw_count, scene.instance_count, scene.first, scene.vertex_offset, 0,
                   1 if ib is not None else 0)
    stats = Stats()
    rc = L.zro_draw(C.byref(tgt), C.byref(st), C.byref(vi), C.byref(cmd), nthreads, C.byref(stats))
    if rc != 0:
        raise RuntimeError(f"zro_draw failed: {rc}")
    out = (color.reshape(H, W, bpp), depth)
    return out + (stats,) if with_stats else out
