"""ctypes binding of libzenith_raster (include/zenith_raster.h).

This is the raw C ABI, one Python function per exported symbol.  The
reference-shaped API (RenderDevice, CommandEncoder, TriangleRenderer, ...) lives
in :mod:`zenith_amd.rhi` / :mod:`zenith_amd.renderer` on top of it.

The library is loaded from the package tree (zenith_amd/lib/), never from a
system path, and there is no fallback: if it is missing, import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZR_LIB_PATH: an alternative build of the same library (A/B experiments)
LIB_PATH = os.environ.get("ZR_LIB_PATH") or os.path.join(_HERE, "lib", "libzenith_raster.so")

# ----------------------------------------------------------------- constants
SUCCESS, NOT_READY, TIMEOUT = 0, 1, 2
ERROR_OUT_OF_HOST_MEMORY = -1
ERROR_OUT_OF_DEVICE_MEMORY = -2
ERROR_INITIALIZATION_FAILED = -3
ERROR_DEVICE_LOST = -4
ERROR_FEATURE_NOT_PRESENT = -8
ERROR_FORMAT_NOT_SUPPORTED = -11
ERROR_UNKNOWN = -13
ERROR_VALIDATION_FAILED = -1000011001
ERROR_MISSING_VERTEX_SHADER = -1100001
ERROR_VERTEX_INPUT_REFLECTION_MISSING = -1100002
ERROR_DUPLICATE_VERTEX_ATTRIBUTE_LOCATION = -1100003
ERROR_MISSING_VERTEX_ATTRIBUTE = -1100004
ERROR_VERTEX_ATTRIBUTE_FORMAT_MISMATCH = -1100005
ERROR_UNEXPECTED_VERTEX_ATTRIBUTE = -1100006
ERROR_BINDING_NOT_FOUND = -1100010
ERROR_BINDING_TYPE_MISMATCH = -1100011
ERROR_SHADER_NOT_FOUND = -1100020

FORMAT_R8G8B8A8_UNORM = 37
FORMAT_R8G8B8A8_SRGB = 43
FORMAT_B8G8R8A8_UNORM = 44
FORMAT_B8G8R8A8_SRGB = 50
FORMAT_R32_SFLOAT = 100
FORMAT_R32G32_SFLOAT = 103
FORMAT_R32G32B32_SFLOAT = 106
FORMAT_R32G32B32A32_SFLOAT = 109
FORMAT_D32_SFLOAT = 126
# the derive's integer vertex formats (zenith-rhi-derive/src/lib.rs:175-231)
FORMAT_R32_UINT, FORMAT_R32_SINT = 98, 99
FORMAT_R32G32_UINT, FORMAT_R32G32_SINT = 101, 102
FORMAT_R32G32B32_UINT, FORMAT_R32G32B32_SINT = 104, 105
FORMAT_R32G32B32A32_UINT, FORMAT_R32G32B32A32_SINT = 107, 108
SHADER_STAGE_VERTEX, SHADER_STAGE_FRAGMENT = 0x1, 0x10
SHADER_STAGE_ALL_GRAPHICS = 0x1F
MAX_PUSH_CONSTANTS_SIZE = 128
DESCRIPTOR_TYPE_UNIFORM_BUFFER = 6
INDEX_TYPE_UINT16, INDEX_TYPE_UINT32 = 0, 1
LOAD_OP_LOAD, LOAD_OP_CLEAR, LOAD_OP_DONT_CARE = 0, 1, 2
STORE_OP_STORE, STORE_OP_DONT_CARE = 0, 1
BUFFER_USAGE_TRANSFER_SRC, BUFFER_USAGE_TRANSFER_DST = 0x1, 0x2
BUFFER_USAGE_UNIFORM, BUFFER_USAGE_STORAGE = 0x10, 0x20
BUFFER_USAGE_INDEX, BUFFER_USAGE_VERTEX = 0x40, 0x80
MEMORY_DEVICE_LOCAL, MEMORY_HOST_VISIBLE, MEMORY_HOST_COHERENT = 0x1, 0x2, 0x4

ERROR_NAMES = {v: k for k, v in dict(globals()).items() if k.startswith("ERROR_") and isinstance(v, int)}


class ZrError(RuntimeError):
    def __init__(self, code: int, what: str, message: str = ""):
        self.code = code
        super().__init__(f"{what} failed: {ERROR_NAMES.get(code, code)} ({code}) {message}".rstrip())


# ------------------------------------------------------------------- structs
class zr_kernel_time(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("total_ms", C.c_double), ("launches", C.c_uint64)]


class zr_transfer_op(C.Structure):
    _fields_ = [("peer", C.c_int32), ("send", C.c_int32), ("offset", C.c_uint64), ("bytes", C.c_uint64),
                ("rows", C.c_uint32), ("reserved", C.c_uint32), ("pitch", C.c_uint64)]


class zr_draw_stats(C.Structure):
    _fields_ = [("triangles_in", C.c_uint64), ("triangles_setup", C.c_uint64),
                ("triangles_dropped_clip", C.c_uint64), ("bin_pairs", C.c_uint64),
                ("bin_capacity", C.c_uint64), ("overflowed_draws", C.c_uint64),
                ("route_max_entries", C.c_uint64), ("route_fallback_draws", C.c_uint64), ("winners", C.c_uint64),
                ("micro_fragments", C.c_uint64), ("bin_pool_pairs", C.c_uint64), ("bin_pool_runs", C.c_uint64),
                ("tile_jobs", C.c_uint64), ("job_key_bytes", C.c_uint64),
                ("tile_size", C.c_uint64)]


class zr_buffer_desc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("size", C.c_uint64), ("usage", C.c_uint32), ("memory_flags", C.c_uint32)]


class zr_texture_desc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("width", C.c_uint32), ("height", C.c_uint32), ("format", C.c_int32),
                ("usage", C.c_uint32)]


class zr_shader_binding(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("set", C.c_uint32), ("binding", C.c_uint32),
                ("descriptor_type", C.c_int32), ("count", C.c_uint32), ("stage_flags", C.c_uint32)]


class zr_vertex_input_attr(C.Structure):
    _fields_ = [("location", C.c_uint32), ("format", C.c_int32)]


class zr_vertex_binding(C.Structure):
    _fields_ = [("binding", C.c_uint32), ("stride", C.c_uint32), ("input_rate", C.c_uint32)]


class zr_vertex_attribute(C.Structure):
    _fields_ = [("location", C.c_uint32), ("binding", C.c_uint32), ("format", C.c_int32), ("offset", C.c_uint32)]


class zr_color_attachment_desc(C.Structure):
    _fields_ = [("blend_enable", C.c_uint32), ("src_color_blend", C.c_int32), ("dst_color_blend", C.c_int32),
                ("color_blend_op", C.c_int32), ("src_alpha_blend", C.c_int32), ("dst_alpha_blend", C.c_int32),
                ("alpha_blend_op", C.c_int32), ("write_mask", C.c_uint32), ("load_op", C.c_int32),
                ("store_op", C.c_int32), ("clear_value", C.c_float * 4)]


class zr_depth_stencil_desc(C.Structure):
    _fields_ = [("depth_test_enable", C.c_uint32), ("depth_write_enable", C.c_uint32),
                ("depth_compare_op", C.c_int32), ("depth_bounds_test_enable", C.c_uint32),
                ("depth_load_op", C.c_int32), ("depth_store_op", C.c_int32), ("depth_clear_value", C.c_float),
                ("stencil_test_enable", C.c_uint32), ("stencil_load_op", C.c_int32),
                ("stencil_store_op", C.c_int32), ("stencil_clear_value", C.c_uint32)]


class zr_rasterization_state(C.Structure):
    _fields_ = [("polygon_mode", C.c_int32), ("cull_mode", C.c_uint32), ("front_face", C.c_int32),
                ("depth_clamp", C.c_uint32), ("depth_bias_enable", C.c_uint32),
                ("depth_bias_constant", C.c_float), ("depth_bias_slope", C.c_float), ("line_width", C.c_float)]


class zr_push_constant_range(C.Structure):
    _fields_ = [("stage_flags", C.c_uint32), ("offset", C.c_uint32), ("size", C.c_uint32)]


class zr_graphic_pipeline_desc(C.Structure):
    _fields_ = [("vertex_shader", C.c_void_p), ("fragment_shader", C.c_void_p),
                ("vertex_binding_count", C.c_uint32), ("vertex_bindings", C.POINTER(zr_vertex_binding)),
                ("vertex_attribute_count", C.c_uint32), ("vertex_attributes", C.POINTER(zr_vertex_attribute)),
                ("topology", C.c_int32), ("primitive_restart", C.c_uint32),
                ("rasterization", zr_rasterization_state), ("samples", C.c_uint32),
                ("depth_stencil", C.POINTER(zr_depth_stencil_desc)),
                ("color_attachment_count", C.c_uint32),
                ("color_attachments", C.POINTER(zr_color_attachment_desc)),
                ("color_formats", C.POINTER(C.c_int32)), ("depth_format", C.c_int32),
                ("push_constant_range_count", C.c_uint32),
                ("push_constant_ranges", C.POINTER(zr_push_constant_range))]


class zr_pipeline_error(C.Structure):
    _fields_ = [("location", C.c_uint32), ("expected_format", C.c_int32), ("provided_format", C.c_int32)]


class zr_viewport(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("width", C.c_float), ("height", C.c_float),
                ("min_depth", C.c_float), ("max_depth", C.c_float)]


class zr_rect2d(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("width", C.c_uint32), ("height", C.c_uint32)]


class zr_rendering_attachment(C.Structure):
    _fields_ = [("texture", C.c_void_p), ("load_op", C.c_int32), ("store_op", C.c_int32),
                ("clear_value", C.c_float * 4)]


class zr_rendering_info(C.Structure):
    _fields_ = [("render_area", zr_rect2d), ("color_attachment_count", C.c_uint32),
                ("color_attachments", C.POINTER(zr_rendering_attachment)),
                ("depth_attachment", C.POINTER(zr_rendering_attachment))]


class zr_replay_exchange(C.Structure):
    _fields_ = [("src", C.c_void_p), ("bytes", C.c_uint64)]


# zr_exchange_fn (include/zenith_raster.h): (user, hip_stream, send, recv, bytes_per_rank) -> zr_result
EXCHANGE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)
RCCL_ID_BYTES = 128


# ------------------------------------------------------------------- loading
_P = C.c_void_p
_R = C.c_int32
_SIGS = {
    "zr_last_error_message": (C.c_char_p, []),
    "zr_build_info": (C.c_char_p, []),
    "zr_device_create": (_R, [C.c_int32, C.POINTER(_P)]),
    "zr_device_destroy": (None, [_P]),
    "zr_device_wait_idle": (_R, [_P]),
    "zr_device_set_profiling": (_R, [_P, C.c_int32]),
    "zr_device_kernel_times": (C.c_int32, [_P, C.POINTER(zr_kernel_time), C.c_int32, C.c_int32]),
    "zr_device_last_draw_stats": (_R, [_P, C.POINTER(zr_draw_stats)]),
    "zr_buffer_create": (_R, [_P, C.POINTER(zr_buffer_desc), C.POINTER(_P)]),
    "zr_buffer_create_external": (_R, [_P, C.POINTER(zr_buffer_desc), _P, C.POINTER(_P)]),
    "zr_buffer_destroy": (None, [_P]),
    "zr_buffer_write": (_R, [_P, C.c_uint64, _P, C.c_uint64]),
    "zr_buffer_read": (_R, [_P, C.c_uint64, _P, C.c_uint64]),
    "zr_buffer_size": (C.c_uint64, [_P]),
    "zr_buffer_device_address": (_P, [_P]),
    "zr_texture_create": (_R, [_P, C.POINTER(zr_texture_desc), C.POINTER(_P)]),
    "zr_texture_create_external": (_R, [_P, C.POINTER(zr_texture_desc), _P, C.POINTER(_P)]),
    "zr_texture_destroy": (None, [_P]),
    "zr_texture_read": (_R, [_P, _P, C.c_uint64]),
    "zr_texture_write": (_R, [_P, _P, C.c_uint64]),
    "zr_texture_device_address": (_P, [_P]),
    "zr_shader_lookup": (_R, [_P, C.c_char_p, C.c_char_p, C.c_uint32, C.POINTER(_P)]),
    "zr_shader_destroy": (None, [_P]),
    "zr_shader_bindings": (C.c_int32, [_P, C.POINTER(zr_shader_binding), C.c_int32]),
    "zr_shader_vertex_inputs": (C.c_int32, [_P, C.POINTER(zr_vertex_input_attr), C.c_int32]),
    "zr_shader_push_constant_size": (C.c_uint32, [_P]),
    "zr_pipeline_create": (_R, [_P, C.POINTER(zr_graphic_pipeline_desc), C.POINTER(_P),
                                C.POINTER(zr_pipeline_error)]),
    "zr_pipeline_destroy": (None, [_P]),
    "zr_pipeline_push_constant_ranges": (C.c_int32, [_P, C.POINTER(zr_push_constant_range), C.c_int32]),
    "zr_cmd_create": (_R, [_P, C.POINTER(_P)]),
    "zr_cmd_destroy": (None, [_P]),
    "zr_cmd_begin": (_R, [_P]),
    "zr_cmd_end": (_R, [_P]),
    "zr_cmd_begin_rendering": (None, [_P, C.POINTER(zr_rendering_info)]),
    "zr_cmd_end_rendering": (None, [_P]),
    "zr_cmd_bind_pipeline": (None, [_P, _P]),
    "zr_cmd_bind_uniform_buffer": (None, [_P, C.c_uint32, C.c_uint32, _P, C.c_uint64, C.c_uint64]),
    "zr_cmd_bind_uniform_by_name": (_R, [_P, _P, C.c_char_p, _P, C.c_uint64, C.c_uint64]),
    "zr_cmd_push_constants": (None, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint32, _P]),
    "zr_cmd_set_viewport": (None, [_P, C.c_uint32, C.c_uint32, C.POINTER(zr_viewport)]),
    "zr_cmd_set_scissor": (None, [_P, C.c_uint32, C.c_uint32, C.POINTER(zr_rect2d)]),
    "zr_cmd_bind_vertex_buffers": (None, [_P, C.c_uint32, C.c_uint32, C.POINTER(_P), C.POINTER(C.c_uint64)]),
    "zr_cmd_bind_index_buffer": (None, [_P, _P, C.c_uint64, C.c_int32]),
    "zr_cmd_draw": (None, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "zr_cmd_draw_indexed": (None, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int32, C.c_uint32]),
    "zr_cmd_set_tile_shard": (None, [_P, C.c_uint32, C.c_uint32]),
    "zr_cmd_clear_color_image": (None, [_P, _P, C.POINTER(C.c_float * 4)]),
    "zr_cmd_set_tile_shard_exchange": (None, [_P, C.c_uint32, C.c_uint32, _P, _P]),
    "zr_cmd_set_route_capacity": (None, [_P, C.c_uint32]),
    "zr_gather_plan": (C.c_int32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int32, C.c_int32, C.c_int32,
                                   C.POINTER(zr_transfer_op), C.c_int32]),
    "zr_exchange_plan": (C.c_int32, [C.c_int32, C.c_int32, C.c_uint64, C.POINTER(zr_transfer_op), C.c_int32]),
    "zr_tile_size": (C.c_uint32, []),
    "zr_device_set_stream": (_R, [_P, _P]),
    "zr_device_stream": (_P, [_P]),
    "zr_rccl_available": (C.c_int32, []),
    "zr_rccl_get_unique_id": (_R, [_P]),
    "zr_device_init_rccl": (_R, [_P, _P, _P, C.c_int32, C.c_int32]),
    "zr_rccl_exchange_fn": (_P, []),
    "zr_replay_exchange_fn": (_P, []),
    "zr_device_gather_tile_rows": (_R, [_P, _P, C.c_int32]),
    "zr_fence_create": (_R, [_P, C.POINTER(_P)]),
    "zr_fence_destroy": (None, [_P]),
    "zr_submit": (_R, [_P, _P, _P]),
    "zr_fence_wait": (_R, [_P, C.c_uint64]),
    "zr_submit_and_wait": (_R, [_P, _P]),
}

_lib = None


def lib():
    """Loads libzenith_raster.so from the package tree (fails loudly if absent)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C zenith_amd)")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("ZR_LIB_PATH") and not hasattr(L, name):
                continue  # an older build under A/B (tools/ab.sh): bind what it has
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return sorted(_SIGS)


def tile_size() -> int:
    """The loaded library's screen-tile edge (zr_tile_size; 32 for a build that
    predates it, under A/B)."""
    L = lib()
    return int(L.zr_tile_size()) if hasattr(L, "zr_tile_size") else 32


def check(rc: int, what: str) -> int:
    if rc < 0:
        msg = lib().zr_last_error_message().decode(errors="replace")
        raise ZrError(rc, what, msg)
    return rc


def out_ptr():
    return C.c_void_p()
