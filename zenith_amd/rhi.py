"""Reference-shaped host API over the C ABI.

Mirrors the zenith-rhi / zenith-rendergraph surface that the draw path touches
 so that callers — and the parity tests — read like
``zenith-renderer/src/triangle.rs``:

  RenderDevice            zenith-rhi/src/device.rs:93-171
  BufferDesc / Buffer     zenith-rhi/src/buffer.rs:36-137, 169-209, 299-321
  TextureDesc / Texture   zenith-rhi/src/texture.rs:131-162, 307-353
  Shader.from_file        zenith-rhi/src/shader.rs:38-64
  GraphicShaderInputBuilder, ColorAttachmentDesc, DepthStencilDesc,
  RasterizationState, GraphicPipelineState
                          zenith-rhi/src/pipeline.rs:68-132, 336-578, 714-800
  CommandEncoder          zenith-rhi/src/command.rs:92-243
  GraphicNodeExecutionContext / DescriptorSetBinder
                          zenith-rendergraph/src/graph.rs:509-633,
                          zenith-rhi/src/descriptor.rs:323-357

Every call goes through libzenith_raster (zenith_amd/lib); there is no
alternative implementation behind it.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import enum
from typing import Callable, Optional, Sequence

import numpy as np

from . import zr
from .zr import ZrError, check, lib


class GraphicShaderInputBuildError(ZrError):
    """pipeline.rs:134-143 (raised by GraphicShaderInputBuilder.build)."""


class ShaderBindingError(ZrError):
    """descriptor.rs ShaderBindingError (BindingNotFound / TypeMismatch)."""


# -------------------------------------------------------------------- device
class RenderDevice:
    def __init__(self, hip_device: int = 0):
        h = C.c_void_p()
        check(lib().zr_device_create(hip_device, C.byref(h)), "zr_device_create")
        self.handle = h
        self._alive = True

    def wait_idle(self):
        check(lib().zr_device_wait_idle(self.handle), "zr_device_wait_idle")

    def set_profiling(self, enable, census: bool = False):
        """Per-kernel event timing; ``census`` also counts each draw's winning
        primitives (last_draw_stats()["winners"]; extra atomics: untimed frames only)."""
        level = (2 if census else 1) if enable else 0
        check(lib().zr_device_set_profiling(self.handle, level), "zr_device_set_profiling")

    def kernel_times(self, reset: bool = False) -> dict:
        arr = (zr.zr_kernel_time * 32)()
        n = lib().zr_device_kernel_times(self.handle, arr, 32, 1 if reset else 0)
        return {arr[i].name.decode(): (arr[i].total_ms, arr[i].launches) for i in range(n)}

    def last_draw_stats(self) -> dict:
        st = zr.zr_draw_stats()
        check(lib().zr_device_last_draw_stats(self.handle, C.byref(st)), "zr_device_last_draw_stats")
        return {f: getattr(st, f) for f, _ in st._fields_}

    def set_stream(self, hip_stream: Optional[int]):
        """Runs the device's work on the caller's HIP stream (e.g. torch's current
        stream, so torch.distributed collectives order against it); None = own."""
        check(lib().zr_device_set_stream(self.handle, C.c_void_p(hip_stream) if hip_stream else None),
              "zr_device_set_stream")

    @property
    def stream(self) -> int:
        return lib().zr_device_stream(self.handle) or 0

    def init_rccl(self, exchange_id: bytes, gather_id: bytes, nranks: int, rank: int):
        """Joins the runtime's RCCL communicators (collective over all ranks; the ids
        come from rank 0's :func:`zenith_amd.zr` ``zr_rccl_get_unique_id``)."""
        check(lib().zr_device_init_rccl(self.handle, exchange_id, gather_id, nranks, rank), "zr_device_init_rccl")

    def gather_tile_rows(self, texture: "Texture", root: int = 0):
        """Sends this rank's tile rows of ``texture`` into the root's (RCCL, on the
        runtime's gather stream; the next pass writing ``texture`` waits for it)."""
        check(lib().zr_device_gather_tile_rows(self.handle, texture.handle, root), "zr_device_gather_tile_rows")

    def submit(self, encoder: "CommandEncoder", fence: Optional["Fence"] = None):
        check(lib().zr_submit(self.handle, encoder.handle, fence.handle if fence else None), "zr_submit")

    def submit_and_wait(self, encoder: "CommandEncoder"):
        check(lib().zr_submit_and_wait(self.handle, encoder.handle), "zr_submit_and_wait")

    def close(self):
        if self._alive:
            lib().zr_device_destroy(self.handle)
            self._alive = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Fence:
    def __init__(self, device: RenderDevice):
        h = C.c_void_p()
        check(lib().zr_fence_create(device.handle, C.byref(h)), "zr_fence_create")
        self.handle = h

    def wait(self, timeout_ns: int = 2**64 - 1) -> int:
        return check(lib().zr_fence_wait(self.handle, timeout_ns), "zr_fence_wait")

    def destroy(self):
        lib().zr_fence_destroy(self.handle)


# ------------------------------------------------------------------- buffers
@dataclasses.dataclass
class BufferDesc:
    name: str
    size: int
    usage: int = 0
    memory_flags: int = zr.MEMORY_DEVICE_LOCAL

    @staticmethod
    def vertex(name, size):
        return BufferDesc(name, size, zr.BUFFER_USAGE_VERTEX | zr.BUFFER_USAGE_TRANSFER_DST)

    @staticmethod
    def index(name, size):
        return BufferDesc(name, size, zr.BUFFER_USAGE_INDEX | zr.BUFFER_USAGE_TRANSFER_DST)

    @staticmethod
    def uniform(name, size):
        return BufferDesc(name, size, zr.BUFFER_USAGE_UNIFORM, zr.MEMORY_HOST_VISIBLE | zr.MEMORY_HOST_COHERENT)

    @staticmethod
    def storage(name, size):
        return BufferDesc(name, size, zr.BUFFER_USAGE_STORAGE)

    @staticmethod
    def staging(name, size):
        return BufferDesc(name, size, zr.BUFFER_USAGE_TRANSFER_SRC, zr.MEMORY_HOST_VISIBLE | zr.MEMORY_HOST_COHERENT)

    def _c(self):
        self._name_bytes = self.name.encode()
        return zr.zr_buffer_desc(self._name_bytes, self.size, self.usage, self.memory_flags)


class Buffer:
    def __init__(self, device: RenderDevice, desc: BufferDesc, external_ptr: Optional[int] = None):
        h = C.c_void_p()
        cd = desc._c()
        if external_ptr is None:
            check(lib().zr_buffer_create(device.handle, C.byref(cd), C.byref(h)), "zr_buffer_create")
        else:
            check(lib().zr_buffer_create_external(device.handle, C.byref(cd), C.c_void_p(external_ptr),
                                                  C.byref(h)), "zr_buffer_create_external")
        self.handle = h
        self.desc = desc

    @property
    def size(self) -> int:
        return lib().zr_buffer_size(self.handle)

    def as_range(self, start: int = 0, end: Optional[int] = None) -> "BufferRange":
        end = self.size if end is None else end
        if start > end or end > self.size:
            raise ZrError(zr.ERROR_VALIDATION_FAILED, "Buffer.as_range", "range out of bounds")
        return BufferRange(self, start, end - start)

    def read(self, size: Optional[int] = None, offset: int = 0) -> bytes:
        n = self.size - offset if size is None else size
        out = (C.c_uint8 * n)()
        check(lib().zr_buffer_read(self.handle, offset, out, n), "zr_buffer_read")
        return bytes(out)

    def destroy(self):
        lib().zr_buffer_destroy(self.handle)


@dataclasses.dataclass
class BufferRange:
    buffer: Buffer
    offset: int
    size: int

    def write(self, data) -> None:
        """BufferRange::write (buffer.rs:299-321): OUT_OF_DEVICE_MEMORY if too long."""
        mv = memoryview(bytes(data) if not isinstance(data, (bytes, bytearray)) else data)
        n = len(mv)
        if n == 0:
            return
        if n > self.size:
            raise ZrError(zr.ERROR_OUT_OF_DEVICE_MEMORY, "BufferRange::write", "data longer than the range")
        src = (C.c_uint8 * n).from_buffer_copy(mv)
        check(lib().zr_buffer_write(self.buffer.handle, self.offset, src, n), "zr_buffer_write")


class UploadPool:
    """UploadPool (upload.rs:22-193): staged copies flushed together (here each
    enqueue is a synchronous H2D copy; flush is a no-op kept for parity)."""

    def __init__(self, device: RenderDevice, capacity: int):
        self.device = device
        self.capacity = capacity

    def enqueue_copy(self, dst: BufferRange, data) -> None:
        dst.write(data)

    def flush(self) -> None:
        pass


# ------------------------------------------------------------------ textures
@dataclasses.dataclass
class TextureDesc:
    name: str
    width: int
    height: int
    format: int
    usage: int = 0

    @staticmethod
    def new_color(name, width, height, fmt):
        return TextureDesc(name, width, height, fmt, 0x10 | 0x4)   # COLOR_ATTACHMENT | SAMPLED

    @staticmethod
    def new_depth(name, width, height):
        return TextureDesc(name, width, height, zr.FORMAT_D32_SFLOAT, 0x20)  # DEPTH_STENCIL_ATTACHMENT


_BPP = {zr.FORMAT_R8G8B8A8_UNORM: 4, zr.FORMAT_R8G8B8A8_SRGB: 4, zr.FORMAT_B8G8R8A8_UNORM: 4,
        zr.FORMAT_B8G8R8A8_SRGB: 4, zr.FORMAT_R32G32B32A32_SFLOAT: 16, zr.FORMAT_D32_SFLOAT: 4}


class Texture:
    def __init__(self, device: RenderDevice, desc: TextureDesc, external_ptr: Optional[int] = None):
        h = C.c_void_p()
        self._name = desc.name.encode()
        cd = zr.zr_texture_desc(self._name, desc.width, desc.height, desc.format, desc.usage)
        if external_ptr is None:
            check(lib().zr_texture_create(device.handle, C.byref(cd), C.byref(h)), "zr_texture_create")
        else:
            check(lib().zr_texture_create_external(device.handle, C.byref(cd), C.c_void_p(external_ptr),
                                                   C.byref(h)), "zr_texture_create_external")
        self.handle = h
        self.desc = desc

    @property
    def format(self) -> int:
        return self.desc.format

    @property
    def nbytes(self) -> int:
        return self.desc.width * self.desc.height * _BPP[self.desc.format]

    def read(self) -> np.ndarray:
        """Headless readback: (H, W, 4) uint8 for 8-bit formats, (H, W) f32 depth,
        (H, W, 4) f32 for R32G32B32A32_SFLOAT."""
        d = self.desc
        if d.format == zr.FORMAT_D32_SFLOAT:
            out = np.empty((d.height, d.width), dtype=np.float32)
        elif d.format == zr.FORMAT_R32G32B32A32_SFLOAT:
            out = np.empty((d.height, d.width, 4), dtype=np.float32)
        else:
            out = np.empty((d.height, d.width, 4), dtype=np.uint8)
        check(lib().zr_texture_read(self.handle, out.ctypes.data, out.nbytes), "zr_texture_read")
        return out

    def write(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        check(lib().zr_texture_write(self.handle, a.ctypes.data, a.nbytes), "zr_texture_write")

    def destroy(self):
        lib().zr_texture_destroy(self.handle)


# ------------------------------------------------------------------- shaders
class ShaderStage(enum.IntEnum):
    Vertex = zr.SHADER_STAGE_VERTEX
    Fragment = zr.SHADER_STAGE_FRAGMENT


class Shader:
    def __init__(self, handle, name, path, entry, stage):
        self.handle, self.name, self.path, self.entry, self.stage = handle, name, path, entry, stage

    @staticmethod
    def from_file(name: str, device: RenderDevice, path: str, entry: str, stage: ShaderStage) -> "Shader":
        h = C.c_void_p()
        check(lib().zr_shader_lookup(device.handle, path.encode(), entry.encode(), int(stage), C.byref(h)),
              "Shader::from_file")
        return Shader(h, name, path, entry, stage)

    def reflection(self) -> dict:
        b = (zr.zr_shader_binding * 16)()
        nb = lib().zr_shader_bindings(self.handle, b, 16)
        v = (zr.zr_vertex_input_attr * 16)()
        nv = lib().zr_shader_vertex_inputs(self.handle, v, 16)
        return {
            "bindings": [dict(name=b[i].name.decode(), set=b[i].set, binding=b[i].binding,
                              descriptor_type=b[i].descriptor_type, stage_flags=b[i].stage_flags)
                         for i in range(nb)],
            "vertex_inputs": [(v[i].location, v[i].format) for i in range(nv)],
            "push_constant_size": int(lib().zr_shader_push_constant_size(self.handle)),
        }


# ----------------------------------------------------------- pipeline state
@dataclasses.dataclass(frozen=True)
class VertexBinding:
    binding: int
    stride: int
    input_rate: int = 0


@dataclasses.dataclass(frozen=True)
class VertexAttribute:
    location: int
    binding: int
    format: int
    offset: int


# vk_format_for_type / vk_format_for_scalar_array (zenith-rhi-derive/src/lib.rs:175-231):
# scalars f32/u32/i32 (n = 1) and arrays [T; 2..4] of them
_VERTEX_FORMATS = {
    ("f32", 1): zr.FORMAT_R32_SFLOAT, ("u32", 1): zr.FORMAT_R32_UINT, ("i32", 1): zr.FORMAT_R32_SINT,
    ("f32", 2): zr.FORMAT_R32G32_SFLOAT, ("f32", 3): zr.FORMAT_R32G32B32_SFLOAT,
    ("f32", 4): zr.FORMAT_R32G32B32A32_SFLOAT,
    ("u32", 2): zr.FORMAT_R32G32_UINT, ("u32", 3): zr.FORMAT_R32G32B32_UINT, ("u32", 4): zr.FORMAT_R32G32B32A32_UINT,
    ("i32", 2): zr.FORMAT_R32G32_SINT, ("i32", 3): zr.FORMAT_R32G32B32_SINT, ("i32", 4): zr.FORMAT_R32G32B32A32_SINT,
}


def vertex_layout(fields: Sequence[tuple]) -> tuple:
    """#[derive(VertexLayout)] (zenith-rhi-derive/src/lib.rs:61-140) for a repr(C)
    struct of 4-byte scalar or [T; n] fields, T in f32/u32/i32 (lib.rs:175-231):
    each field is ``(name, n)`` (f32) or ``(name, n, "u32" | "i32" | "f32")``, n = 1
    for a scalar.  location = field index, offset = running sum, binding 0,
    stride = size_of, per-vertex rate.  Types the derive rejects (other scalars,
    arrays of 1 or more than 4) raise TypeError, as the derive fails to compile."""
    attrs, off = [], 0
    for i, f in enumerate(fields):
        n, kind = f[1], (f[2] if len(f) > 2 else "f32")
        key = (kind, n) if n != 1 else (kind, 1)
        if key not in _VERTEX_FORMATS:
            raise TypeError(f"unsupported vertex field type for `{f[0]}`: {kind} x {n} "
                            "(supported: f32/u32/i32 scalars and [T; 2..4])")
        attrs.append(VertexAttribute(i, 0, _VERTEX_FORMATS[key], off))
        off += 4 * n
    return VertexBinding(0, off, 0), attrs


@dataclasses.dataclass
class GraphicShaderInput:
    vertex_shader: Shader
    fragment_shader: Optional[Shader]
    vertex_bindings: list
    vertex_attributes: list
    push_constant_size: int = 0  # merged reflection's (pipeline.rs:78, :105)


class GraphicShaderInputBuilder:
    def __init__(self):
        self._vs = self._fs = None
        self._bindings, self._attrs = [], []

    def vertex_shader(self, s):
        self._vs = s
        return self

    def fragment_shader(self, s):
        self._fs = s
        return self

    def push_vertex_binding(self, b):
        self._bindings.append(b)
        return self

    def push_vertex_attribute(self, a):
        self._attrs.append(a)
        return self

    def vertex_layout(self, fields):
        b, a = vertex_layout(fields)
        self._bindings.append(b)
        self._attrs.extend(a)
        return self

    def build(self) -> GraphicShaderInput:
        """GraphicShaderInput::new (pipeline.rs:82-109): strict vertex-input
        validation, performed by the C ABI's pipeline validator."""
        inp = GraphicShaderInput(self._vs, self._fs, list(self._bindings), list(self._attrs))
        # ShaderReflection::merge (shader.rs:224-228): the largest stage block
        inp.push_constant_size = max([lib().zr_shader_push_constant_size(sh.handle)
                                      for sh in (self._vs, self._fs) if sh is not None] + [0])
        dev_free_desc = _pipeline_desc(inp, GraphicPipelineState(), [], None)
        h = C.c_void_p()
        err = zr.zr_pipeline_error()
        rc = lib().zr_pipeline_create(None, C.byref(dev_free_desc[0]), C.byref(h), C.byref(err))
        if rc < 0:
            e = GraphicShaderInputBuildError(rc, "GraphicShaderInputBuilder::build",
                                             lib().zr_last_error_message().decode())
            e.location, e.expected, e.provided = err.location, err.expected_format, err.provided_format
            raise e
        lib().zr_pipeline_destroy(h)
        return inp


@dataclasses.dataclass
class ColorAttachmentDesc:
    """pipeline.rs:336-412 with its Default."""
    blend_enable: bool = False
    write_mask: int = 0xF
    load_op: int = zr.LOAD_OP_CLEAR
    store_op: int = zr.STORE_OP_STORE
    clear_value: tuple = (0.0, 0.0, 0.0, 1.0)

    def clear_input(self):
        self.load_op = zr.LOAD_OP_CLEAR
        return self

    def discard_input(self):
        self.load_op = zr.LOAD_OP_DONT_CARE
        return self

    def discard_output(self):
        self.store_op = zr.STORE_OP_DONT_CARE
        return self


@dataclasses.dataclass
class DepthStencilDesc:
    """pipeline.rs:414-453 with its Default (test/write off, LESS, clear 1.0)."""
    depth_test_enable: bool = False
    depth_write_enable: bool = False
    depth_compare_op: int = 1
    depth_load_op: int = zr.LOAD_OP_CLEAR
    depth_store_op: int = zr.STORE_OP_STORE
    depth_clear_value: float = 1.0


@dataclasses.dataclass
class RasterizationState:
    """pipeline.rs:507-578 with its Default (FILL, cull BACK, front CCW)."""
    polygon_mode: int = 0
    cull_mode: int = 2
    front_face: int = 0


@dataclasses.dataclass
class GraphicPipelineState:
    """pipeline.rs:714-737: TRIANGLE_LIST, 1x, dynamic VIEWPORT+SCISSOR."""
    topology: int = 3
    rasterization: RasterizationState = dataclasses.field(default_factory=RasterizationState)
    samples: int = 1
    depth_stencil: Optional[DepthStencilDesc] = None
    color_attachments: list = dataclasses.field(default_factory=list)


def _pipeline_desc(inp: GraphicShaderInput, state: GraphicPipelineState, color_formats, depth_format,
                   push_constant_ranges=None):
    nb, na = len(inp.vertex_bindings), len(inp.vertex_attributes)
    vbs = (zr.zr_vertex_binding * max(nb, 1))(*[zr.zr_vertex_binding(b.binding, b.stride, b.input_rate)
                                                 for b in inp.vertex_bindings])
    vas = (zr.zr_vertex_attribute * max(na, 1))(*[zr.zr_vertex_attribute(a.location, a.binding, a.format, a.offset)
                                                   for a in inp.vertex_attributes])
    ncol = len(state.color_attachments)
    cols = (zr.zr_color_attachment_desc * max(ncol, 1))()
    for i, ca in enumerate(state.color_attachments):
        cols[i].blend_enable = 1 if ca.blend_enable else 0
        cols[i].write_mask = ca.write_mask
        cols[i].load_op = ca.load_op
        cols[i].store_op = ca.store_op
        cols[i].clear_value = (C.c_float * 4)(*ca.clear_value)
    fmts = (C.c_int32 * max(ncol, 1))(*(list(color_formats) + [0] * (max(ncol, 1) - len(color_formats))))
    ds_ptr = None
    keep = [vbs, vas, cols, fmts]
    if state.depth_stencil is not None:
        d = state.depth_stencil
        ds = zr.zr_depth_stencil_desc(1 if d.depth_test_enable else 0, 1 if d.depth_write_enable else 0,
                                      d.depth_compare_op, 0, d.depth_load_op, d.depth_store_op,
                                      d.depth_clear_value, 0, 2, 1, 0)
        keep.append(ds)
        ds_ptr = C.pointer(ds)
    r = state.rasterization
    desc = zr.zr_graphic_pipeline_desc(
        inp.vertex_shader.handle if inp.vertex_shader else None,
        inp.fragment_shader.handle if inp.fragment_shader else None,
        nb, vbs, na, vas, state.topology, 0,
        zr.zr_rasterization_state(r.polygon_mode, r.cull_mode, r.front_face, 0, 0, 0.0, 0.0, 1.0),
        state.samples, ds_ptr, ncol, cols, fmts, depth_format or 0)
    if push_constant_ranges:  # else derived from the reflection (pipeline.rs:112-128)
        pcr = (zr.zr_push_constant_range * len(push_constant_ranges))(
            *[zr.zr_push_constant_range(*r) for r in push_constant_ranges])
        keep.append(pcr)
        desc.push_constant_range_count = len(push_constant_ranges)
        desc.push_constant_ranges = pcr
    return desc, keep


class GraphicPipeline:
    """CommonPipeline::new_graphic (pipeline.rs:931-1052) over zr_pipeline_create."""

    def __init__(self, device: Optional[RenderDevice], shader: GraphicShaderInput, state: GraphicPipelineState,
                 color_formats: Sequence[int], depth_format: Optional[int],
                 push_constant_ranges: Optional[Sequence[tuple]] = None):
        """``push_constant_ranges``: (stage_flags, offset, size) tuples of the
        layout; None derives them from the shaders' reflection as
        GraphicShaderInput::create_pipeline_layout does (pipeline.rs:112-128)."""
        desc, self._keep = _pipeline_desc(shader, state, color_formats, depth_format, push_constant_ranges)
        h = C.c_void_p()
        err = zr.zr_pipeline_error()
        check(lib().zr_pipeline_create(device.handle if device else None, C.byref(desc), C.byref(h),
                                       C.byref(err)), "zr_pipeline_create")
        self.handle = h
        self.shader = shader
        self.state = state

    def push_constant_ranges(self) -> list:
        """The layout's vk::PushConstantRange list as (stage_flags, offset, size)."""
        arr = (zr.zr_push_constant_range * 8)()
        n = lib().zr_pipeline_push_constant_ranges(self.handle, arr, 8)
        return [(arr[i].stage_flags, arr[i].offset, arr[i].size) for i in range(min(n, 8))]

    def layout(self) -> "GraphicPipeline":
        """CommonPipeline::layout: the pipeline stands in for its layout in
        push_constants / bind_descriptor_sets."""
        return self

    def destroy(self):
        lib().zr_pipeline_destroy(self.handle)


# ------------------------------------------------------------ command encoder
@dataclasses.dataclass
class Viewport:
    x: float
    y: float
    width: float
    height: float
    min_depth: float = 0.0
    max_depth: float = 1.0


@dataclasses.dataclass
class Rect2D:
    x: int
    y: int
    width: int
    height: int


class CommandEncoder:
    """command.rs:92-243 (recording only; submit through RenderDevice)."""

    def __init__(self, device: RenderDevice):
        h = C.c_void_p()
        check(lib().zr_cmd_create(device.handle, C.byref(h)), "zr_cmd_create")
        self.handle = h
        self.device = device
        self._keep = []

    def begin(self):
        check(lib().zr_cmd_begin(self.handle), "zr_cmd_begin")  # waits for its in-flight submissions
        self._keep = []

    def end(self):
        check(lib().zr_cmd_end(self.handle), "zr_cmd_end")

    def set_viewport(self, first: int, viewports: Sequence[Viewport]):
        arr = (zr.zr_viewport * len(viewports))(*[zr.zr_viewport(v.x, v.y, v.width, v.height, v.min_depth,
                                                                  v.max_depth) for v in viewports])
        lib().zr_cmd_set_viewport(self.handle, first, len(viewports), arr)

    def set_scissor(self, first: int, scissors: Sequence[Rect2D]):
        arr = (zr.zr_rect2d * len(scissors))(*[zr.zr_rect2d(s.x, s.y, s.width, s.height) for s in scissors])
        lib().zr_cmd_set_scissor(self.handle, first, len(scissors), arr)

    def bind_vertex_buffers(self, first_binding: int, buffers: Sequence[Buffer], offsets: Sequence[int]):
        n = len(buffers)
        hs = (C.c_void_p * n)(*[b.handle.value for b in buffers])
        offs = (C.c_uint64 * n)(*offsets)
        lib().zr_cmd_bind_vertex_buffers(self.handle, first_binding, n, hs, offs)

    def push_constants(self, layout: "GraphicPipeline", stages: int, offset: int, data) -> None:
        """CommandEncoder::push_constants (command.rs:180-185): the bytes of ``data``
        (bytes, a numpy array or any buffer) are copied now, at ``offset`` of the
        push-constant state; errors latch until end()/submit."""
        b = bytes(memoryview(data).cast("B")) if not isinstance(data, (bytes, bytearray)) else bytes(data)
        buf = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b or b"\0")
        lib().zr_cmd_push_constants(self.handle, layout.handle, stages, offset, len(b), buf)

    def bind_index_buffer(self, buffer: Buffer, offset: int, index_type: int):
        lib().zr_cmd_bind_index_buffer(self.handle, buffer.handle, offset, index_type)

    def draw(self, vertex_count, instance_count, first_vertex, first_instance):
        lib().zr_cmd_draw(self.handle, vertex_count, instance_count, first_vertex, first_instance)

    def draw_indexed(self, index_count, instance_count, first_index, vertex_offset, first_instance):
        lib().zr_cmd_draw_indexed(self.handle, index_count, instance_count, first_index, vertex_offset,
                                  first_instance)

    def clear_color_image(self, texture: "Texture", value=(0.0, 0.0, 0.0, 0.0)):
        """vkCmdClearColorImage as zenith-sandbox records it through
        CommandEncoder::custom (zenith-sandbox/src/main.rs:35-45)."""
        lib().zr_cmd_clear_color_image(self.handle, texture.handle, C.byref((C.c_float * 4)(*value)))

    def set_tile_shard(self, rank: int, count: int, exchange=None, route_capacity: int = 0):
        """Tile-row shard of the following render passes.  With ``exchange`` (a
        :class:`zenith_amd.shard.Exchange`) primitive setup is partitioned across
        the ranks too and its records routed through that all-to-all (DESIGN.md
        §7), ``route_capacity`` records per block (0: the runtime's default; the
        same on every rank)."""
        if exchange is not None:
            lib().zr_cmd_set_route_capacity(self.handle, route_capacity)
        if exchange is None:
            lib().zr_cmd_set_tile_shard(self.handle, rank, count)
        elif exchange == "rccl":  # the runtime's own all-to-all (RenderDevice.init_rccl)
            lib().zr_cmd_set_tile_shard_exchange(self.handle, rank, count, lib().zr_rccl_exchange_fn(),
                                                 self.device.handle)
        elif hasattr(exchange, "native"):  # a runtime-side zr_exchange_fn and its user data
            fn, user, keep = exchange.native()
            self._keep.append(keep)
            lib().zr_cmd_set_tile_shard_exchange(self.handle, rank, count, fn, user)
        else:
            cb = exchange.c_callback()
            self._keep.append(cb)  # the callback must outlive every submission of this list
            lib().zr_cmd_set_tile_shard_exchange(self.handle, rank, count, C.cast(cb, C.c_void_p), None)

    def destroy(self):
        lib().zr_cmd_destroy(self.handle)


class DescriptorSetBinder:
    """descriptor.rs:323-357: bind_buffer by reflected name."""

    def __init__(self, ctx: "GraphicNodeExecutionContext"):
        self.ctx = ctx
        self.pending = []

    def bind_buffer(self, name: str, rng: BufferRange):
        rc = lib().zr_cmd_bind_uniform_by_name(self.ctx.encoder().handle, self.ctx.pipeline.handle,
                                               name.encode(), rng.buffer.handle, rng.offset, rng.size)
        if rc < 0:
            raise ShaderBindingError(rc, "DescriptorSetBinder::bind_buffer", lib().zr_last_error_message().decode())
        self.pending.append(name)
        return self


class GraphicNodeExecutionContext:
    """graph.rs:509-633: what a graphic node's closure sees."""

    def __init__(self, device: RenderDevice, encoder: CommandEncoder, pipeline: GraphicPipeline,
                 color_targets: Sequence[Texture], depth_target: Optional[Texture]):
        self.device = device
        self._encoder = encoder
        self.pipeline = pipeline
        self.color_targets = list(color_targets)
        self.depth_target = depth_target

    def get(self, resource):
        return resource

    def encoder(self) -> CommandEncoder:
        return self._encoder

    def bind_pipeline(self):
        lib().zr_cmd_bind_pipeline(self._encoder.handle, self.pipeline.handle)

    def begin_rendering(self, extent: tuple):
        """graph.rs:539-601: attachment infos come from the pipeline's state."""
        infos = self.pipeline.state.color_attachments
        if len(self.color_targets) != len(infos):
            raise ZrError(zr.ERROR_VALIDATION_FAILED, "begin_rendering",
                          f"node has {len(self.color_targets)} color targets but pipeline state has "
                          f"{len(infos)} color attachments")
        n = len(self.color_targets)
        cols = (zr.zr_rendering_attachment * max(n, 1))()
        for i, (t, a) in enumerate(zip(self.color_targets, infos)):
            cols[i] = zr.zr_rendering_attachment(t.handle.value, a.load_op, a.store_op,
                                                 (C.c_float * 4)(*a.clear_value))
        depth_ptr = None
        ds = self.pipeline.state.depth_stencil
        if self.depth_target is not None and ds is not None:
            self._depth_att = zr.zr_rendering_attachment(self.depth_target.handle.value, ds.depth_load_op,
                                                         ds.depth_store_op,
                                                         (C.c_float * 4)(ds.depth_clear_value, 0, 0, 0))
            depth_ptr = C.pointer(self._depth_att)
        info = zr.zr_rendering_info(zr.zr_rect2d(0, 0, extent[0], extent[1]), n, cols, depth_ptr)
        lib().zr_cmd_begin_rendering(self._encoder.handle, C.byref(info))

    def end_rendering(self):
        lib().zr_cmd_end_rendering(self._encoder.handle)

    def create_binder(self) -> DescriptorSetBinder:
        return DescriptorSetBinder(self)

    def bind_descriptor_sets(self, binder: DescriptorSetBinder):
        return None  # bindings were recorded by bind_buffer


def execute_graphic_node(device: RenderDevice, encoder: CommandEncoder, pipeline: GraphicPipeline,
                         color_targets: Sequence[Texture], depth_target: Optional[Texture],
                         job: Callable[[GraphicNodeExecutionContext], None]):
    """Records one graphic node the way CompiledRenderGraph::present records it
    (graph.rs:276-348): begin the encoder, run the node closure, end."""
    encoder.begin()
    ctx = GraphicNodeExecutionContext(device, encoder, pipeline, color_targets, depth_target)
    job(ctx)
    encoder.end()
    return ctx
