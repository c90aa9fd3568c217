"""CPU tests of the C ABI boundary (no compute calls: no GPU in this container).

Checks that libzenith_raster loads, exports every symbol include/zenith_raster.h
declares, and that the host-side validation that needs no device behaves like
the reference: Shader::from_file lookups + reflection (shader.rs:38-64,
triangle.slang:3-8,27-32), validate_vertex_inputs error kinds
(pipeline.rs:134-143, 228-287), unsupported-state errors.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

from zenith_amd import rhi, zr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zenith_raster.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"ZR_API\s+[^;(]*?\b(zr_\w+)\s*\(", src)))


def test_header_symbols_exported():
    L = zr.lib()
    syms = header_symbols()
    assert len(syms) >= 45
    for name in syms:
        assert hasattr(L, name), f"{name} missing from libzenith_raster.so"
    assert sorted(zr.exported_symbols()) == syms  # the ctypes table binds exactly the header


def test_nm_exports_match_header():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", zr.LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r" T (zr_\w+)", out)))
    assert exported == header_symbols()


def test_build_info():
    assert b"gfx950" in zr.lib().zr_build_info()


def test_device_create_without_gpu_fails_cleanly():
    h = C.c_void_p()
    rc = zr.lib().zr_device_create(0, C.byref(h))
    assert rc in (zr.SUCCESS, zr.ERROR_INITIALIZATION_FAILED)
    if rc == zr.SUCCESS:
        zr.lib().zr_device_destroy(h)


class _NoDevice:
    handle = None


def shader(path, entry, stage):
    return rhi.Shader.from_file("t", _NoDevice(), path, entry, stage)


def test_shader_lookup_and_reflection():
    vs = shader("content/shaders/triangle.slang", "vsmain", rhi.ShaderStage.Vertex)
    ps = shader("some/dir/triangle.slang", "psmain", rhi.ShaderStage.Fragment)
    assert vs.reflection()["vertex_inputs"] == [(0, zr.FORMAT_R32G32B32_SFLOAT), (1, zr.FORMAT_R32G32B32_SFLOAT)]
    b = ps.reflection()["bindings"]
    assert b == [dict(name="Time", set=0, binding=0, descriptor_type=zr.DESCRIPTOR_TYPE_UNIFORM_BUFFER,
                      stage_flags=zr.SHADER_STAGE_FRAGMENT)]
    bp = shader("content/shaders/blinn_phong.slang", "vsmain", rhi.ShaderStage.Vertex)
    assert len(bp.reflection()["vertex_inputs"]) == 3
    with pytest.raises(zr.ZrError) as e:
        shader("content/shaders/missing.slang", "vsmain", rhi.ShaderStage.Vertex)
    assert e.value.code == zr.ERROR_SHADER_NOT_FOUND
    with pytest.raises(zr.ZrError):
        shader("content/shaders/triangle.slang", "psmain", rhi.ShaderStage.Vertex)  # wrong stage


def _builder():
    vs = shader("content/shaders/triangle.slang", "vsmain", rhi.ShaderStage.Vertex)
    ps = shader("content/shaders/triangle.slang", "psmain", rhi.ShaderStage.Fragment)
    return rhi.GraphicShaderInputBuilder().vertex_shader(vs).fragment_shader(ps)


def test_vertex_layout_derive():
    b, attrs = rhi.vertex_layout((("position", 3), ("color", 3)))
    assert b == rhi.VertexBinding(0, 24, 0)
    assert attrs == [rhi.VertexAttribute(0, 0, zr.FORMAT_R32G32B32_SFLOAT, 0),
                     rhi.VertexAttribute(1, 0, zr.FORMAT_R32G32B32_SFLOAT, 12)]
    _builder().vertex_layout((("position", 3), ("color", 3))).build()  # triangle.rs:104-108 succeeds


@pytest.mark.parametrize("attrs,code,loc", [
    ([rhi.VertexAttribute(0, 0, zr.FORMAT_R32G32B32_SFLOAT, 0)], zr.ERROR_MISSING_VERTEX_ATTRIBUTE, 1),
    ([rhi.VertexAttribute(0, 0, zr.FORMAT_R32G32B32_SFLOAT, 0), rhi.VertexAttribute(1, 0, zr.FORMAT_R32G32_SFLOAT, 12)],
     zr.ERROR_VERTEX_ATTRIBUTE_FORMAT_MISMATCH, 1),
    ([rhi.VertexAttribute(0, 0, zr.FORMAT_R32G32B32_SFLOAT, 0), rhi.VertexAttribute(1, 0, zr.FORMAT_R32G32B32_SFLOAT, 12),
      rhi.VertexAttribute(2, 0, zr.FORMAT_R32G32B32_SFLOAT, 24)], zr.ERROR_UNEXPECTED_VERTEX_ATTRIBUTE, 2),
    ([rhi.VertexAttribute(0, 0, zr.FORMAT_R32G32B32_SFLOAT, 0), rhi.VertexAttribute(0, 0, zr.FORMAT_R32_SFLOAT, 0),
      rhi.VertexAttribute(1, 0, zr.FORMAT_R32G32B32_SFLOAT, 12)], zr.ERROR_DUPLICATE_VERTEX_ATTRIBUTE_LOCATION, 0),
])
def test_validate_vertex_inputs_errors(attrs, code, loc):
    b = _builder().push_vertex_binding(rhi.VertexBinding(0, 36, 0))
    for a in attrs:
        b.push_vertex_attribute(a)
    with pytest.raises(rhi.GraphicShaderInputBuildError) as e:
        b.build()
    assert e.value.code == code and e.value.location == loc


def test_duplicate_same_format_is_allowed():
    b = _builder().vertex_layout((("position", 3), ("color", 3)))
    b.push_vertex_attribute(rhi.VertexAttribute(1, 0, zr.FORMAT_R32G32B32_SFLOAT, 12))
    b.build()


def test_missing_vertex_shader():
    with pytest.raises(rhi.GraphicShaderInputBuildError) as e:
        rhi.GraphicShaderInputBuilder().build()
    assert e.value.code == zr.ERROR_MISSING_VERTEX_SHADER


def _pipeline(state, color_formats=(zr.FORMAT_B8G8R8A8_SRGB,), depth=None):
    shader_in = _builder().vertex_layout((("position", 3), ("color", 3))).build()
    return rhi.GraphicPipeline(None, shader_in, state, list(color_formats), depth)


def test_pipeline_state_support_matrix():
    ok = rhi.GraphicPipelineState(rasterization=rhi.RasterizationState(cull_mode=0))
    ok.color_attachments = [rhi.ColorAttachmentDesc()]
    _pipeline(ok).destroy()
    blend = rhi.GraphicPipelineState()
    blend.color_attachments = [rhi.ColorAttachmentDesc(blend_enable=True)]
    strip = rhi.GraphicPipelineState(topology=4)
    msaa = rhi.GraphicPipelineState(samples=4)
    lines = rhi.GraphicPipelineState(rasterization=rhi.RasterizationState(polygon_mode=1))
    ne = rhi.GraphicPipelineState(depth_stencil=rhi.DepthStencilDesc(True, True, 5))
    for st in (blend, strip, msaa, lines, ne):
        with pytest.raises(zr.ZrError) as e:
            _pipeline(st)
        assert e.value.code == zr.ERROR_FEATURE_NOT_PRESENT


def test_mixed_program_stages_rejected():
    vs = shader("content/shaders/triangle.slang", "vsmain", rhi.ShaderStage.Vertex)
    ps = shader("content/shaders/flat_color.slang", "psmain", rhi.ShaderStage.Fragment)
    with pytest.raises(zr.ZrError) as e:  # no HIP variant pairs these stages
        rhi.GraphicShaderInputBuilder().vertex_shader(vs).fragment_shader(ps) \
            .vertex_layout((("position", 3), ("color", 3))).build()
    assert e.value.code == zr.ERROR_FEATURE_NOT_PRESENT


def test_buffer_range_write_overflow_is_host_checked():
    class FakeBuf:
        handle = None
    rng = rhi.BufferRange(FakeBuf(), 0, 4)
    with pytest.raises(zr.ZrError) as e:
        rng.write(b"12345")
    assert e.value.code == zr.ERROR_OUT_OF_DEVICE_MEMORY
    rng.write(b"")  # empty write is a no-op (buffer.rs:301-303)


# ----------------------------------------------- collective plans (host only)
def _plan(fn, *args):
    n = fn(*args, None, 0)
    assert n >= 0
    ops = (zr.zr_transfer_op * max(n, 1))()
    assert fn(*args, ops, n) == n
    return [(o.peer, o.send, o.offset, o.bytes, o.rows, o.pitch) for o in ops[:n]]


@pytest.mark.parametrize("w,h", [(1920, 1080), (3840, 2160), (320, 120), (100, 40), (33, 33), (70, 1)])
@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("root", [0, 1])
def test_gather_plan_covers_every_pixel_once(w, h, world, root):
    """zr_device_gather_tile_rows' plan (zr_gather_plan) against shard.owned_mask:
    the root receives every pixel it does not own exactly once, from that pixel's
    owner, into its own place; each peer sends exactly its own pixels; the root's
    pixels never move; round-robin tile rows travel as whole-row spans, a
    leftover row's tile runs as rectangles (rows spans, pitch = the image row)."""
    from zenith_amd import shard
    root = root % world
    bpp = 4
    row_bytes = w * bpp
    lib = zr.lib()

    def ops_of(r):
        n = lib.zr_gather_plan(w, h, bpp, world, r, root, None, 0)
        assert n >= 0
        arr = (zr.zr_transfer_op * max(n, 1))()
        assert lib.zr_gather_plan(w, h, bpp, world, r, root, arr, n) == n
        return [(o.peer, o.send, o.offset, o.bytes, o.rows, o.pitch) for o in arr[:n]]

    def pixels(off, nbytes, rows, pitch):
        assert off % bpp == 0 and nbytes % bpp == 0 and nbytes > 0 and rows >= 1
        starts = off + np.arange(rows, dtype=np.int64) * pitch
        if rows > 1:  # each rectangle row stays inside one image row
            assert ((starts // row_bytes) == ((starts + nbytes - 1) // row_bytes)).all()
        return ((starts // bpp)[:, None] + np.arange(nbytes // bpp)[None, :]).reshape(-1)

    owner = np.full(h * w, -1)
    for r in range(world):
        owner[shard.owned_mask(w, h, r, world).reshape(-1)] = r
    got = np.zeros(h * w, dtype=np.int64)
    src = np.full(h * w, -1)
    recv = ops_of(root)
    for peer, send, off, nb, rows, pitch in recv:
        assert send == 0 and peer != root
        assert rows == 1 or pitch == row_bytes
        px = pixels(off, nb, rows, pitch)
        got[px] += 1
        src[px] = peer
    assert (got[owner != root] == 1).all() and (got[owner == root] == 0).all(), "a pixel missed or received twice"
    assert np.array_equal(src[owner != root], owner[owner != root])
    sent = []
    for r in range(world):
        if r == root:
            continue
        ops = ops_of(r)
        assert all(send == 1 and peer == root for peer, send, *_ in ops)
        px = np.sort(np.concatenate([pixels(off, nb, rows, pitch) for _, _, off, nb, rows, pitch in ops])) \
            if ops else np.zeros(0, np.int64)
        assert np.array_equal(px, np.flatnonzero(owner == r))
        sent += [(r, off, nb, rows, pitch) for _, _, off, nb, rows, pitch in ops]
    assert sorted(sent) == sorted((p, off, nb, rows, pitch) for p, _, off, nb, rows, pitch in recv)


@pytest.mark.parametrize("world", [1, 2, 3, 8, 32])
def test_exchange_plan_pairs_every_peer(world):
    """The built-in exchange's grouped send/recv (zr_exchange_plan): block p of the
    send buffer goes to rank p, and rank p's block lands at p * bytes_per_rank; per
    rank one send and one receive with every peer (itself included)."""
    lib = zr.lib()
    bpr = 16 + 48 * 1000
    for r in range(world):
        ops = _plan(lib.zr_exchange_plan, world, r, bpr)
        assert sorted((p, s) for p, s, *_ in ops) == sorted((p, s) for p in range(world) for s in (0, 1))
        assert all(off == p * bpr and nb == bpr for p, _, off, nb, *_ in ops)
    assert lib.zr_exchange_plan(33, 0, bpr, None, 0) == -1
    assert lib.zr_gather_plan(1920, 1080, 4, 2, 2, 0, None, 0) == -1
    assert lib.zr_gather_plan(0, 1080, 4, 2, 0, 0, None, 0) == -1


@pytest.mark.parametrize("nbytes,bpr", [(0, 64), (100, 64), (64 * 33, 64), (64, 0), (96, 64)])
def test_replay_exchange_refuses_foreign_layouts(nbytes, bpr):
    """zr_replay_exchange_fn copies the recorded blocks into the draw's receive
    buffer (shard count x bytes_per_rank): a recording that is not whole blocks of
    the draw's layout, or more than kMaxShards of them, is refused before any
    copy (exec_draw also checks the count against the draw's shard count)."""
    fn = zr.EXCHANGE_FN(zr.lib().zr_replay_exchange_fn())
    src = (C.c_uint8 * 16)()
    desc = zr.zr_replay_exchange(C.cast(src, C.c_void_p), nbytes)
    rc = fn(C.addressof(desc), None, None, None, bpr)
    assert rc == zr.ERROR_VALIDATION_FAILED
    assert b"whole exchange blocks" in zr.lib().zr_last_error_message()
    empty = zr.zr_replay_exchange(None, 64)
    assert fn(C.addressof(empty), None, None, None, 64) == zr.ERROR_VALIDATION_FAILED


# ------------------------------------------------- push constants (host only)
# CommandEncoder::push_constants (command.rs:180-185), ShaderReflection::
# push_constant_size (shader.rs:214, :224-228, :408-413) and the pipeline
# layout's push-constant range (pipeline.rs:78, :105, :112-128).
MESH_FIELDS = (("position", 3), ("normal", 3), ("uv", 2))  # zenith-asset Vertex (render.rs:12-16)


def _mesh_input(path="content/shaders/mesh_push.slang"):
    vs = shader(path, "vsmain", rhi.ShaderStage.Vertex)
    ps = shader(path, "psmain", rhi.ShaderStage.Fragment)
    return vs, ps, rhi.GraphicShaderInputBuilder().vertex_shader(vs).fragment_shader(ps) \
        .vertex_layout(MESH_FIELDS).build()


def _mesh_pipeline(path="content/shaders/mesh_push.slang", ranges=None):
    _, _, inp = _mesh_input(path)
    st = rhi.GraphicPipelineState()
    st.color_attachments = [rhi.ColorAttachmentDesc()]
    return rhi.GraphicPipeline(None, inp, st, [zr.FORMAT_B8G8R8A8_SRGB], zr.FORMAT_D32_SFLOAT, ranges)


def test_push_constant_reflection_and_layout():
    vs, ps, inp = _mesh_input()
    assert vs.reflection()["push_constant_size"] == 64 and vs.reflection()["bindings"] == []
    assert ps.reflection()["push_constant_size"] == 0
    assert inp.push_constant_size == 64  # merged: the max over the stages
    # the uniform form of the program reflects no push constants
    assert shader("content/shaders/mesh.slang", "vsmain", rhi.ShaderStage.Vertex).reflection()["push_constant_size"] == 0
    assert _mesh_input("content/shaders/mesh.slang")[2].push_constant_size == 0
    p = _mesh_pipeline()
    assert p.push_constant_ranges() == [(zr.SHADER_STAGE_ALL_GRAPHICS, 0, 64)]  # derived (pipeline.rs:112-120)
    p.destroy()
    q = _mesh_pipeline("content/shaders/mesh.slang")
    assert q.push_constant_ranges() == []  # size 0: no range
    q.destroy()
    r = _mesh_pipeline(ranges=[(zr.SHADER_STAGE_VERTEX, 0, 128)])  # a caller's range covering the block
    assert r.push_constant_ranges() == [(zr.SHADER_STAGE_VERTEX, 0, 128)]
    r.destroy()


@pytest.mark.parametrize("ranges", [
    [(zr.SHADER_STAGE_VERTEX, 0, 60)],                                   # block [0, 64) not covered
    [(zr.SHADER_STAGE_FRAGMENT, 0, 64)],                                 # no range holds the vertex stage
    [(zr.SHADER_STAGE_VERTEX, 2, 64)],                                   # offset not a multiple of 4
    [(zr.SHADER_STAGE_VERTEX, 0, 66)],                                   # size not a multiple of 4
    [(zr.SHADER_STAGE_VERTEX, 0, 132)],                                  # past maxPushConstantsSize
    [(zr.SHADER_STAGE_VERTEX, 0, 0)],                                    # empty
    [(0, 0, 64)],                                                        # no stage
    [(zr.SHADER_STAGE_VERTEX, 0, 32), (zr.SHADER_STAGE_VERTEX, 32, 32)],  # a stage in two ranges
])
def test_push_constant_range_validation(ranges):
    with pytest.raises(zr.ZrError) as e:
        _mesh_pipeline(ranges=ranges)
    assert e.value.code == zr.ERROR_VALIDATION_FAILED


def test_push_constant_ranges_split_by_stage():
    # two ranges, one per stage, covering the vertex block: valid layout
    p = _mesh_pipeline(ranges=[(zr.SHADER_STAGE_VERTEX, 0, 64), (zr.SHADER_STAGE_FRAGMENT, 64, 16)])
    assert len(p.push_constant_ranges()) == 2
    p.destroy()


class _DevicelessEncoder(rhi.CommandEncoder):
    """A command list without a device (zr_cmd_create(NULL)): records and
    validates on the host; zr_submit would reject it."""

    def __init__(self):
        h = C.c_void_p()
        zr.check(zr.lib().zr_cmd_create(None, C.byref(h)), "zr_cmd_create")
        self.handle, self.device, self._keep = h, None, []


VIEW = np.arange(16, dtype=np.float32)


@pytest.mark.parametrize("stages,offset,data,ok", [
    (zr.SHADER_STAGE_ALL_GRAPHICS, 0, VIEW, True),                   # the whole block, the range's stages
    (zr.SHADER_STAGE_ALL_GRAPHICS, 32, VIEW[:8], True),              # a sub-range at an offset
    (zr.SHADER_STAGE_VERTEX, 0, VIEW, False),                        # misses stages of the range (01796)
    (zr.SHADER_STAGE_ALL_GRAPHICS, 4, VIEW, False),                  # bytes past the range (01795)
    (zr.SHADER_STAGE_ALL_GRAPHICS, 2, VIEW[:4], False),              # offset not a multiple of 4
    (zr.SHADER_STAGE_ALL_GRAPHICS, 0, b"\0" * 6, False),             # size not a multiple of 4
    (zr.SHADER_STAGE_ALL_GRAPHICS, 0, b"", False),                   # empty
    (zr.SHADER_STAGE_ALL_GRAPHICS, 124, VIEW[:2], False),            # past maxPushConstantsSize
    (0, 0, VIEW, False),                                             # no stage flags
])
def test_push_constants_recording_validation(stages, offset, data, ok):
    p = _mesh_pipeline()
    enc = _DevicelessEncoder()
    try:
        enc.begin()
        enc.push_constants(p.layout(), stages, offset, data)
        if ok:
            enc.end()
        else:
            with pytest.raises(zr.ZrError) as e:
                enc.end()  # the recording error is latched (vkCmd* return void)
            assert e.value.code == zr.ERROR_VALIDATION_FAILED
    finally:
        enc.destroy()
        p.destroy()


def test_push_constants_without_layout_range():
    # mesh.slang has no push-constant block, so its layout has no range at all
    q = _mesh_pipeline("content/shaders/mesh.slang")
    enc = _DevicelessEncoder()
    try:
        enc.begin()
        enc.push_constants(q.layout(), zr.SHADER_STAGE_ALL_GRAPHICS, 0, VIEW)
        with pytest.raises(zr.ZrError) as e:
            enc.end()
        assert e.value.code == zr.ERROR_VALIDATION_FAILED
    finally:
        enc.destroy()
        q.destroy()


def test_deviceless_list_is_not_submittable():
    enc = _DevicelessEncoder()
    try:
        enc.begin()
        enc.end()
        # (the device pointer is never dereferenced: the list's own device is checked first)
        rc = zr.lib().zr_submit(C.c_void_p(0x10), enc.handle, None)
        assert rc == zr.ERROR_VALIDATION_FAILED
    finally:
        enc.destroy()


@pytest.mark.parametrize("fields,fmts", [
    ((("position", 3), ("id", 1, "u32")), [zr.FORMAT_R32G32B32_SFLOAT, zr.FORMAT_R32_UINT]),
    ((("p", 2), ("q", 4, "i32"), ("r", 3, "u32"), ("s", 1, "i32"), ("t", 1)),
     [zr.FORMAT_R32G32_SFLOAT, zr.FORMAT_R32G32B32A32_SINT, zr.FORMAT_R32G32B32_UINT, zr.FORMAT_R32_SINT,
      zr.FORMAT_R32_SFLOAT]),
])
def test_vertex_layout_integer_fields(fields, fmts):
    """The derive's u32 / i32 mapping (zenith-rhi-derive/src/lib.rs:175-231)."""
    b, attrs = rhi.vertex_layout(fields)
    assert [a.format for a in attrs] == fmts
    assert b.stride == 4 * sum(f[1] for f in fields)
    assert [a.offset for a in attrs] == list(np.cumsum([0] + [4 * f[1] for f in fields[:-1]]))


def test_vertex_layout_rejects_what_the_derive_rejects():
    for bad in ((("x", 5),), (("x", 2, "f64"),), (("x", 3, "u16"),)):
        with pytest.raises(TypeError):
            rhi.vertex_layout(bad)


def test_integer_field_mismatch_is_reported():
    """A Vertex whose colour is [u32; 3] against triangle.slang (float3 color):
    VertexAttributeFormatMismatch at location 1, as validate_vertex_inputs
    reports it (pipeline.rs:259-270)."""
    with pytest.raises(rhi.GraphicShaderInputBuildError) as e:
        _builder().vertex_layout((("position", 3), ("color", 3, "u32"))).build()
    assert e.value.code == zr.ERROR_VERTEX_ATTRIBUTE_FORMAT_MISMATCH
    assert (e.value.location, e.value.expected, e.value.provided) == (1, zr.FORMAT_R32G32B32_SFLOAT,
                                                                      zr.FORMAT_R32G32B32_UINT)
