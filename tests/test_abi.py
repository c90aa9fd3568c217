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
    return [(o.peer, o.send, o.offset, o.bytes) for o in ops[:n]]


@pytest.mark.parametrize("height", [1080, 2160, 120, 40, 33, 1])
@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("root", [0, 1])
def test_gather_plan_covers_every_row_once(height, world, root):
    """zr_device_gather_tile_rows' plan (zr_gather_plan) against shard.owned_rows:
    the root receives every row it does not own exactly once, from that row's
    owner, into the row's own place; each peer sends exactly its own rows to the
    root; the root's rows never move; a partial last tile row moves only its rows."""
    from zenith_amd import shard
    root = root % world
    row_bytes = 7680
    lib = zr.lib()
    want = {r: set(shard.owned_rows(height, r, world).tolist()) for r in range(world)}
    recv = _plan(lib.zr_gather_plan, height, row_bytes, world, root, root)
    got_rows = {}
    for peer, send, off, nbytes in recv:
        assert send == 0 and peer != root
        assert off % row_bytes == 0 and nbytes % row_bytes == 0 and nbytes > 0
        for y in range(off // row_bytes, (off + nbytes) // row_bytes):
            assert y not in got_rows, f"row {y} received twice"
            got_rows[y] = peer
    assert set(got_rows) == set(range(height)) - want[root]
    assert all(y in want[p] for y, p in got_rows.items())
    sent = []
    for r in range(world):
        ops = _plan(lib.zr_gather_plan, height, row_bytes, world, r, root)
        if r == root:
            continue
        assert all(send == 1 and peer == root for peer, send, _, _ in ops)
        rows = {y for _, _, off, nb in ops for y in range(off // row_bytes, (off + nb) // row_bytes)}
        assert rows == want[r]
        sent += [(r, off, nb) for _, _, off, nb in ops]
    assert sorted(sent) == sorted((p, off, nb) for p, _, off, nb in recv)  # every send has its receive


@pytest.mark.parametrize("world", [1, 2, 3, 8, 32])
def test_exchange_plan_pairs_every_peer(world):
    """The built-in exchange's grouped send/recv (zr_exchange_plan): block p of the
    send buffer goes to rank p, and rank p's block lands at p * bytes_per_rank; per
    rank one send and one receive with every peer (itself included)."""
    lib = zr.lib()
    bpr = 16 + 48 * 1000
    for r in range(world):
        ops = _plan(lib.zr_exchange_plan, world, r, bpr)
        assert sorted((p, s) for p, s, _, _ in ops) == sorted((p, s) for p in range(world) for s in (0, 1))
        assert all(off == p * bpr and nb == bpr for p, _, off, nb in ops)
    assert lib.zr_exchange_plan(33, 0, bpr, None, 0) == -1
    assert lib.zr_gather_plan(1080, 7680, 2, 2, 0, None, 0) == -1
