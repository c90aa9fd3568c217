"""Renderers on the HIP draw path.

``TriangleRenderer`` restates zenith-renderer/src/triangle.rs call for call
(the reference's only renderer).  ``SceneRenderer`` drives the same node
sequence for the benchmark scenes (a depth attachment,
a larger vertex/index buffer, a different built-in program).
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np

from . import rhi, zr
from .scenes import PROGRAM_FILES, Scene


class TriangleRenderer:
    """zenith-renderer/src/triangle.rs:18-180."""

    VERTEX_FIELDS = (("position", 3), ("color", 3))  # triangle.rs:11-16

    def __init__(self, device: rhi.RenderDevice):
        self.device = device
        # triangle.rs:28-33
        vertices = np.array([[0.0, 0.5, 0.0, 1.0, 0.0, 0.0],
                             [-0.5, -0.5, 0.0, 0.0, 1.0, 0.0],
                             [0.5, -0.5, 0.0, 0.0, 0.0, 1.0]], dtype=np.float32)
        indices = np.array([0, 1, 2], dtype=np.uint16)
        vertex_data, index_data = vertices.tobytes(), indices.tobytes()
        # triangle.rs:38-49
        self.vertex_buffer = rhi.Buffer(device, rhi.BufferDesc.vertex("triangle.vertex", len(vertex_data)))
        self.index_buffer = rhi.Buffer(device, rhi.BufferDesc.index("triangle.index", len(index_data)))
        pool = rhi.UploadPool(device, len(vertex_data) + len(index_data))
        pool.enqueue_copy(self.vertex_buffer.as_range(), vertex_data)
        pool.enqueue_copy(self.index_buffer.as_range(), index_data)
        pool.flush()
        # triangle.rs:52-66
        self.vertex_shader = rhi.Shader.from_file("shader.triangle.vs", device, "content/shaders/triangle.slang",
                                                  "vsmain", rhi.ShaderStage.Vertex)
        self.fragment_shader = rhi.Shader.from_file("shader.triangle.ps", device,
                                                    "content/shaders/triangle.slang", "psmain",
                                                    rhi.ShaderStage.Fragment)
        self.start_time = time.monotonic()
        self._time_buffer = rhi.Buffer(device, rhi.BufferDesc.uniform("triangle.time", 4))
        self._pipelines = {}
        self._encoder = rhi.CommandEncoder(device)

    def _pipeline(self, fmt: int) -> rhi.GraphicPipeline:
        # PipelineCache::get_or_create keyed on the pipeline desc (pipeline_cache.rs:63-72)
        if fmt not in self._pipelines:
            shader = (rhi.GraphicShaderInputBuilder().vertex_shader(self.vertex_shader)
                      .fragment_shader(self.fragment_shader).vertex_layout(self.VERTEX_FIELDS).build())
            color_info = rhi.ColorAttachmentDesc().clear_input()
            color_info.clear_value = (0.1, 0.1, 0.1, 1.0)                    # triangle.rs:110-113
            state = rhi.GraphicPipelineState(rasterization=rhi.RasterizationState(cull_mode=0))  # :115-117
            state.color_attachments = [color_info]                            # push_color (:120-122)
            self._pipelines[fmt] = rhi.GraphicPipeline(self.device, shader, state, [fmt], None)
        return self._pipelines[fmt]

    def render_to(self, output: rhi.Texture, width: int, height: int, elapsed: Optional[float] = None,
                  shard: Optional[tuple] = None) -> rhi.CommandEncoder:
        """Records the "triangle" graphic node (triangle.rs:78-180) and returns the
        encoder; the caller submits it (CompiledRenderGraph::present)."""
        pipeline = self._pipeline(output.format)
        if elapsed is None:
            elapsed = time.monotonic() - self.start_time                      # triangle.rs:125
        vb, ib, tb = self.vertex_buffer, self.index_buffer, self._time_buffer

        def job(ctx: rhi.GraphicNodeExecutionContext):                       # triangle.rs:127-178
            encoder = ctx.encoder()
            if shard is not None:
                encoder.set_tile_shard(*shard)
            elapsed_bytes = np.float32(elapsed).tobytes()
            time_buffer = ctx.get(tb).as_range(0, len(elapsed_bytes))
            time_buffer.write(elapsed_bytes)
            binder = ctx.create_binder()
            binder.bind_buffer("Time", time_buffer)
            ctx.bind_descriptor_sets(binder)
            ctx.begin_rendering((width, height))
            ctx.bind_pipeline()
            encoder.set_viewport(0, [rhi.Viewport(0.0, 0.0, float(width), float(height), 0.0, 1.0)])
            encoder.set_scissor(0, [rhi.Rect2D(0, 0, width, height)])
            encoder.bind_vertex_buffers(0, [ctx.get(vb)], [0])
            encoder.bind_index_buffer(ctx.get(ib), 0, zr.INDEX_TYPE_UINT16)
            encoder.draw_indexed(3, 1, 0, 0, 0)
            ctx.end_rendering()

        rhi.execute_graphic_node(self.device, self._encoder, pipeline, [output], None, job)
        return self._encoder


class SceneRenderer:
    """Uploads a :class:`Scene` once and records its node like triangle.rs does,
    plus the depth attachment the benchmark configs use."""

    def __init__(self, device: rhi.RenderDevice, scene: Scene):
        self.device = device
        self.scene = scene
        vdata = scene.vertex_bytes()
        self.vertex_buffer = rhi.Buffer(device, rhi.BufferDesc.vertex(f"{scene.name}.vertex", len(vdata)))
        self.vertex_buffer.as_range().write(vdata)
        self.index_buffer = None
        if scene.indices is not None:
            idata = scene.index_bytes()
            self.index_buffer = rhi.Buffer(device, rhi.BufferDesc.index(f"{scene.name}.index", len(idata)))
            self.index_buffer.as_range().write(idata)
        path = PROGRAM_FILES[scene.program]
        if scene.push_view:  # the camera matrix as push constants (command.rs:180-185)
            path = "content/shaders/mesh_push.slang"
        self.vs = rhi.Shader.from_file(f"{scene.name}.vs", device, path, "vsmain", rhi.ShaderStage.Vertex)
        self.fs = rhi.Shader.from_file(f"{scene.name}.ps", device, path, "psmain", rhi.ShaderStage.Fragment)
        fields = [("position", 3)] + [(f"a{i}", n) for i, n in enumerate(scene.layout[1:], 1)]
        shader = (rhi.GraphicShaderInputBuilder().vertex_shader(self.vs).fragment_shader(self.fs)
                  .vertex_layout(fields).build())
        color_info = rhi.ColorAttachmentDesc().clear_input()
        color_info.clear_value = tuple(scene.clear_color)
        color_info.write_mask = scene.write_mask
        state = rhi.GraphicPipelineState(
            rasterization=rhi.RasterizationState(cull_mode=scene.cull_mode, front_face=scene.front_face))
        state.color_attachments = [color_info]
        if scene.depth:
            state.depth_stencil = rhi.DepthStencilDesc(depth_test_enable=scene.depth_test,
                                                       depth_write_enable=scene.depth_write,
                                                       depth_compare_op=scene.depth_op,
                                                       depth_clear_value=scene.depth_clear)
        self.pipeline = rhi.GraphicPipeline(device, shader, state, [scene.color_format],
                                            zr.FORMAT_D32_SFLOAT if scene.depth else None)
        self.time_buffer = None
        if scene.program == 0:
            self.time_buffer = rhi.Buffer(device, rhi.BufferDesc.uniform(f"{scene.name}.time", 4))
        self.view_buffer = None
        if scene.view_proj is not None and not scene.push_view:  # mesh.slang's View { float4x4 view_proj }
            self.view_buffer = rhi.Buffer(device, rhi.BufferDesc.uniform(f"{scene.name}.view", 64))
        self.encoder = rhi.CommandEncoder(device)

    def record(self, color: rhi.Texture, depth: Optional[rhi.Texture], shard: Optional[tuple] = None,
               viewport=None, scissor=None, encoder: Optional[rhi.CommandEncoder] = None) -> rhi.CommandEncoder:
        """Records the scene's node into ``encoder`` (default: the renderer's own)."""
        encoder = encoder or self.encoder
        s = self.scene
        W, H = s.width, s.height

        def job(ctx):
            enc = ctx.encoder()
            if shard is not None:
                enc.set_tile_shard(*shard)
            if self.time_buffer is not None:
                rng = self.time_buffer.as_range(0, 4)
                rng.write(np.float32(s.time).tobytes())
                binder = ctx.create_binder()
                binder.bind_buffer("Time", rng)
                ctx.bind_descriptor_sets(binder)
            if self.view_buffer is not None:
                rng = self.view_buffer.as_range(0, 64)
                rng.write(np.asarray(s.view_proj, np.float32).tobytes())
                binder = ctx.create_binder()
                binder.bind_buffer("View", rng)
                ctx.bind_descriptor_sets(binder)
            ctx.begin_rendering((W, H))
            ctx.bind_pipeline()
            if s.push_view:  # mesh_push.slang: View.view_proj at push-constant offset 0
                enc.push_constants(ctx.pipeline.layout(), zr.SHADER_STAGE_ALL_GRAPHICS, 0,
                                   np.asarray(s.view_proj, np.float32))
            vp = viewport or (0.0, 0.0, float(W), float(H), 0.0, 1.0)
            sc = scissor or (0, 0, W, H)
            enc.set_viewport(0, [rhi.Viewport(*vp)])
            enc.set_scissor(0, [rhi.Rect2D(*sc)])
            enc.bind_vertex_buffers(0, [self.vertex_buffer], [0])
            if self.index_buffer is not None:
                enc.bind_index_buffer(self.index_buffer, 0, s.index_type)
                enc.draw_indexed(s.draw_count, s.instance_count, s.first, s.vertex_offset, 0)
            else:
                enc.draw(s.draw_count, s.instance_count, s.first, 0)
            ctx.end_rendering()

        rhi.execute_graphic_node(self.device, encoder, self.pipeline, [color], depth, job)
        return encoder


def render_scene(device: rhi.RenderDevice, scene: Scene, shard: Optional[tuple] = None, viewport=None,
                 scissor=None, frames: int = 1):
    """``frames`` frames of ``scene`` on the GPU, submitted back to back with no
    host wait in between; returns the last one's (colour, depth) host arrays."""
    color = rhi.Texture(device, rhi.TextureDesc.new_color("rt", scene.width, scene.height, scene.color_format))
    depth = rhi.Texture(device, rhi.TextureDesc.new_depth("ds", scene.width, scene.height)) if scene.depth else None
    r = SceneRenderer(device, scene)
    enc = r.record(color, depth, shard=shard, viewport=viewport, scissor=scissor)
    for _ in range(frames - 1):
        device.submit(enc)
    device.submit_and_wait(enc)
    out = (color.read(), depth.read() if depth is not None else None)
    enc.destroy()
    color.destroy()
    if depth is not None:
        depth.destroy()
    return out


class SimpleAppRenderer:
    """zenith-sandbox's SimpleApp (zenith-sandbox/src/main.rs:12-50): one lambda
    node that clears the swapchain image to (0.2, 0.3, 0.8, 1.0) with
    cmd_clear_color_image."""

    CLEAR = (0.2, 0.3, 0.8, 1.0)  # main.rs:40

    def __init__(self, device: rhi.RenderDevice):
        self.device = device
        self._encoder = rhi.CommandEncoder(device)

    def render_to(self, output: rhi.Texture) -> rhi.CommandEncoder:
        enc = self._encoder
        enc.begin()
        enc.clear_color_image(output, self.CLEAR)
        enc.end()
        return enc
