/*
 * zenith_raster.h — C ABI of the MI355X-native draw path ("libzenith_raster").
 *
 * Replaces zenith's GPU draw path: the content/shaders vertex and
 * fragment stages plus the Vulkan fixed-function rasterizer behind zenith-rhi's
 * draw-submit API.  Each entry point below names the reference interface it
 * stands in for (paths relative to the reference repo root).  A zenith-rhi
 * backend binds these through Rust FFI; tests and the bench bind
 * them through ctypes.
 *
 * Conventions:
 *   - every enum argument carries the numeric Vulkan value (vk::Format::as_raw()
 *     etc.), so the Rust shim forwards ash values unchanged;
 *   - functions return zr_result, VkResult-compatible (0 = success, < 0 = error),
 *     and never unwind across the boundary;
 *   - zr_cmd_* recording calls return void like vkCmd*; recording errors are
 *     latched in the command buffer and returned by zr_cmd_end / zr_submit;
 *   - external synchronisation: a zr_device and its zr_cmds are used from one
 *     thread at a time (the reference's RenderDevice is !Sync: device.rs:85);
 *   - caller-owned host memory is only read during the call (copy semantics,
 *     buffer.rs:316).
 */
#ifndef ZENITH_RASTER_H
#define ZENITH_RASTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define ZR_API __attribute__((visibility("default")))
#else
#define ZR_API
#endif

typedef int32_t zr_result;

/* VkResult subset + the reference's typed errors, mapped to stable codes. */
enum {
    ZR_SUCCESS = 0,
    ZR_NOT_READY = 1,
    ZR_TIMEOUT = 2,
    ZR_ERROR_OUT_OF_HOST_MEMORY = -1,
    ZR_ERROR_OUT_OF_DEVICE_MEMORY = -2, /* also BufferRange::write overflow, buffer.rs:304-306 */
    ZR_ERROR_INITIALIZATION_FAILED = -3,
    ZR_ERROR_DEVICE_LOST = -4,
    ZR_ERROR_FEATURE_NOT_PRESENT = -8,
    ZR_ERROR_FORMAT_NOT_SUPPORTED = -11,
    ZR_ERROR_UNKNOWN = -13,
    ZR_ERROR_VALIDATION_FAILED = -1000011001, /* VK_ERROR_VALIDATION_FAILED_EXT */
    /* GraphicShaderInputBuildError, zenith-rhi/src/pipeline.rs:134-143 */
    ZR_ERROR_MISSING_VERTEX_SHADER = -1100001,
    ZR_ERROR_VERTEX_INPUT_REFLECTION_MISSING = -1100002,
    ZR_ERROR_DUPLICATE_VERTEX_ATTRIBUTE_LOCATION = -1100003,
    ZR_ERROR_MISSING_VERTEX_ATTRIBUTE = -1100004,
    ZR_ERROR_VERTEX_ATTRIBUTE_FORMAT_MISMATCH = -1100005,
    ZR_ERROR_UNEXPECTED_VERTEX_ATTRIBUTE = -1100006,
    /* ShaderBindingError, zenith-rhi/src/descriptor.rs:323-357 */
    ZR_ERROR_BINDING_NOT_FOUND = -1100010,
    ZR_ERROR_BINDING_TYPE_MISMATCH = -1100011,
    /* Shader::from_file failure (unknown file/entry), zenith-rhi/src/shader.rs:38-64 */
    ZR_ERROR_SHADER_NOT_FOUND = -1100020,
};

/* Vulkan numeric values used by this ABI (subset the path supports). */
enum {
    ZR_FORMAT_R8G8B8A8_UNORM = 37,
    ZR_FORMAT_R8G8B8A8_SRGB = 43,
    ZR_FORMAT_B8G8R8A8_UNORM = 44,
    ZR_FORMAT_B8G8R8A8_SRGB = 50,
    ZR_FORMAT_R32_SFLOAT = 100,
    ZR_FORMAT_R32G32_SFLOAT = 103,
    ZR_FORMAT_R32G32B32_SFLOAT = 106,
    ZR_FORMAT_R32G32B32A32_SFLOAT = 109,
    ZR_FORMAT_D32_SFLOAT = 126,
};
enum { ZR_SHADER_STAGE_VERTEX = 0x1, ZR_SHADER_STAGE_FRAGMENT = 0x10 };
enum { ZR_DESCRIPTOR_TYPE_UNIFORM_BUFFER = 6, ZR_DESCRIPTOR_TYPE_STORAGE_BUFFER = 7 };
enum { ZR_INDEX_TYPE_UINT16 = 0, ZR_INDEX_TYPE_UINT32 = 1 };
enum { ZR_ATTACHMENT_LOAD_OP_LOAD = 0, ZR_ATTACHMENT_LOAD_OP_CLEAR = 1, ZR_ATTACHMENT_LOAD_OP_DONT_CARE = 2 };
enum { ZR_ATTACHMENT_STORE_OP_STORE = 0, ZR_ATTACHMENT_STORE_OP_DONT_CARE = 1 };
enum { ZR_BUFFER_USAGE_TRANSFER_SRC = 0x1, ZR_BUFFER_USAGE_TRANSFER_DST = 0x2,
       ZR_BUFFER_USAGE_UNIFORM = 0x10, ZR_BUFFER_USAGE_STORAGE = 0x20,
       ZR_BUFFER_USAGE_INDEX = 0x40, ZR_BUFFER_USAGE_VERTEX = 0x80 };
enum { ZR_MEMORY_DEVICE_LOCAL = 0x1, ZR_MEMORY_HOST_VISIBLE = 0x2, ZR_MEMORY_HOST_COHERENT = 0x4 };

typedef struct zr_device_t zr_device;
typedef struct zr_buffer_t zr_buffer;
typedef struct zr_texture_t zr_texture;
typedef struct zr_shader_t zr_shader;
typedef struct zr_pipeline_t zr_pipeline;
typedef struct zr_cmd_t zr_cmd;
typedef struct zr_fence_t zr_fence;

/* ------------------------------------------------------------------ device */

/* RhiCore::create_render_device (core.rs:97-103) / RenderDevice::new
 * (device.rs:93-171): one HIP device, one in-order stream (the graphics queue). */
ZR_API zr_result zr_device_create(int32_t hip_device, zr_device **out);
ZR_API void zr_device_destroy(zr_device *dev);
/* RenderDevice::wait_idle analogue; also the point where the stats of the last
 * draw are read and a bin buffer that overflowed (those draws were rasterized
 * exactly by the slow all-records scan) is grown for later draws. */
ZR_API zr_result zr_device_wait_idle(zr_device *dev);
/* Runs the device's work on the caller's HIP stream (e.g. the one a collective
 * library orders its work on), NULL = the device's own stream again.  Waits for
 * the device first.  No reference counterpart (the reference has one queue). */
ZR_API zr_result zr_device_set_stream(zr_device *dev, void *hip_stream);
ZR_API void *zr_device_stream(const zr_device *dev);
/* Per-kernel HIP-event timing of every draw (off by default).  enable = 2 also
 * takes a winner census of every draw (zr_draw_stats.winners): the resolve marks
 * each primitive that wins a pixel in a bitmap -- extra atomics, so level 2 is
 * for a separate untimed frame, never for the timing passes. */
ZR_API zr_result zr_device_set_profiling(zr_device *dev, int32_t enable);
/* Accumulated timings since the last reset: for each kernel name (setup_bin,
 * tile, clear) total ms and launch count.  Returns the number of
 * entries written (<= capacity). */
typedef struct zr_kernel_time {
    char name[32];
    double total_ms;
    uint64_t launches;
} zr_kernel_time;
ZR_API int32_t zr_device_kernel_times(zr_device *dev, zr_kernel_time *out, int32_t capacity, int32_t reset);
/* Counters of the last completed draw (after a sync point). */
typedef struct zr_draw_stats {
    uint64_t triangles_in, triangles_setup, triangles_dropped_clip;
    uint64_t bin_pairs, bin_capacity, overflowed_draws;
    /* partitioned tile shards (zr_cmd_set_tile_shard_exchange): the largest block
     * total this rank RECEIVED (the entries one source rank routed to this rank,
     * counted before the block capacity cuts them) in the draws since the previous
     * sync point -- size zr_cmd_set_route_capacity from the maximum over ranks --
     * and the draws (so far) whose received blocks overflowed
     * zr_cmd_set_route_capacity and were set up in full instead */
    uint64_t route_max_entries, route_fallback_draws;
    /* distinct draw primitives that won at least one pixel in the last draw taken
     * with zr_device_set_profiling(dev, 2) (0 otherwise): the resolve's per-winner
     * gathers (vertex ids, attributes) are counted against it (bench.py) */
    uint64_t winners;
    /* micro primitives (a clipped bbox of one pixel) of the last draw that cover
     * their sample: setup tests each one and drops those that miss it before
     * they are binned */
    uint64_t micro_fragments;
    /* (tile, primitive) pairs of the last draw stored in pool runs past their
     * tiles' slabs, and those runs; bin_capacity counts slabs and
     * pool together */
    uint64_t bin_pool_pairs, bin_pool_runs;
    /* tile jobs of the last draw beyond one per tile: long tile lists split
     * over several workgroups */
    uint64_t tile_jobs;
    /* device memory held for tile-job key buffers (all scratch sets), sized per
     * draw shape from what its split needed and shrunk with the bin buffer */
    uint64_t job_key_bytes;
    /* the tile edge (pixels) of the last draw recorded: 16, 32 or 64, chosen per
     * draw; tile-row shards always 32 (zr_tile_size) */
    uint64_t tile_size;
} zr_draw_stats;
ZR_API zr_result zr_device_last_draw_stats(zr_device *dev, zr_draw_stats *out);
/* Last error message recorded on this thread (for logging; never NULL). */
ZR_API const char *zr_last_error_message(void);

/* ------------------------------------------------------------------ buffers */

typedef struct zr_buffer_desc {
    const char *name;      /* debug name (BufferDesc::name)                   */
    uint64_t size;
    uint32_t usage;        /* VkBufferUsageFlags bits                          */
    uint32_t memory_flags; /* VkMemoryPropertyFlags bits                       */
} zr_buffer_desc;

/* Buffer::new (buffer.rs:169-209); BufferDesc::{vertex,index,uniform,storage,staging}
 * (buffer.rs:47-94).  All buffers are HBM-resident; HOST_VISIBLE buffers are
 * written through zr_buffer_write (coherent: ordered before later submissions). */
ZR_API zr_result zr_buffer_create(zr_device *dev, const zr_buffer_desc *desc, zr_buffer **out);
/* Wraps caller-owned device memory (e.g. a torch tensor) without copying; the
 * caller keeps it alive until zr_buffer_destroy. */
ZR_API zr_result zr_buffer_create_external(zr_device *dev, const zr_buffer_desc *desc, void *device_ptr,
                                           zr_buffer **out);
ZR_API void zr_buffer_destroy(zr_buffer *buf);
/* BufferRange::write (buffer.rs:299-321) + UploadPool::enqueue_copy/flush
 * (upload.rs:46-176): ZR_ERROR_OUT_OF_DEVICE_MEMORY when offset+size > buffer size. */
ZR_API zr_result zr_buffer_write(zr_buffer *buf, uint64_t offset, const void *src, uint64_t size);
ZR_API zr_result zr_buffer_read(zr_buffer *buf, uint64_t offset, void *dst, uint64_t size);
ZR_API uint64_t zr_buffer_size(const zr_buffer *buf);
ZR_API void *zr_buffer_device_address(const zr_buffer *buf);

/* ----------------------------------------------------------------- textures */

typedef struct zr_texture_desc {
    const char *name;
    uint32_t width, height;
    int32_t format; /* ZR_FORMAT_* (VkFormat)                                  */
    uint32_t usage; /* VkImageUsageFlags bits (informational)                  */
} zr_texture_desc;

/* Texture::new (texture.rs:307-353); TextureDesc::new_color / new_depth
 * (texture.rs:131-162).  Linear row-major storage, pitch = width * bytes/pixel. */
ZR_API zr_result zr_texture_create(zr_device *dev, const zr_texture_desc *desc, zr_texture **out);
ZR_API zr_result zr_texture_create_external(zr_device *dev, const zr_texture_desc *desc, void *device_ptr,
                                            zr_texture **out);
ZR_API void zr_texture_destroy(zr_texture *tex);
/* Headless readback / upload (replaces swapchain present). */
ZR_API zr_result zr_texture_read(zr_texture *tex, void *dst, uint64_t size);
ZR_API zr_result zr_texture_write(zr_texture *tex, const void *src, uint64_t size);
ZR_API void *zr_texture_device_address(const zr_texture *tex);

/* ------------------------------------------------------------------ shaders */

typedef struct zr_shader_binding {
    char name[32];
    uint32_t set, binding;
    int32_t descriptor_type; /* VkDescriptorType */
    uint32_t count;
    uint32_t stage_flags;
} zr_shader_binding;

typedef struct zr_vertex_input_attr {
    uint32_t location;
    int32_t format; /* VkFormat */
} zr_vertex_input_attr;

/* Shader::from_file (shader.rs:38-64): maps (file, entry, stage) onto a built-in
 * HIP stage variant and returns its reflection (ShaderReflection, shader.rs:211-270).
 * Known files (matched on basename): triangle.slang (reference),
 * flat_color.slang, blinn_phong.slang, mesh.slang (camera matrix in the View
 * uniform) and mesh_push.slang (the same program, matrix in push constants)
 * (this repo, content/shaders/). */
ZR_API zr_result zr_shader_lookup(zr_device *dev, const char *path, const char *entry, uint32_t stage,
                                  zr_shader **out);
ZR_API void zr_shader_destroy(zr_shader *sh);
ZR_API int32_t zr_shader_bindings(const zr_shader *sh, zr_shader_binding *out, int32_t capacity);
ZR_API int32_t zr_shader_vertex_inputs(const zr_shader *sh, zr_vertex_input_attr *out, int32_t capacity);
/* ShaderReflection::push_constant_size (shader.rs:214; reflected from the SPIR-V
 * push-constant block at shader.rs:408-413): bytes of the stage's push-constant
 * block, 0 when it has none.  mesh_push.slang's vsmain: 64 (View.view_proj). */
ZR_API uint32_t zr_shader_push_constant_size(const zr_shader *sh);

/* ---------------------------------------------------------------- pipelines */

typedef struct zr_vertex_binding { uint32_t binding, stride, input_rate; } zr_vertex_binding;
typedef struct zr_vertex_attribute { uint32_t location, binding; int32_t format; uint32_t offset; } zr_vertex_attribute;

/* ColorAttachmentDesc, pipeline.rs:336-412 */
typedef struct zr_color_attachment_desc {
    uint32_t blend_enable;
    int32_t src_color_blend, dst_color_blend, color_blend_op;
    int32_t src_alpha_blend, dst_alpha_blend, alpha_blend_op;
    uint32_t write_mask;
    int32_t load_op, store_op;
    float clear_value[4];
} zr_color_attachment_desc;

/* DepthStencilDesc, pipeline.rs:414-453 */
typedef struct zr_depth_stencil_desc {
    uint32_t depth_test_enable, depth_write_enable;
    int32_t depth_compare_op;
    uint32_t depth_bounds_test_enable;
    int32_t depth_load_op, depth_store_op;
    float depth_clear_value;
    uint32_t stencil_test_enable;
    int32_t stencil_load_op, stencil_store_op;
    uint32_t stencil_clear_value;
} zr_depth_stencil_desc;

/* RasterizationState, pipeline.rs:507-578 */
typedef struct zr_rasterization_state {
    int32_t polygon_mode;
    uint32_t cull_mode;
    int32_t front_face;
    uint32_t depth_clamp, depth_bias_enable;
    float depth_bias_constant, depth_bias_slope, line_width;
} zr_rasterization_state;

/* vk::PushConstantRange of a pipeline layout (pipeline.rs:112-128). */
typedef struct zr_push_constant_range {
    uint32_t stage_flags; /* VkShaderStageFlags; ALL_GRAPHICS = 0x1F */
    uint32_t offset, size;
} zr_push_constant_range;
enum { ZR_SHADER_STAGE_ALL_GRAPHICS = 0x1F, ZR_MAX_PUSH_CONSTANTS_SIZE = 128 };

/* GraphicPipelineDesc = GraphicShaderInput + GraphicPipelineState +
 * GraphicPipelineAttachments (pipeline.rs:18-132, 714-737, 877-920). */
typedef struct zr_graphic_pipeline_desc {
    const zr_shader *vertex_shader;   /* NULL -> ZR_ERROR_MISSING_VERTEX_SHADER */
    const zr_shader *fragment_shader; /* nullable                                */
    uint32_t vertex_binding_count;
    const zr_vertex_binding *vertex_bindings;
    uint32_t vertex_attribute_count;
    const zr_vertex_attribute *vertex_attributes;
    int32_t topology;                 /* InputAssemblyState, pipeline.rs:455-505 */
    uint32_t primitive_restart;
    zr_rasterization_state rasterization;
    uint32_t samples;                 /* MultisampleState, pipeline.rs:580-614   */
    const zr_depth_stencil_desc *depth_stencil; /* nullable (Option)             */
    uint32_t color_attachment_count;
    const zr_color_attachment_desc *color_attachments;
    const int32_t *color_formats;     /* color_attachment_count VkFormats         */
    int32_t depth_format;             /* 0 = none                                 */
    /* The layout's push-constant ranges.  0 ranges: derived as
     * GraphicShaderInput::create_pipeline_layout does (pipeline.rs:112-128) --
     * one {ALL_GRAPHICS, 0, merged push_constant_size} range when the merged
     * reflection's size (ShaderReflection::merge, shader.rs:224-228: the max over
     * the stages) is > 0, none otherwise.  Given ranges are validated as
     * vkCreatePipelineLayout + vkCreateGraphicsPipelines would: offset and size
     * multiples of 4, size > 0, offset + size <= ZR_MAX_PUSH_CONSTANTS_SIZE, a
     * stage in at most one range, and every stage's push-constant block covered by
     * a range holding that stage (else ZR_ERROR_VALIDATION_FAILED). */
    uint32_t push_constant_range_count;
    const zr_push_constant_range *push_constant_ranges;
} zr_graphic_pipeline_desc;

/* Details of a pipeline validation failure (validate_vertex_inputs,
 * pipeline.rs:228-287). */
typedef struct zr_pipeline_error {
    uint32_t location;
    int32_t expected_format, provided_format;
} zr_pipeline_error;

/* GraphicShaderInput::new (validate + merge reflection) and
 * PipelineCache::get_or_create / CommonPipeline::new_graphic (pipeline_cache.rs:63-72,
 * pipeline.rs:931-1052).  `err` (nullable) receives the failing location/formats. */
ZR_API zr_result zr_pipeline_create(zr_device *dev, const zr_graphic_pipeline_desc *desc, zr_pipeline **out,
                                    zr_pipeline_error *err);
ZR_API void zr_pipeline_destroy(zr_pipeline *p);
/* The pipeline layout's push-constant ranges (derived or given, see the desc);
 * returns their number, writes at most `capacity`. */
ZR_API int32_t zr_pipeline_push_constant_ranges(const zr_pipeline *p, zr_push_constant_range *out,
                                                int32_t capacity);

/* ------------------------------------------------------------ command buffers */

typedef struct zr_viewport { float x, y, width, height, min_depth, max_depth; } zr_viewport;
typedef struct zr_rect2d { int32_t x, y; uint32_t width, height; } zr_rect2d;

typedef struct zr_rendering_attachment {
    zr_texture *texture;
    int32_t load_op, store_op;
    float clear_value[4]; /* colour RGBA, or clear_value[0] = depth */
} zr_rendering_attachment;

/* vk::RenderingInfo as GraphicNodeExecutionContext::begin_rendering builds it
 * (zenith-rendergraph/src/graph.rs:539-601). */
typedef struct zr_rendering_info {
    zr_rect2d render_area;
    uint32_t color_attachment_count;
    const zr_rendering_attachment *color_attachments;
    const zr_rendering_attachment *depth_attachment; /* nullable */
} zr_rendering_info;

/* CommandPool::allocate + CommandEncoder::new/begin (command.rs:44-62, 99-113).
 * dev may be NULL: the list records and validates on the host but zr_submit
 * rejects it (a list is submitted only to the device it was created for). */
ZR_API zr_result zr_cmd_create(zr_device *dev, zr_cmd **out);
ZR_API void zr_cmd_destroy(zr_cmd *cmd);
ZR_API zr_result zr_cmd_begin(zr_cmd *cmd); /* resets previous contents */
ZR_API zr_result zr_cmd_end(zr_cmd *cmd);   /* returns the latched recording error */

/* graph.rs:539-601 / command.rs:188-194 */
ZR_API void zr_cmd_begin_rendering(zr_cmd *cmd, const zr_rendering_info *info);
ZR_API void zr_cmd_end_rendering(zr_cmd *cmd);
/* vkCmdClearColorImage over the whole colour texture (one level / layer), as
 * zenith-sandbox's SimpleApp clear node records it through CommandEncoder::custom
 * (zenith-sandbox/src/main.rs:35-45).  Outside a render pass; the clear value is
 * linear float RGBA (encoded like a render-pass clear, sRGB formats included). */
ZR_API void zr_cmd_clear_color_image(zr_cmd *cmd, zr_texture *tex, const float clear_value[4]);
/* GraphicNodeExecutionContext::bind_pipeline (graph.rs:527-531) */
ZR_API void zr_cmd_bind_pipeline(zr_cmd *cmd, const zr_pipeline *p);
/* DescriptorSetBinder::bind_buffer + bind_descriptor_sets (descriptor.rs:323-357,
 * graph.rs:618-632), by (set, binding) */
ZR_API void zr_cmd_bind_uniform_buffer(zr_cmd *cmd, uint32_t set, uint32_t binding, const zr_buffer *buf,
                                       uint64_t offset, uint64_t range);
/* Same, by reflected name ("Time"); returns ZR_ERROR_BINDING_NOT_FOUND /
 * ZR_ERROR_BINDING_TYPE_MISMATCH immediately like bind_buffer does. */
ZR_API zr_result zr_cmd_bind_uniform_by_name(zr_cmd *cmd, const zr_pipeline *p, const char *name,
                                             const zr_buffer *buf, uint64_t offset, uint64_t range);
/* CommandEncoder::push_constants (command.rs:180-185): `layout` is the pipeline
 * whose layout the reference passes (CommonPipeline::layout); `size` bytes of
 * `data` are copied at record time (vkCmdPushConstants semantics) into the
 * push-constant state at `offset`, and later draws read them from their kernel
 * arguments.  Latched ZR_ERROR_VALIDATION_FAILED (the vkCmdPushConstants valid
 * usage): offset or size not a multiple of 4, size 0, offset + size >
 * ZR_MAX_PUSH_CONSTANTS_SIZE, stage_flags 0, a byte of the update outside a range
 * of `layout` holding every stage in stage_flags, or stage_flags missing a stage
 * of a range the update overlaps.  A draw whose pipeline reads push constants
 * fails (VALIDATION_FAILED) if the bytes it reads were not pushed, or were pushed
 * with a layout whose ranges differ from its own. */
ZR_API void zr_cmd_push_constants(zr_cmd *cmd, const zr_pipeline *layout, uint32_t stage_flags, uint32_t offset,
                                  uint32_t size, const void *data);
/* command.rs:171-177 */
ZR_API void zr_cmd_set_viewport(zr_cmd *cmd, uint32_t first, uint32_t count, const zr_viewport *vps);
ZR_API void zr_cmd_set_scissor(zr_cmd *cmd, uint32_t first, uint32_t count, const zr_rect2d *rects);
/* command.rs:153-159 */
ZR_API void zr_cmd_bind_vertex_buffers(zr_cmd *cmd, uint32_t first_binding, uint32_t count,
                                       const zr_buffer *const *bufs, const uint64_t *offsets);
ZR_API void zr_cmd_bind_index_buffer(zr_cmd *cmd, const zr_buffer *buf, uint64_t offset, int32_t index_type);
/* command.rs:162-168 — THE hot-path entry (triangle.rs:173) */
ZR_API void zr_cmd_draw(zr_cmd *cmd, uint32_t vertex_count, uint32_t instance_count, uint32_t first_vertex,
                        uint32_t first_instance);
ZR_API void zr_cmd_draw_indexed(zr_cmd *cmd, uint32_t index_count, uint32_t instance_count, uint32_t first_index,
                                int32_t vertex_offset, uint32_t first_instance);
/* Multi-GPU extension (no reference counterpart): subsequent
 * render passes touch only the 32x32 screen tiles this rank owns.  Ownership
 * (DESIGN.md §7): of a target's tiles_y tile rows, the first F = floor(tiles_y /
 * count) * count go round robin (row ty to rank ty % count); the n tiles of the
 * remaining rows (row-major) are cut into count runs, rank r owning tiles
 * [ceil(r n / count), ceil((r + 1) n / count)), so every rank owns the floor or
 * ceiling of tiles / count. */
ZR_API void zr_cmd_set_tile_shard(zr_cmd *cmd, uint32_t rank, uint32_t count);
/* Partitioned tile-row shards: as zr_cmd_set_tile_shard, but each
 * draw's primitive setup is split across the ranks too.  Rank r sets up only its
 * 1/count of the primitives and ships each one's setup record to the ranks
 * owning the tile rows it touches; the blocks of records are exchanged by
 * `exchange`, an all-to-all the caller provides (RCCL, MPI, ...), called from
 * zr_submit once per draw on every rank:
 *   send: `count` blocks of bytes_per_rank, block d for rank d;
 *   recv: the block each rank s addressed to this rank, at s * bytes_per_rank.
 * It must be ordered after earlier work on hip_stream and before later work on
 * it (enqueue on that stream, or synchronise), and return ZR_SUCCESS or an error
 * that zr_submit then returns.  count <= 32. */
typedef zr_result (*zr_exchange_fn)(void *user, void *hip_stream, const void *send, void *recv,
                                    uint64_t bytes_per_rank);
ZR_API void zr_cmd_set_tile_shard_exchange(zr_cmd *cmd, uint32_t rank, uint32_t count, zr_exchange_fn exchange,
                                           void *user);
/* Records per exchange block of later partitioned draws (bytes_per_rank = 16 +
 * 48 * entries); 0 = the runtime's default (twice a uniform share + 4096 from 3
 * ranks on).  Every rank must record the same value.  A block that would need
 * more keeps `entries` and flags the overflow: its receiver then sets up every
 * primitive of that draw itself (exact, slower; zr_draw_stats reports it). */
ZR_API void zr_cmd_set_route_capacity(zr_cmd *cmd, uint32_t entries);

/* Multi-GPU over RCCL inside the runtime (no reference counterpart).
 * One process per GPU.  Rank 0 makes two ids (zr_rccl_get_unique_id), the caller
 * distributes them (any side channel), and every rank calls zr_device_init_rccl
 * (collective, blocking).  Then:
 *   zr_cmd_set_tile_shard_exchange(cmd, rank, nranks, zr_rccl_exchange_fn(), dev)
 *     partitions setup with the built-in all-to-all (grouped send/recv);
 *   zr_device_gather_tile_rows(dev, tex, root) sends this rank's tile rows of
 *     `tex` into the root's `tex` (the root receives all others) on a stream of
 *     its own after the work enqueued so far; the next render pass writing `tex`
 *     waits for it.  Collective: every rank calls it for its frame, in order.
 * RCCL is loaded at run time (the process's copy if one is loaded, else
 * librccl.so); ZR_ERROR_INITIALIZATION_FAILED when unavailable. */
#define ZR_RCCL_ID_BYTES 128
ZR_API int32_t zr_rccl_available(void); /* 1 if RCCL can be loaded in this process */
ZR_API zr_result zr_rccl_get_unique_id(void *out);
ZR_API zr_result zr_device_init_rccl(zr_device *dev, const void *exchange_id, const void *gather_id, int32_t nranks,
                                     int32_t rank);
ZR_API zr_exchange_fn zr_rccl_exchange_fn(void);
/* A zr_exchange_fn that delivers a recorded receive buffer instead of running a
 * collective: `user` points to a zr_replay_exchange whose `src` (device memory,
 * count x bytes_per_rank) is copied into the receive buffer on the runtime's
 * stream.  For emulating one rank of a partitioned shard on one GPU with the
 * blocks the other ranks really routed to it (bench.py --emulate-shard): the
 * copy stands in for the all-to-all's transfer, without a host callback. */
typedef struct zr_replay_exchange {
    const void *src;
    uint64_t bytes;
} zr_replay_exchange;
ZR_API zr_exchange_fn zr_replay_exchange_fn(void);
ZR_API zr_result zr_device_gather_tile_rows(zr_device *dev, zr_texture *tex, int32_t root);
/* The point-to-point transfers the two collectives enqueue on this rank (host
 * only, no device): zr_device_gather_tile_rows of a width x height image of
 * `bytes_per_pixel`, and the built-in exchange's grouped send/recv pairing.  Each
 * op moves `rows` spans of `bytes` (`pitch` apart; rows == 1: one contiguous
 * span) at byte `offset` of the image (gather: the same offset on both sides; a
 * rectangle travels packed through a staging buffer) or of the send / receive
 * buffer (exchange) to or from `peer`.  Returns the number of ops (at most
 * `capacity` written; out may be NULL), or -1 for bad ranks or extents.
 * Ownership (zr_cmd_set_tile_shard): the round-robin tile rows are whole-row
 * spans; a leftover row yields one op per owner of a run of its tiles. */
typedef struct zr_transfer_op {
    int32_t peer;
    int32_t send; /* 1 = send to peer, 0 = receive from peer */
    uint64_t offset, bytes;
    uint32_t rows, reserved;
    uint64_t pitch;
} zr_transfer_op;
ZR_API int32_t zr_gather_plan(uint32_t width, uint32_t height, uint32_t bytes_per_pixel, int32_t nranks, int32_t rank,
                              int32_t root, zr_transfer_op *out, int32_t capacity);
ZR_API int32_t zr_exchange_plan(int32_t nranks, int32_t rank, uint64_t bytes_per_rank, zr_transfer_op *out,
                                int32_t capacity);
/* The screen-tile edge of tile-row shards in pixels (32): the unit of shard
 * ownership above (zenith_amd/shard.py owned_mask).  Unsharded draws pick 16,
 * 32 or 64 per draw (zr_draw_stats.tile_size). */
ZR_API uint32_t zr_tile_size(void);

/* -------------------------------------------------------------- submission */

ZR_API zr_result zr_fence_create(zr_device *dev, zr_fence **out);
ZR_API void zr_fence_destroy(zr_fence *f);
/* RenderDevice::submit_commands (device.rs:297-338): enqueue on the device stream,
 * signal `fence` (nullable) when done.  Asynchronous. */
ZR_API zr_result zr_submit(zr_device *dev, zr_cmd *cmd, zr_fence *fence);
/* begin_frame fence wait (device.rs:185-193).  timeout_ns = UINT64_MAX waits. */
ZR_API zr_result zr_fence_wait(zr_fence *f, uint64_t timeout_ns);
/* ImmediateCommandEncoder::submit_and_wait (command.rs:274-299). */
ZR_API zr_result zr_submit_and_wait(zr_device *dev, zr_cmd *cmd);

/* Library/kernel identification for provenance in tests and bench output. */
ZR_API const char *zr_build_info(void);

#ifdef __cplusplus
}
#endif
#endif
