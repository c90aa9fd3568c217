/*
 * zr_oracle.h — CPU restatement of zenith's draw path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X rasterizer in zenith_amd/.  It is a
 * plain-C, in-order, per-fragment restatement of what the reference's draw path
 * computes:
 *   - content/shaders/triangle.slang:19-38 (vsmain / psmain arithmetic),
 *   - zenith-renderer/src/triangle.rs:28-33,110-117,154-173 (scene, clear, cull NONE,
 *     viewport, scissor, draw_indexed),
 *   - zenith-rhi/src/pipeline.rs:336-412,414-453,455-505,507-578,580-614 (pipeline
 *     state defaults: blend off, depth LESS/clear 1, TRIANGLE_LIST, FILL/BACK/CCW, 1x),
 *   - zenith-rhi/src/swapchain.rs:69-78 (B8G8R8A8_SRGB target),
 * plus the Vulkan 1.3 fixed-function rules the reference delegates to the driver
 * (SURVEY.md §8a row a4, §8c).  Implementation-defined Vulkan choices are pinned
 * in DESIGN.md §3 ("raster contract") and restated in zr_oracle.c.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product path (zenith_amd/) never links or calls it.
 *
 * Parity pinning: the reference has no tests, fixtures or golden images
 *  and cannot be built here (no Rust/Vulkan/slangc),
 * so this oracle is pinned by analytic known-answer tests derived from the
 * reference's own constants (tests/test_oracle.py) — see DESIGN.md §5.
 */
#ifndef ZR_ORACLE_H
#define ZR_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Built-in shader programs (VS+FS pairs) the oracle knows. */
enum {
    ZRO_PROGRAM_TRIANGLE = 0,    /* content/shaders/triangle.slang vsmain/psmain      */
    ZRO_PROGRAM_FLAT_COLOR = 1,  /* content/shaders/flat_color.slang (this repo)      */
    ZRO_PROGRAM_BLINN_PHONG = 2, /* content/shaders/blinn_phong.slang (this repo)     */
    ZRO_PROGRAM_MESH = 3,        /* content/shaders/mesh.slang: View.view_proj camera,  */
                                 /* near/far clip, perspective-correct (this repo)      */
};

typedef struct zro_target {
    uint32_t width, height;   /* attachment extent; linear row-major, no padding      */
    int32_t color_format;     /* VkFormat numeric value                              */
    uint8_t *color;           /* width*height*bpp bytes, may be NULL                 */
    float *depth;             /* D32_SFLOAT, width*height floats, may be NULL        */
} zro_target;

typedef struct zro_vertex_input {
    const uint8_t *vertex_data;
    uint64_t vertex_bytes;
    uint32_t stride;
    uint32_t attr_count;       /* locations 0..attr_count-1, 32-bit float vectors    */
    uint32_t attr_offset[4];
    uint32_t attr_size[4];     /* bytes: 12 (R32G32B32_SFLOAT) or 8 (R32G32_SFLOAT)   */
    const uint8_t *index_data; /* NULL for non-indexed draws                         */
    uint64_t index_bytes;
    int32_t index_type;        /* VkIndexType: 0 = UINT16, 1 = UINT32                */
} zro_vertex_input;

typedef struct zro_draw_state {
    int32_t program;
    float time;                /* Time.time (triangle.slang:27-32)                    */
    float viewport[6];         /* x, y, width, height, minDepth, maxDepth            */
    int32_t scissor[4];        /* x, y, width, height                                */
    int32_t render_area[4];    /* x, y, width, height                                */
    uint32_t cull_mode;        /* VkCullModeFlags                                    */
    int32_t front_face;        /* VkFrontFace                                        */
    uint32_t depth_test, depth_write;
    int32_t depth_op;          /* VkCompareOp                                        */
    uint32_t color_write_mask; /* VkColorComponentFlags                              */
    uint32_t tile_size;        /* screen-tile edge (shards own whole tiles)           */
    uint32_t shard_rank, shard_count; /* only this rank's tiles are drawn (zr_oracle.c owned_cols) */
    float view_proj[16];       /* mesh program: View.view_proj, column-major (glam)   */
} zro_draw_state;

typedef struct zro_draw_cmd {
    uint32_t count;            /* vertex_count or index_count                        */
    uint32_t instance_count;
    uint32_t first;            /* first_vertex or first_index                        */
    int32_t vertex_offset;
    uint32_t first_instance;
    uint32_t indexed;
} zro_draw_cmd;

typedef struct zro_stats {
    uint64_t triangles_in, triangles_setup, fragments_covered, fragments_passed;
    uint64_t triangles_dropped_clip; /* w<=0 or beyond guard band   */
} zro_stats;

/* Clear the render area's owned rows (fused-attachment CLEAR semantics). */
void zro_clear(const zro_target *t, const int32_t render_area[4], const float clear_color[4],
               int clear_colour, float clear_depth, int clear_depth_enable, uint32_t tile_size,
               uint32_t shard_rank, uint32_t shard_count);

/* One draw, in Vulkan submission order.  nthreads > 1 uses OpenMP over tile-row
 * bands (identical results: each band still visits primitives in order). */
int zro_draw(const zro_target *t, const zro_draw_state *s, const zro_vertex_input *vi,
             const zro_draw_cmd *cmd, int nthreads, zro_stats *stats);

/* Unit-level entry points for known-answer tests. */
int32_t zro_snap(float coord);                   /* float pixel coord -> 24.8 fixed   */
float zro_sinf(float x);
uint32_t zro_encode_unorm8(float c);
uint32_t zro_encode_srgb8(float c);
float zro_srgb_threshold(uint32_t k);            /* T[k], k in [0,255)                */
int64_t zro_signed_area2(const float xy[6]);     /* from framebuffer coords (snapped) */
uint32_t zro_format_bpp(int32_t vk_format);

#ifdef __cplusplus
}
#endif
#endif
