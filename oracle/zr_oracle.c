/*
 * zr_oracle.c — CPU restatement of zenith's draw path.  TEST INFRASTRUCTURE ONLY:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Semantics: one Vulkan 1.3 draw processed strictly in submission order, one
 * fragment at a time (the textbook pipeline; no visibility buffer, no binning),
 * so that the GPU path's order-independent formulation is checked against the
 * plain sequential rule.  Every arithmetic step that feeds an output bit is
 * written out explicitly (explicit fmaf, compiled with -ffp-contract=off) and is
 * the contract in DESIGN.md §3.  Citations are to /root/reference unless noted.
 */
#include "zr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* VkFormat values (Vulkan registry) */
#define F_R8G8B8A8_UNORM 37
#define F_R8G8B8A8_SRGB 43
#define F_B8G8R8A8_UNORM 44
#define F_B8G8R8A8_SRGB 50
#define F_R32G32B32A32_SFLOAT 109

/* VkCompareOp */
enum { OP_NEVER, OP_LESS, OP_EQUAL, OP_LEQUAL, OP_GREATER, OP_NOTEQUAL, OP_GEQUAL, OP_ALWAYS };

/* ---------------------------------------------------------------- numerics */

/* Sub-pixel snap: subPixelPrecisionBits = 8, round-to-nearest-even
 * (Vulkan 1.3 §Rasterization: implementation-defined precision). */
int32_t zro_snap(float coord) { return (int32_t)rintf(coord * 256.0f); }

/* sin() of triangle.slang:36.  SPIR-V GLSL.std.450 Sin only promises 2^-11 abs
 * error, so the contract fixes one implementation: 3-part Cody-Waite reduction by
 * pi/2, then degree-11/12 Taylor polynomials. */
float zro_sinf(float x) {
    const float q = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(q, -0x1.921fb6p+0f, x);
    r = fmaf(q, 0x1.777a5cp-25f, r);
    r = fmaf(q, 0x1.0p-49f, r);
    const int qi = ((int)q) & 3;
    const float r2 = r * r;
    float s = fmaf(r2, -0x1.ae64568p-26f, 0x1.71de3a6p-19f);   /* -1/11!, 1/9!  */
    s = fmaf(r2, s, -0x1.a01a01ap-13f);                           /* -1/7!         */
    s = fmaf(r2, s, 0x1.111112p-7f);                              /*  1/5!         */
    s = fmaf(r2, s, -0x1.555556p-3f);                             /* -1/3!         */
    s = fmaf(r2 * r, s, r);
    float c = fmaf(r2, 0x1.1ee9ebp-29f, -0x1.27e4fbp-22f);        /* 1/12!, -1/10! */
    c = fmaf(r2, c, 0x1.a01a01ap-16f);                            /*  1/8!         */
    c = fmaf(r2, c, -0x1.6c16c16p-10f);                           /* -1/6!         */
    c = fmaf(r2, c, 0x1.555556p-5f);                              /*  1/4!         */
    c = fmaf(r2, c, -0.5f);
    c = fmaf(r2, c, 1.0f);
    switch (qi) {
    case 0: return s;
    case 1: return c;
    case 2: return -s;
    default: return -c;
    }
}

/* sRGB encode thresholds.  T[k] = the smallest float >= the exact linear value at
 * which round(255 * OETF(c)) steps from k to k+1 (Khronos Data Format §13.3).
 * code = #{k : c >= T[k]} is the correctly-rounded sRGB encode. */
static float g_srgb_T[255];
static int g_srgb_init = 0;

static void srgb_init(void) {
    if (g_srgb_init) return;
    for (int k = 0; k < 255; ++k) {
        const double v = ((double)k + 0.5) / 255.0;
        const double lin = (v <= 0.04045) ? v / 12.92 : pow((v + 0.055) / 1.055, 2.4);
        float f = (float)lin;
        if ((double)f < lin) f = nextafterf(f, INFINITY);
        g_srgb_T[k] = f;
    }
    g_srgb_init = 1;
}

float zro_srgb_threshold(uint32_t k) {
    srgb_init();
    return k < 255 ? g_srgb_T[k] : NAN;
}

static float clamp01(float c) {
    if (!(c > 0.0f)) return 0.0f; /* NaN -> 0 */
    if (c > 1.0f) return 1.0f;
    return c;
}

uint32_t zro_encode_unorm8(float c) { return (uint32_t)rintf(clamp01(c) * 255.0f); }

uint32_t zro_encode_srgb8(float c) {
    srgb_init();
    c = clamp01(c);
    uint32_t lo = 0, hi = 255; /* count of thresholds <= c, by bisection */
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (c >= g_srgb_T[mid]) lo = mid + 1; else hi = mid;
    }
    return lo;
}

uint32_t zro_format_bpp(int32_t f) {
    switch (f) {
    case F_R8G8B8A8_UNORM: case F_R8G8B8A8_SRGB: case F_B8G8R8A8_UNORM: case F_B8G8R8A8_SRGB:
        return 4;
    case F_R32G32B32A32_SFLOAT: return 16;
    default: return 0;
    }
}

static void store_color(const zro_target *t, uint32_t x, uint32_t y, const float c[4], uint32_t mask) {
    const int32_t f = t->color_format;
    const size_t idx = (size_t)y * t->width + x;
    if (f == F_R32G32B32A32_SFLOAT) {
        float *p = (float *)t->color + idx * 4;
        for (int i = 0; i < 4; ++i) if (mask & (1u << i)) p[i] = c[i];
        return;
    }
    uint8_t *p = t->color + idx * 4;
    const int srgb = (f == F_B8G8R8A8_SRGB || f == F_R8G8B8A8_SRGB);
    const int bgra = (f == F_B8G8R8A8_SRGB || f == F_B8G8R8A8_UNORM);
    uint32_t code[4];
    for (int i = 0; i < 3; ++i) code[i] = srgb ? zro_encode_srgb8(c[i]) : zro_encode_unorm8(c[i]);
    code[3] = zro_encode_unorm8(c[3]); /* sRGB formats store alpha linearly */
    const int pos[4] = {bgra ? 2 : 0, 1, bgra ? 0 : 2, 3};
    for (int i = 0; i < 4; ++i) if (mask & (1u << i)) p[pos[i]] = (uint8_t)code[i];
}

/* ------------------------------------------------------------------ clear */

/* Shard ownership (this repo's multi-GPU split; no reference
 * counterpart): the pixel columns [*x0, *x1) of tile row ty (tile x tile tiles)
 * that rank `rank` of `count` owns on a width x height target.  The first F =
 * floor(rows / count) * count tile rows go round robin (row ty to rank ty %
 * count); the tiles of the rows after them, row-major, are cut into count
 * consecutive runs, run r = [ceil(r n / count), ceil((r + 1) n / count)) of their
 * n tiles.  An empty range when the rank owns none of the row. */
static void owned_cols(uint32_t ty, uint32_t width, uint32_t height, uint32_t tile, uint32_t rank, uint32_t count,
                       int32_t *x0, int32_t *x1) {
    *x0 = 0;
    *x1 = (int32_t)width;
    if (count <= 1) return;
    const uint64_t tiles_x = (width + tile - 1) / tile, rows = (height + tile - 1) / tile;
    const uint64_t full = rows / count * count;
    if (ty < full) {
        if (ty % count != rank) *x1 = 0;
        return;
    }
    const uint64_t n = (rows - full) * tiles_x;
    const uint64_t lo = (rank * n + count - 1) / count, hi = ((rank + 1) * n + count - 1) / count;
    const int64_t i0 = (int64_t)((ty - full) * tiles_x);
    int64_t c0 = (int64_t)lo - i0, c1 = (int64_t)hi - i0; /* tiles [c0, c1) of this row */
    if (c0 < 0) c0 = 0;
    if (c1 > (int64_t)tiles_x) c1 = (int64_t)tiles_x;
    if (c0 >= c1) { *x1 = 0; return; }
    *x0 = (int32_t)(c0 * tile);
    *x1 = (int32_t)(c1 * tile < (int64_t)width ? c1 * tile : (int64_t)width);
}

void zro_clear(const zro_target *t, const int32_t ra[4], const float cc[4], int clear_colour,
               float cd, int clear_depth, uint32_t tile, uint32_t rank, uint32_t count) {
    int32_t x0 = ra[0] < 0 ? 0 : ra[0], y0 = ra[1] < 0 ? 0 : ra[1];
    int32_t x1 = ra[0] + ra[2], y1 = ra[1] + ra[3];
    if (x1 > (int32_t)t->width) x1 = (int32_t)t->width;
    if (y1 > (int32_t)t->height) y1 = (int32_t)t->height;
    for (int32_t y = y0; y < y1; ++y) {
        int32_t ox0, ox1;
        owned_cols((uint32_t)y / tile, t->width, t->height, tile, rank, count, &ox0, &ox1);
        for (int32_t x = x0 > ox0 ? x0 : ox0; x < x1 && x < ox1; ++x) {
            if (clear_colour && t->color) store_color(t, (uint32_t)x, (uint32_t)y, cc, 0xF);
            if (clear_depth && t->depth) t->depth[(size_t)y * t->width + x] = cd;
        }
    }
}

/* ------------------------------------------------------------ shader stages */

/* Vertex stages: SV_Position = float4(position, 1) (triangle.slang:21-22) for the
 * triangle / flat / Blinn-Phong programs; mul(View.view_proj, float4(position, 1))
 * for mesh.slang.  Varyings are the remaining inputs. */
static int program_attr_count(int32_t p) {
    return (p == ZRO_PROGRAM_BLINN_PHONG || p == ZRO_PROGRAM_MESH) ? 3 : 2;
}

typedef struct tri_setup {
    int32_t X[3], Y[3];
    float z[3], invw[3];
    float invA2;
    int32_t bias[3];
    int32_t px0, py0, px1, py1;
    uint32_t vid[3];     /* record order (after the orientation swap)                  */
    uint32_t ovid[3];    /* mesh: the primitive's vertex ids in API order               */
    float clip[3][4];    /* mesh: the primitive's clip-space vertices in API order      */
    int32_t valid;
} tri_setup;

static const float *fetchv(const zro_vertex_input *vi, uint32_t vid, uint32_t loc) {
    const uint32_t size = vi->attr_size[loc] ? vi->attr_size[loc] : 12u;
    const uint64_t off = (uint64_t)vid * vi->stride + vi->attr_offset[loc];
    if (off + size > vi->vertex_bytes) return NULL;
    return (const float *)(vi->vertex_data + off);
}

/* scissor ∩ render area ∩ attachment, inclusive */
static void clip_rect(const zro_target *t, const zro_draw_state *s, int32_t r[4]) {
    int32_t cx0 = s->scissor[0], cy0 = s->scissor[1];
    int32_t cx1 = s->scissor[0] + s->scissor[2] - 1, cy1 = s->scissor[1] + s->scissor[3] - 1;
    if (s->render_area[0] > cx0) cx0 = s->render_area[0];
    if (s->render_area[1] > cy0) cy0 = s->render_area[1];
    if (s->render_area[0] + s->render_area[2] - 1 < cx1) cx1 = s->render_area[0] + s->render_area[2] - 1;
    if (s->render_area[1] + s->render_area[3] - 1 < cy1) cy1 = s->render_area[1] + s->render_area[3] - 1;
    if (cx0 < 0) cx0 = 0;
    if (cy0 < 0) cy0 = 0;
    if (cx1 > (int32_t)t->width - 1) cx1 = (int32_t)t->width - 1;
    if (cy1 > (int32_t)t->height - 1) cy1 = (int32_t)t->height - 1;
    r[0] = cx0; r[1] = cy0; r[2] = cx1; r[3] = cy1;
}

static int64_t area2(const int32_t X[3], const int32_t Y[3]) {
    return (int64_t)(X[1] - X[0]) * (Y[2] - Y[0]) - (int64_t)(X[2] - X[0]) * (Y[1] - Y[0]);
}

/* Orientation (A2 > 0, v0 keeps its slot), top-left biases and clipped pixel bbox
 * of one snapped triangle whose facing was already tested.  1 if it can cover. */
static int finish_tri(const zro_target *t, const zro_draw_state *s, tri_setup *o) {
    int64_t A2 = area2(o->X, o->Y);
    if (A2 == 0) return 0;
    if (A2 < 0) {
        int32_t ti; float tf; uint32_t tu;
        ti = o->X[1]; o->X[1] = o->X[2]; o->X[2] = ti;
        ti = o->Y[1]; o->Y[1] = o->Y[2]; o->Y[2] = ti;
        tf = o->z[1]; o->z[1] = o->z[2]; o->z[2] = tf;
        tf = o->invw[1]; o->invw[1] = o->invw[2]; o->invw[2] = tf;
        tu = o->vid[1]; o->vid[1] = o->vid[2]; o->vid[2] = tu;
        A2 = -A2;
    }
    o->invA2 = 1.0f / (float)A2;
    /* top-left rule in y-down framebuffer space, edges opposite v0, v1, v2 */
    for (int i = 0; i < 3; ++i) {
        const int a = (i + 1) % 3, b = (i + 2) % 3;
        const int32_t dx = o->X[b] - o->X[a], dy = o->Y[b] - o->Y[a];
        const int tl = (dy < 0) || (dy == 0 && dx > 0);
        o->bias[i] = tl ? 0 : 1;
    }
    int32_t minX = o->X[0], maxX = o->X[0], minY = o->Y[0], maxY = o->Y[0];
    for (int k = 1; k < 3; ++k) {
        if (o->X[k] < minX) minX = o->X[k];
        if (o->X[k] > maxX) maxX = o->X[k];
        if (o->Y[k] < minY) minY = o->Y[k];
        if (o->Y[k] > maxY) maxY = o->Y[k];
    }
    /* pixel centres (p + 1/2) inside the fixed-point bbox, within the clip rect */
    int32_t cr[4];
    clip_rect(t, s, cr);
    int32_t px0 = (minX - 128 + 255) >> 8, px1 = (maxX - 128) >> 8;
    int32_t py0 = (minY - 128 + 255) >> 8, py1 = (maxY - 128) >> 8;
    if (px0 < cr[0]) px0 = cr[0];
    if (py0 < cr[1]) py0 = cr[1];
    if (px1 > cr[2]) px1 = cr[2];
    if (py1 > cr[3]) py1 = cr[3];
    if (px0 > px1 || py0 > py1) return 0;
    o->px0 = px0; o->py0 = py0; o->px1 = px1; o->py1 = py1;
    o->valid = 1;
    return 1;
}

/* Vertex ids of draw primitive `tri` (API order); 0 if an index is out of range. */
static int fetch_ids(const zro_vertex_input *vi, const zro_draw_cmd *cmd, uint32_t tri, int nattr, uint32_t vid[3]) {
    for (int k = 0; k < 3; ++k) {
        const uint64_t e = (uint64_t)cmd->first + (uint64_t)tri * 3u + (uint64_t)k;
        int64_t v;
        if (cmd->indexed) {
            const uint32_t isz = vi->index_type == 0 ? 2u : 4u;
            if ((e + 1) * isz > vi->index_bytes) return 0;
            const uint32_t ix = isz == 2 ? ((const uint16_t *)vi->index_data)[e]
                                         : ((const uint32_t *)vi->index_data)[e];
            v = (int64_t)ix + (int64_t)cmd->vertex_offset;
        } else {
            v = (int64_t)e;
        }
        if (v < 0 || v > 0xFFFFFFFFll) return 0;
        vid[k] = (uint32_t)v;
        for (int a = 0; a < nattr; ++a)
            if (!fetchv(vi, vid[k], (uint32_t)a)) return 0;
    }
    return 1;
}

/* mesh.slang vsmain: clip = view_proj * (p, 1), column-major M[c*4 + r]; per row
 * t = M0r*x, t = fma(M1r, y, t), t = fma(M2r, z, t), c_r = t + M3r. */
static void transform(const float *M, const float *p, float c[4]) {
    for (int r = 0; r < 4; ++r) {
        float t = M[r] * p[0];
        t = fmaf(M[4 + r], p[1], t);
        t = fmaf(M[8 + r], p[2], t);
        c[r] = t + M[12 + r];
    }
}

/* Sutherland-Hodgman against the Vulkan depth planes z >= 0, then z <= w (x and y
 * use the guard band), vertex order kept from v0; new vertex a + t (b - a),
 * t = da / (da - db).  Returns the polygon size (0, 3, 4 or 5). */
static int clip_polygon(const float in[3][4], float out[5][4]) {
    float a_[5][4], b_[5][4];
    int n = 3;
    memcpy(a_, in, sizeof(float) * 12);
    for (int plane = 0; plane < 2; ++plane) {
        const float(*src)[4] = plane == 0 ? (const float(*)[4])a_ : (const float(*)[4])b_;
        float(*dst)[4] = plane == 0 ? b_ : a_;
        int m = 0;
        for (int i = 0; i < n; ++i) {
            const float *a = src[i], *b = src[(i + 1) % n];
            const float da = plane == 0 ? a[2] : a[3] - a[2];
            const float db = plane == 0 ? b[2] : b[3] - b[2];
            if (da >= 0.0f) { memcpy(dst[m], a, sizeof(float) * 4); ++m; }
            if ((da >= 0.0f) != (db >= 0.0f)) {
                const float tt = da / (da - db);
                for (int k = 0; k < 4; ++k) dst[m][k] = fmaf(tt, b[k] - a[k], a[k]);
                ++m;
            }
        }
        n = m;
        if (n == 0) return 0;
    }
    memcpy(out, a_, sizeof(float) * 4 * (size_t)n);
    return n;
}

/* Primitive assembly + vertex stage + clip + viewport + snap + facing/cull +
 * bbox.  Fills up to 3 triangles (the mesh program's clipped fan; one otherwise)
 * and returns how many may produce fragments. */
static int setup_prim(const zro_target *t, const zro_draw_state *s, const zro_vertex_input *vi,
                      const zro_draw_cmd *cmd, uint32_t tri, tri_setup o[3], int *dropped_clip) {
    *dropped_clip = 0;
    o[0].valid = o[1].valid = o[2].valid = 0;
    const int nattr = program_attr_count(s->program);
    if (vi->attr_count < (uint32_t)nattr) return 0;
    uint32_t vid[3];
    if (!fetch_ids(vi, cmd, tri, nattr, vid)) return 0;
    /* viewport transform, Vulkan 1.3 §Controlling the Viewport */
    const float hw = s->viewport[2] * 0.5f, hh = s->viewport[3] * 0.5f;
    const float cx = s->viewport[0] + hw, cy = s->viewport[1] + hh;
    const float dr = s->viewport[5] - s->viewport[4], dmin = s->viewport[4];
    float poly[5][4];
    int n = 3;
    float clip[3][4];
    for (int k = 0; k < 3; ++k) {
        const float *pos = fetchv(vi, vid[k], 0);
        if (s->program == ZRO_PROGRAM_MESH) {
            transform(s->view_proj, pos, clip[k]);
        } else {
            clip[k][0] = pos[0]; clip[k][1] = pos[1]; clip[k][2] = pos[2]; clip[k][3] = 1.0f;
        }
    }
    if (s->program == ZRO_PROGRAM_MESH) {
        n = clip_polygon((const float(*)[4])clip, poly);
        if (n == 0) { *dropped_clip = 1; return 0; }
    } else {
        memcpy(poly, clip, sizeof clip);
    }
    int32_t X[5], Y[5];
    float Z[5], IW[5];
    for (int k = 0; k < n; ++k) {
        const float x = poly[k][0], y = poly[k][1], z = poly[k][2], w = poly[k][3];
        if (!(w > 0.0f)) { *dropped_clip = 1; return 0; }
        const float xd = x / w, yd = y / w, zd = z / w;
        const float xf = fmaf(xd, hw, cx), yf = fmaf(yd, hh, cy);
        if (!(fabsf(xf) < 4194304.0f && fabsf(yf) < 4194304.0f)) { *dropped_clip = 1; return 0; }
        X[k] = zro_snap(xf);
        Y[k] = zro_snap(yf);
        Z[k] = fmaf(zd, dr, dmin) + 0.0f; /* -0 -> +0 */
        IW[k] = 1.0f / w;
    }
    /* Vulkan facing of the (clipped) polygon: a = -1/2 sum(x_i y_{i+1} - x_{i+1} y_i),
     * summed over its fan as -A2/2 each; a > 0 is CCW. */
    int64_t Asum = 0;
    for (int k = 1; k + 1 < n; ++k) {
        const int32_t fx[3] = {X[0], X[k], X[k + 1]}, fy[3] = {Y[0], Y[k], Y[k + 1]};
        Asum += area2(fx, fy);
    }
    if (Asum == 0) return 0;
    const int ccw = Asum < 0;
    const int front = (s->front_face == 0) ? ccw : !ccw;
    if ((s->cull_mode & 1u) && front) return 0;
    if ((s->cull_mode & 2u) && !front) return 0;
    int nvalid = 0;
    for (int k = 1; k + 1 < n; ++k) {
        tri_setup *f = &o[k - 1];
        const int idx[3] = {0, k, k + 1};
        for (int j = 0; j < 3; ++j) {
            f->X[j] = X[idx[j]];
            f->Y[j] = Y[idx[j]];
            f->z[j] = Z[idx[j]];
            f->invw[j] = IW[idx[j]];
            f->vid[j] = vid[j];     /* unclipped (n == 3): the primitive's own vertices */
            f->ovid[j] = vid[j];
            for (int c = 0; c < 4; ++c) f->clip[j][c] = clip[j][c];
        }
        nvalid += finish_tri(t, s, f);
    }
    return nvalid;
}

static int depth_pass(int32_t op, float z, float d) {
    switch (op) {
    case OP_NEVER: return 0;
    case OP_LESS: return z < d;
    case OP_EQUAL: return z == d;
    case OP_LEQUAL: return z <= d;
    case OP_GREATER: return z > d;
    case OP_NOTEQUAL: return z != d;
    case OP_GEQUAL: return z >= d;
    default: return 1;
    }
}

static float dot3(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }

/* Perspective-correct interpolation (Vulkan 1.3 §Polygon Rasterization, Basic
 * Polygon Rasterization / barycentric interpolation), fixed operation order. */
static void interp3(const float *f0, const float *f1, const float *f2, const float pw[3], float inv,
                    float out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = ((pw[0] * f0[i] + pw[1] * f1[i]) + pw[2] * f2[i]) * inv;
}

/* mesh.slang barycentric planes E_i(p) = p . (h_j x h_k) of the primitive's
 * homogeneous screen vertices h = (x hw + w cx, y hh + w cy, w).
 * The plane constants are formed in double, relative to a reference pixel r =
 * floor(vertex 0's screen position) (clamped to the guard band), and rounded
 * once to float: E_i = c0 (px - rx) + c1 (py - ry) + c2r, c2r = E_i at r's
 * centre.  Evaluated per fragment in float with two fmaf. */
static void mesh_planes_eval(const zro_draw_state *s, const float clip[3][4], int32_t px, int32_t py, float E[3]) {
    const float hw = s->viewport[2] * 0.5f, hh = s->viewport[3] * 0.5f;
    const float cx = s->viewport[0] + hw, cy = s->viewport[1] + hh;
    double hX[3], hY[3], hW[3];
    for (int k = 0; k < 3; ++k) {
        hX[k] = (double)clip[k][0] * (double)hw + (double)clip[k][3] * (double)cx;
        hY[k] = (double)clip[k][1] * (double)hh + (double)clip[k][3] * (double)cy;
        hW[k] = (double)clip[k][3];
    }
    double rx = hW[0] > 0.0 ? floor(hX[0] / hW[0]) : 0.0, ry = hW[0] > 0.0 ? floor(hY[0] / hW[0]) : 0.0;
    rx = fmin(fmax(rx, -4194304.0), 4194304.0);
    ry = fmin(fmax(ry, -4194304.0), 4194304.0);
    const float dx = (float)px - (float)rx, dy = (float)py - (float)ry;
    for (int i = 0; i < 3; ++i) {
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        const double c0 = hY[j] * hW[k] - hW[j] * hY[k];
        const double c1 = hW[j] * hX[k] - hX[j] * hW[k];
        const double c2 = hX[j] * hY[k] - hY[j] * hX[k];
        const float c2r = (float)((c0 * (rx + 0.5) + c1 * (ry + 0.5)) + c2);
        E[i] = fmaf((float)c0, dx, fmaf((float)c1, dy, c2r));
    }
}

/* blinn_phong.slang / mesh.slang lighting: ks = 0.5, n = 32, ambient 0.05 */
static void blinn_phong(const float n[3], const float kd[3], float out[4]) {
    static const float L[3] = {0x1.3651a0p-2f, 0x1.02995cp-1f, 0x1.9dc22cp-1f}; /* norm(.3,.5,.8) */
    static const float H[3] = {0x1.465e8ap-3f, 0x1.0ff974p-2f, 0x1.e6d20ap-1f}; /* norm(L+V)     */
    const float len2 = dot3(n, n);
    const float rl = len2 > 0.0f ? 1.0f / sqrtf(len2) : 0.0f;
    const float N[3] = {n[0] * rl, n[1] * rl, n[2] * rl};
    float ndl = dot3(N, L), ndh = dot3(N, H);
    ndl = ndl > 0.0f ? ndl : 0.0f;
    ndh = ndh > 0.0f ? ndh : 0.0f;
    float sp = ndh * ndh; /* ndh^32 by five squarings */
    sp = sp * sp; sp = sp * sp; sp = sp * sp; sp = sp * sp;
    const float amb = 0.05f + ndl;
    for (int i = 0; i < 3; ++i) out[i] = kd[i] * amb + 0.5f * sp;
    out[3] = 1.0f;
}

/* Fragment stage for each built-in program. */
static void shade(const zro_draw_state *s, const zro_vertex_input *vi, const tri_setup *o,
                  int64_t w0, int64_t w1, int64_t w2, int32_t pxl, int32_t pyl, float out[4]) {
    const float b0 = (float)w0 * o->invA2, b1 = (float)w1 * o->invA2, b2 = (float)w2 * o->invA2;
    const float pw[3] = {b0 * o->invw[0], b1 * o->invw[1], b2 * o->invw[2]};
    const float inv = 1.0f / ((pw[0] + pw[1]) + pw[2]);
    out[3] = 1.0f;
    if (s->program == ZRO_PROGRAM_FLAT_COLOR) {
        /* flat_color.slang: nointerpolation colour from the provoking (first) vertex */
        const float *c = fetchv(vi, o->vid[0], 1);
        out[0] = c[0]; out[1] = c[1]; out[2] = c[2];
        return;
    }
    if (s->program == ZRO_PROGRAM_TRIANGLE) {
        /* triangle.slang:34-38: animated = c * (0.5 + 0.5*sin(Time.time*3 + c*6.28)) */
        float c[3];
        interp3(fetchv(vi, o->vid[0], 1), fetchv(vi, o->vid[1], 1), fetchv(vi, o->vid[2], 1), pw, inv, c);
        const float t3 = s->time * 3.0f;
        for (int i = 0; i < 3; ++i) {
            const float arg = t3 + c[i] * 6.28f;
            out[i] = c[i] * (0.5f + 0.5f * zro_sinf(arg));
        }
        return;
    }
    if (s->program == ZRO_PROGRAM_MESH) {
        /* mesh.slang: perspective-correct barycentrics of the primitive (not of
         * its clipped fan triangle) from its homogeneous screen vertices
         * h_i = (x_i*hw + w_i*cx, y_i*hh + w_i*cy, w_i): b_i = E_i / sum E, with
         * E_i = p . (h_j x h_k) at the pixel centre p = (px + .5, py + .5, 1). */
        float E[3];
        mesh_planes_eval(s, o->clip, pxl, pyl, E);
        const float einv = 1.0f / ((E[0] + E[1]) + E[2]);
        const float bb[3] = {E[0] * einv, E[1] * einv, E[2] * einv};
        float nrm[3], uv[2];
        const float *n0 = fetchv(vi, o->ovid[0], 1), *n1 = fetchv(vi, o->ovid[1], 1), *n2 = fetchv(vi, o->ovid[2], 1);
        const float *u0 = fetchv(vi, o->ovid[0], 2), *u1 = fetchv(vi, o->ovid[1], 2), *u2 = fetchv(vi, o->ovid[2], 2);
        for (int i = 0; i < 3; ++i) nrm[i] = (bb[0] * n0[i] + bb[1] * n1[i]) + bb[2] * n2[i];
        for (int i = 0; i < 2; ++i) uv[i] = (bb[0] * u0[i] + bb[1] * u1[i]) + bb[2] * u2[i];
        const float kdm[3] = {fmaf(uv[0], 0.3f, 0.35f), fmaf(uv[1], 0.3f, 0.35f), 0.7f};
        blinn_phong(nrm, kdm, out);
        return;
    }
    /* blinn_phong.slang: kd = colour */
    float n[3], kd[3];
    interp3(fetchv(vi, o->vid[0], 1), fetchv(vi, o->vid[1], 1), fetchv(vi, o->vid[2], 1), pw, inv, n);
    interp3(fetchv(vi, o->vid[0], 2), fetchv(vi, o->vid[1], 2), fetchv(vi, o->vid[2], 2), pw, inv, kd);
    blinn_phong(n, kd, out);
}

/* Rasterize one set-up triangle over rows [ry0, ry1] (inclusive) and columns
 * [cx0, cx1) (the band's owned pixels), in order. */
static void raster_rows(const zro_target *t, const zro_draw_state *s, const zro_vertex_input *vi,
                        const tri_setup *o, int32_t ry0, int32_t ry1, int32_t cx0, int32_t cx1, zro_stats *st) {
    int32_t y0 = o->py0 > ry0 ? o->py0 : ry0, y1 = o->py1 < ry1 ? o->py1 : ry1;
    const int32_t x0 = o->px0 > cx0 ? o->px0 : cx0, x1 = o->px1 < cx1 - 1 ? o->px1 : cx1 - 1;
    const int32_t dx0 = o->X[2] - o->X[1], dy0 = o->Y[2] - o->Y[1];
    const int32_t dx1 = o->X[0] - o->X[2], dy1 = o->Y[0] - o->Y[2];
    const int32_t dx2 = o->X[1] - o->X[0], dy2 = o->Y[1] - o->Y[0];
    const float dz1 = o->z[1] - o->z[0], dz2 = o->z[2] - o->z[0];
    /* depth is a plane in the biased edge values w_i - bias_i,
     * z = fmaf(w2', C2, fmaf(w1', C1, Z0)), C_i = dz_i * invA2, Z0 its value at w' = 0 */
    const float C1 = dz1 * o->invA2, C2 = dz2 * o->invA2;
    const float Z0 = fmaf((float)o->bias[2], C2, fmaf((float)o->bias[1], C1, o->z[0]));
    const float dlo = s->viewport[4] < s->viewport[5] ? s->viewport[4] : s->viewport[5];
    const float dhi = s->viewport[4] < s->viewport[5] ? s->viewport[5] : s->viewport[4];
    const int test = s->depth_test && t->depth;
    for (int32_t py = y0; py <= y1; ++py) {
        const int64_t Sy = (int64_t)py * 256 + 128;
        for (int32_t px = x0; px <= x1; ++px) {
            const int64_t Sx = (int64_t)px * 256 + 128;
            const int64_t w0 = (int64_t)dx0 * (Sy - o->Y[1]) - (int64_t)dy0 * (Sx - o->X[1]);
            const int64_t w1 = (int64_t)dx1 * (Sy - o->Y[2]) - (int64_t)dy1 * (Sx - o->X[2]);
            const int64_t w2 = (int64_t)dx2 * (Sy - o->Y[0]) - (int64_t)dy2 * (Sx - o->X[0]);
            if (w0 < o->bias[0] || w1 < o->bias[1] || w2 < o->bias[2]) continue;
            if (st) st->fragments_covered++;
            float z = fmaf((float)(w2 - o->bias[2]), C2, fmaf((float)(w1 - o->bias[1]), C1, Z0));
            if (z == 0.0f) z = 0.0f; /* canonical +0 */
            if (!(z >= dlo && z <= dhi)) continue; /* depth clip == 0<=z<=w clip for w>0 */
            const size_t idx = (size_t)py * t->width + (size_t)px;
            if (test) {
                if (!depth_pass(s->depth_op, z, t->depth[idx])) continue;
                if (s->depth_write) t->depth[idx] = z;
            }
            if (st) st->fragments_passed++;
            if (t->color) {
                float c[4];
                shade(s, vi, o, w0, w1, w2, px, py, c);
                store_color(t, (uint32_t)px, (uint32_t)py, c, s->color_write_mask);
            }
        }
    }
}

#define CHUNK 65536

int zro_draw(const zro_target *t, const zro_draw_state *s, const zro_vertex_input *vi,
             const zro_draw_cmd *cmd, int nthreads, zro_stats *stats) {
    if (s->tile_size == 0 || s->shard_count == 0 || s->shard_rank >= s->shard_count) return -1;
    if (t->color && zro_format_bpp(t->color_format) == 0) return -11;
    srgb_init();
    const uint64_t per_inst = cmd->count / 3u;
    const uint64_t total = per_inst * (uint64_t)cmd->instance_count;
    zro_stats st;
    memset(&st, 0, sizeof st);
    st.triangles_in = total;
    if (total == 0) { if (stats) *stats = st; return 0; }
    tri_setup *buf = (tri_setup *)malloc(sizeof(tri_setup) * 3 * (total < CHUNK ? total : CHUNK));
    if (!buf) return -1;
    const int32_t band = (int32_t)s->tile_size;
    const int32_t nbands = (int32_t)((t->height + (uint32_t)band - 1) / (uint32_t)band);
    (void)nthreads;
    for (uint64_t c0 = 0; c0 < total; c0 += CHUNK) {
        const int64_t n = (int64_t)((total - c0) < CHUNK ? (total - c0) : CHUNK);
        uint64_t ns = 0, nd = 0;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : ns, nd) schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            const uint32_t tri = (uint32_t)((c0 + (uint64_t)i) % per_inst);
            int dc = 0;
            ns += setup_prim(t, s, vi, cmd, tri, &buf[3 * i], &dc) > 0 ? 1u : 0u;
            nd += (uint64_t)dc;
        }
        st.triangles_setup += ns;
        st.triangles_dropped_clip += nd;
        uint64_t fc = 0, fp = 0;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : fc, fp) schedule(dynamic, 1)
        for (int32_t b = 0; b < nbands; ++b) {
            zro_stats ls;
            memset(&ls, 0, sizeof ls);
            const int32_t ry0 = b * band, ry1 = b * band + band - 1;
            int32_t cx0, cx1;
            owned_cols((uint32_t)b, t->width, t->height, s->tile_size, s->shard_rank, s->shard_count, &cx0, &cx1);
            if (cx0 >= cx1) continue;
            for (int64_t i = 0; i < 3 * n; ++i) { /* in API order; a primitive's fan triangles do not overlap */
                const tri_setup *o = &buf[i];
                if (!o->valid || o->py1 < ry0 || o->py0 > ry1 || o->px1 < cx0 || o->px0 >= cx1) continue;
                raster_rows(t, s, vi, o, ry0, ry1, cx0, cx1, &ls);
            }
            fc += ls.fragments_covered;
            fp += ls.fragments_passed;
        }
        st.fragments_covered += fc;
        st.fragments_passed += fp;
    }
    free(buf);
    if (stats) *stats = st;
    return 0;
}

int64_t zro_signed_area2(const float xy[6]) {
    int32_t X[3], Y[3];
    for (int k = 0; k < 3; ++k) { X[k] = zro_snap(xy[2 * k]); Y[k] = zro_snap(xy[2 * k + 1]); }
    return (int64_t)(X[1] - X[0]) * (Y[2] - Y[0]) - (int64_t)(X[2] - X[0]) * (Y[1] - Y[0]);
}
