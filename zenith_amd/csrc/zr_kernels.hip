// zr_kernels.hip — the MI355X (gfx950) draw path.
//
//   k_setup_bin  one launch, one 1024-thread workgroup per CU (fewer for small
//                draws), no grid barrier: vertex stage, clip (mesh program),
//                viewport, 8-bit sub-pixel snap, facing/cull, orientation,
//                top-left biases, clipped pixel bbox -> 32-B compact record (64-B
//                full record for large primitives); an LDS histogram of the
//                workgroup's (tile, primitive) pairs; returning atomics on the
//                per-tile counters give the workgroup's offsets in each tile's
//                fixed slab of the bin buffer; scatter of (primitive | cost
//                class) entries into the slabs.  Workgroups never wait for each
//                other, so nothing assumes co-residency.
//   k_tile       one 256- or 512-thread workgroup per 32x32 tile: LDS-resident
//                64-bit visibility keys (depth | primitive sequence) updated with
//                ds_min_u64 -- lane per primitive for small ones (cost-sorted
//                64-lane chunks), wave per primitive for large ones -- then a
//                resolve that shades each pixel's winner once, encodes to the
//                attachment format and writes colour + depth with coalesced
//                stores.  The attachment CLEAR is fused into the resolve.
//   k_route      partitioned multi-GPU setup: route primitives to the ranks
//                owning the tile rows they touch.
//   k_clear      a render pass without draws.
//
// Coverage/depth arithmetic is exact integer + explicitly ordered float math,
// bit-identical to the in-order CPU oracle (oracle/zr_oracle.c).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "zr_internal.h"
#include "zr_shading.h"

namespace zr {

// Diagnostic builds only (tools/build_variant.sh); production builds keep both 0.
#ifndef ZR_TILE_WORK_STATS
// Per-tile lane-walk steps and wave-path sweeps in the debug stamps (the counting
// code costs k_tile 5 VGPRs, one wave per SIMD at 512 threads).
#define ZR_TILE_WORK_STATS 0
#endif
#ifndef ZR_XCD_TILES
#define ZR_XCD_TILES 8       // tiles per XCD run (xcd_tile); 0 or 1: blockIdx order
#endif
#ifndef ZR_LANE_STEP
#define ZR_LANE_STEP 4       // pixels of a row per lane-walk step (2 or 4; 4: C3 tile pass -6.6 us, C1 -3)
#endif
#ifndef ZR_LARGE_LANES
#define ZR_LARGE_LANES 1     // 0: every large primitive takes k_tile's wave path; 2: the last cost bucket's too (A/B)
#endif
#ifndef ZR_TAB
#define ZR_TAB 1
#endif
#ifndef ZR_RESOLVE_DEDUP512
#define ZR_RESOLVE_DEDUP512 0  // 1: 512-thread tiles resolve through resolve_tile (each distinct winner fetched once per tile)
#endif
#ifndef ZR_TILE_DEBUG
#define ZR_TILE_DEBUG 0      // 1: k_tile honours the ZR_DEBUG timing switches and stamps
                             // (the checks cost the production kernel SGPRs)
#endif

// k_tile tuning constants (DESIGN.md §4 has the measurements behind each).
constexpr uint32_t kTileWgs = 8;  // 256-thread k_tile workgroups per CU the register budget is sized for
constexpr int kLaneStep = ZR_LANE_STEP;
// (8 pixels per step was measured slower and has no parity run: not a build option)
static_assert(kLaneStep == 2 || kLaneStep == 4, "lane walk: 2 or 4 pixels per step");
constexpr uint32_t kResolveBatch = 2;  // pixels per thread whose gathers are in flight together in the resolve
#ifndef ZR_BIG_LANES
#define ZR_BIG_LANES 8
#endif
#ifndef ZR_MID_LANES
#define ZR_MID_LANES 4
#endif
#ifndef ZR_MID_BUCKET
#define ZR_MID_BUCKET 24
#endif
constexpr uint32_t kBigLanes = ZR_BIG_LANES;    // lanes per entry at least, for the last cost bucket (127+ pair steps, ~253+ px)
constexpr uint32_t kMidLanes = ZR_MID_LANES;    // lanes per entry at least, for buckets kMidBucket..62
constexpr uint32_t kMidBucket = ZR_MID_BUCKET;  // first bucket of the middle run: 49+ pair steps (~97+ px of bbox ∩ tile)

__constant__ float c_srgbT[255] = ZR_SRGB_THRESHOLDS_INIT;

// k_tile's view of DrawParams::debug: zero unless built with ZR_TILE_DEBUG.
__device__ __forceinline__ uint32_t tile_debug(const DrawParams& P) { return ZR_TILE_DEBUG ? P.debug : 0u; }

// The draw's parameters read through an opaque pointer to the kernel-argument
// segment (every kernel here takes one DrawParams, at offset 0).  Each call starts
// a fresh reference: fields read after it are loaded there (s_load, scalar cache)
// instead of being hoisted to the kernel entry and held in SGPRs -- or spilled --
// across the whole kernel.  Used at phase boundaries of the large kernels.
typedef const __attribute__((address_space(4))) DrawParams* KernargParams;
__device__ __forceinline__ const DrawParams& kernarg_params() {
    KernargParams kp = (KernargParams)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *(const DrawParams*)kp;
}

// ------------------------------------------------------------------ helpers

__device__ __forceinline__ bool fetch_index(const DrawParams& P, uint64_t e, int64_t& v) {
    if (P.index_size == 0) {
        v = (int64_t)e;
        return true;
    }
    if ((e + 1) * P.index_size > P.ib_bytes) return false;
    const uint32_t ix = P.index_size == 2 ? (uint32_t)((const uint16_t*)P.ib)[e] : ((const uint32_t*)P.ib)[e];
    v = (int64_t)ix + (int64_t)P.vertex_offset;
    return true;
}

// Vertex ids of a primitive that k_setup_bin already validated (it won a pixel, so
// its indices were in range): no bounds checks, 32-bit arithmetic (a valid id fits).
// Triangle (within its instance) of draw primitive `gid` (instance-major order).
__device__ __forceinline__ uint32_t tri_of(const DrawParams& P, uint32_t gid) {
    return (P.tris_per_instance == P.draw_prims) ? gid : gid % P.tris_per_instance;
}

__device__ __forceinline__ void winner_vids(const DrawParams& P, uint32_t prim, uint32_t v[3]) {
    const uint32_t tri = tri_of(P, prim);
    const uint32_t e0 = P.first + tri * 3u;
    if (P.index_size == 4) {
        const uint3 ix = *reinterpret_cast<const uint3*>(P.ib + (uint64_t)e0 * 4);
        v[0] = ix.x; v[1] = ix.y; v[2] = ix.z;
    } else if (P.index_size == 2) {
        const uint16_t* ib = reinterpret_cast<const uint16_t*>(P.ib) + e0;
        v[0] = ib[0]; v[1] = ib[1]; v[2] = ib[2];
    } else {
        v[0] = e0; v[1] = e0 + 1u; v[2] = e0 + 2u;
        return;
    }
    const uint32_t off = (uint32_t)P.vertex_offset;  // two's complement: id + offset wraps to the valid id
    v[0] += off; v[1] += off; v[2] += off;
}

__device__ __forceinline__ const float* attr_ptr(const DrawParams& P, uint32_t vid, uint32_t loc) {
    return (const float*)(P.vb + (uint64_t)vid * P.stride + P.attr_offset[loc]);
}

__device__ __forceinline__ bool depth_pass(int op, float z, float d) {
    switch (op) {
    case 0: return false;
    case 1: return z < d;
    case 2: return z == d;
    case 3: return z <= d;
    case 4: return z > d;
    case 5: return z != d;
    case 6: return z >= d;
    default: return true;
    }
}

template <int MODE>
__device__ __forceinline__ unsigned long long init_key(float d) {
    const unsigned long long zb = __float_as_uint(d);
    const unsigned long long nz = (unsigned long long)(~__float_as_uint(d));
    switch (MODE) {
    case kDepthMinStrict: return zb << 32;
    case kDepthMinNonStrict: return (zb << 32) | 0xFFFFFFFFull;
    case kDepthMaxStrict: return nz << 32;
    case kDepthMaxNonStrict: return (nz << 32) | 0xFFFFFFFFull;
    default: return ~0ull;
    }
}

template <int MODE>
__device__ __forceinline__ unsigned long long frag_key(float z, uint32_t seq) {
    const unsigned long long zb = __float_as_uint(z);
    const unsigned long long nz = (unsigned long long)(~__float_as_uint(z));
    switch (MODE) {
    case kDepthMinStrict: return (zb << 32) | seq;
    case kDepthMinNonStrict: return (zb << 32) | (uint32_t)~seq;
    case kDepthMaxStrict: return (nz << 32) | seq;
    case kDepthMaxNonStrict: return (nz << 32) | (uint32_t)~seq;
    default: return (unsigned long long)(uint32_t)~seq;
    }
}

// 0 = no fragment of this draw won the pixel.
template <int MODE>
__device__ __forceinline__ uint32_t winner_seq(unsigned long long key) {
    const uint32_t lo = (uint32_t)key;
    switch (MODE) {
    case kDepthMinStrict:
    case kDepthMaxStrict: return lo;
    case kDepthMinNonStrict:
    case kDepthMaxNonStrict: return (uint32_t)~lo;
    default: return key == ~0ull ? 0u : (uint32_t)~lo;
    }
}

template <int MODE>
__device__ __forceinline__ float key_depth(unsigned long long key) {
    const uint32_t hi = (uint32_t)(key >> 32);
    return (MODE == kDepthMaxStrict || MODE == kDepthMaxNonStrict) ? __uint_as_float(~hi) : __uint_as_float(hi);
}

struct EdgeEval {
    long long w0, w1, w2;
};

__device__ __forceinline__ EdgeEval eval_edges(const TriRecord& r, int px, int py) {
    const int Sx = px * 256 + 128, Sy = py * 256 + 128;
    EdgeEval e;
    e.w0 = (long long)(r.X2 - r.X1) * (Sy - r.Y1) - (long long)(r.Y2 - r.Y1) * (Sx - r.X1);
    e.w1 = (long long)(r.X0 - r.X2) * (Sy - r.Y2) - (long long)(r.Y0 - r.Y2) * (Sx - r.X2);
    e.w2 = (long long)(r.X1 - r.X0) * (Sy - r.Y0) - (long long)(r.Y1 - r.Y0) * (Sx - r.X0);
    return e;
}

// Depth: a plane in the biased edge values w_i' = w_i - bias_i,
// z = fmaf(w2', C2, fmaf(w1', C1, Z0)) with C_i = dz_i * invA2 and Z0 = the plane
// at w' = 0, fmaf(bias2, C2, fmaf(bias1, C1, z0)).  The lane walk steps the
// biased values, so a sample costs two conversions and two FMAs.  Never -0 (z0
// is canonical +0 and a sum of nonzero terms that cancels rounds to +0).
struct DepthPlane {
    float C1, C2, Z0;
};
__device__ __forceinline__ DepthPlane depth_plane(float z0, float dz1, float dz2, float invA2, int b1, int b2) {
    DepthPlane d;
    d.C1 = dz1 * invA2;
    d.C2 = dz2 * invA2;
    d.Z0 = fmaf((float)b2, d.C2, fmaf((float)b1, d.C1, z0));
    return d;
}
__device__ __forceinline__ float plane_z(const DepthPlane& d, float w1b, float w2b) {
    return fmaf(w2b, d.C2, fmaf(w1b, d.C1, d.Z0));
}
// The top-left bias of the edge from vertex a to vertex b (y-down: an edge is
// top-left iff dy < 0 || (dy == 0 && dx > 0)); edge i is opposite vertex i.
__device__ __forceinline__ int edge_bias(int dx, int dy) { return ((dy < 0) || (dy == 0 && dx > 0)) ? 0 : 1; }

// The contract depth of record r at pixel (px, py) (last-wins resolve: no key
// carries it), from the record's vertices alone.
__device__ __forceinline__ float winner_depth(const TriRecord& r, int px, int py) {
    const EdgeEval e = eval_edges(r, px, py);
    const int b1 = edge_bias(r.X0 - r.X2, r.Y0 - r.Y2), b2 = edge_bias(r.X1 - r.X0, r.Y1 - r.Y0);
    const DepthPlane d = depth_plane(r.z0, r.dz1, r.dz2, r.invA2, b1, b2);
    return plane_z(d, (float)(e.w1 - b1), (float)(e.w2 - b2));
}

// Edge values at a pixel centre as floats (resolve: the winner's barycentrics).
// A small primitive's values fit int32 exactly (bbox <= 64 px a side),
// so (float)int32 equals (float)int64 there and the 64-bit products are skipped.
struct EdgeEvalF {
    float f0, f1, f2;
};

__device__ __forceinline__ EdgeEvalF eval_edges_f(const TriRecord& r, int px, int py) {
    const int Sx = px * 256 + 128, Sy = py * 256 + 128;
    EdgeEvalF e;
    if (r.flags & kFlagSmall) {
        // unsigned products: defined wraparound for the (discarded) fallback primitive
        // of pixels no fragment won, which may lie far outside its bbox
        auto ew = [](int ax, int ay, int bx, int by) {
            return (float)(int)((uint32_t)ax * (uint32_t)ay - (uint32_t)bx * (uint32_t)by);
        };
        e.f0 = ew(r.X2 - r.X1, Sy - r.Y1, r.Y2 - r.Y1, Sx - r.X1);
        e.f1 = ew(r.X0 - r.X2, Sy - r.Y2, r.Y0 - r.Y2, Sx - r.X2);
        e.f2 = ew(r.X1 - r.X0, Sy - r.Y0, r.Y1 - r.Y0, Sx - r.X0);
    } else {
        const EdgeEval w = eval_edges(r, px, py);
        e.f0 = (float)w.w0;
        e.f1 = (float)w.w1;
        e.f2 = (float)w.w2;
    }
    return e;
}

// ------------------------------------------------------------------ k_setup
//
// One workgroup per chunk of 256 * tris_per_thread primitives (coalesced: step k
// of every thread covers 256 consecutive primitives).  Tile overlaps are counted
// in an LDS histogram (no global atomics); the histogram row is written to
// counts[wg][*] for the column scan.

// Primitive assembly, split in stages so that a thread's loads for several
// primitives are in flight together (index loads, then position loads, then math).
struct PrimIn {
    uint32_t vid[3];
    float3 p[3];
    bool ok;
};

__device__ __forceinline__ void fetch_indices_gid(const DrawParams& P, uint32_t gid, PrimIn& in) {
    const uint32_t tri = tri_of(P, gid);
    const uint64_t e0 = (uint64_t)P.first + (uint64_t)tri * 3u;
    bool ok = true;
    if (P.index_size == 4 && tri < P.ib_tris) {  // ib_tris: the triangles whose 3 indices are in the buffer
        const uint3 ix = *reinterpret_cast<const uint3*>(P.ib + e0 * 4);  // one 12-B load
        if (P.vertex_offset == 0) {  // wave-uniform: u32 ids need no range check
            in.vid[0] = ix.x; in.vid[1] = ix.y; in.vid[2] = ix.z;
        } else {
            const int64_t v0 = (int64_t)ix.x + P.vertex_offset, v1 = (int64_t)ix.y + P.vertex_offset,
                          v2 = (int64_t)ix.z + P.vertex_offset;
            ok = v0 >= 0 && v0 <= 0xFFFFFFFFll && v1 >= 0 && v1 <= 0xFFFFFFFFll && v2 >= 0 && v2 <= 0xFFFFFFFFll;
            in.vid[0] = (uint32_t)v0; in.vid[1] = (uint32_t)v1; in.vid[2] = (uint32_t)v2;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            int64_t v = 0;
            ok = ok && fetch_index(P, e0 + (uint64_t)k, v);
            ok = ok && v >= 0 && v <= 0xFFFFFFFFll;
            in.vid[k] = (uint32_t)v;
        }
    }
    in.ok = ok;
}

// Setup record `pos` (< n_pos): the draw primitive itself.
__device__ __forceinline__ void fetch_indices(const DrawParams& P, uint32_t pos, uint32_t n_pos, PrimIn& in) {
    in.ok = pos < n_pos;
    if (in.ok) fetch_indices_gid(P, pos, in);
}

__device__ __forceinline__ void fetch_positions(const DrawParams& P, PrimIn& in) {
    if (!in.ok) return;
    // every attribute of the three vertices inside the buffer (vid_count: DrawParams)
    const bool ok = in.vid[0] < P.vid_count && in.vid[1] < P.vid_count && in.vid[2] < P.vid_count;
    in.ok = ok;
    if (!ok) return;
#pragma unroll
    for (int k = 0; k < 3; ++k) in.p[k] = *reinterpret_cast<const float3*>(attr_ptr(P, in.vid[k], 0));  // 12-B loads
}

// Setup geometry of one primitive (vertex stage, viewport, snap, facing/cull,
// orientation, top-left biases, clipped pixel bbox): false when the primitive
// produces no sample (dropped, culled, degenerate or outside the clip rect).
// k_route and k_setup_bin both call it, so a routed primitive's bbox is the one
// its owner's setup computes.
struct PrimGeom {
    int32_t X[3], Y[3];
    float z[3];
    uint32_t rv[3];
    uint32_t flags;
    long long A2;
    int32_t px0, py0, px1, py1;
};

// Orientation to A2 > 0 (v1/v2 swapped, v0 kept: kFlagSwapped), top-left biases,
// the small flag and the clipped pixel bbox of a snapped triangle whose facing
// was already tested.  False when no pixel centre of the clip rect is inside the bbox.
__device__ __forceinline__ bool orient_and_bound(const DrawParams& P, PrimGeom& g, long long A2) {
    int32_t* X = g.X;
    int32_t* Y = g.Y;
    uint32_t flags = 0;
    if (A2 < 0) {
        int32_t t = X[1]; X[1] = X[2]; X[2] = t;
        t = Y[1]; Y[1] = Y[2]; Y[2] = t;
        const float f = g.z[1]; g.z[1] = g.z[2]; g.z[2] = f;
        const uint32_t u = g.rv[1]; g.rv[1] = g.rv[2]; g.rv[2] = u;
        A2 = -A2;
        flags |= kFlagSwapped;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // top-left rule (y-down), edge i opposite vertex i
        const int a = (i + 1) % 3, b = (i + 2) % 3;
        const int32_t dx = X[b] - X[a], dy = Y[b] - Y[a];
        const bool tl = (dy < 0) || (dy == 0 && dx > 0);
        if (!tl) flags |= (kFlagBias0 << i);
    }
    const int32_t minX = min(X[0], min(X[1], X[2])), maxX = max(X[0], max(X[1], X[2]));
    const int32_t minY = min(Y[0], min(Y[1], Y[2])), maxY = max(Y[0], max(Y[1], Y[2]));
    if (maxX - minX <= kSmallExtent && maxY - minY <= kSmallExtent) flags |= kFlagSmall;
    g.px0 = max((minX - 128 + 255) >> 8, P.clip_x0);
    g.px1 = min((maxX - 128) >> 8, P.clip_x1);
    g.py0 = max((minY - 128 + 255) >> 8, P.clip_y0);
    g.py1 = min((maxY - 128) >> 8, P.clip_y1);
    g.flags = flags;
    g.A2 = A2;
    return g.px0 <= g.px1 && g.py0 <= g.py1;
}

__device__ __forceinline__ bool prim_geometry(const DrawParams& P, const PrimIn& in, PrimGeom& g, int& ndropped) {
    if (!in.ok) return false;
    g.rv[0] = in.vid[0]; g.rv[1] = in.vid[1]; g.rv[2] = in.vid[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float x = in.p[k].x, y = in.p[k].y, zc = in.p[k].z, w = 1.0f;  // vsmain (triangle.slang:22)
        if (!(w > 0.0f)) { ++ndropped; return false; }
        const float xd = x / w, yd = y / w, zd = zc / w;
        const float xf = fmaf(xd, P.hw, P.cx), yf = fmaf(yd, P.hh, P.cy);
        if (!(fabsf(xf) < 4194304.0f && fabsf(yf) < 4194304.0f)) { ++ndropped; return false; }
        g.X[k] = (int32_t)rintf(xf * 256.0f);
        g.Y[k] = (int32_t)rintf(yf * 256.0f);
        g.z[k] = fmaf(zd, P.dr, P.dmin) + 0.0f;  // -0 -> +0 (k_tile relies on it)
    }
    long long A2 = (long long)(g.X[1] - g.X[0]) * (g.Y[2] - g.Y[0]) - (long long)(g.X[2] - g.X[0]) * (g.Y[1] - g.Y[0]);
    const bool ccw = A2 < 0;  // Vulkan: a = -A2/2 > 0 is counter-clockwise
    const bool front = (P.front_face == 0) ? ccw : !ccw;
    if (A2 == 0 || ((P.cull_mode & 1u) && front) || ((P.cull_mode & 2u) && !front)) return false;
    return orient_and_bound(P, g, A2);
}

// mesh.slang vsmain: clip = view_proj * (p, 1), column-major M[c * 4 + r], per row
// t = M0r x; t = fma(M1r, y, t); t = fma(M2r, z, t); c_r = t + M3r (zr_oracle.c).
__device__ __forceinline__ void mesh_transform(const float* M, const float3 p, float c[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float t = M[r] * p.x;
        t = fmaf(M[4 + r], p.y, t);
        t = fmaf(M[8 + r], p.z, t);
        c[r] = t + M[12 + r];
    }
}

// The camera matrix of the draw: the View uniform (device memory), or for a
// pipeline whose vertex stage takes it as push constants (mesh_push.slang) the
// bytes zr_cmd_push_constants recorded, carried in this launch's kernel arguments
// (DrawParams::push; every kernel here takes the one DrawParams at offset 0).
__device__ __forceinline__ const float* view_matrix(const DrawParams& P) {
    if (P.view_push) {
        const KernargParams kp = (KernargParams)__builtin_amdgcn_kernarg_segment_ptr();
        return (const float*)kp->push;
    }
    return P.view_proj;
}

// Sutherland-Hodgman against the Vulkan depth planes z >= 0, then z <= w (x / y
// use the guard band), vertex order kept from v0: new vertex a + t (b - a),
// t = da / (da - db).  Returns the polygon size (0, 3, 4 or 5).  Only primitives
// crossing a plane get here (mesh_geometry's fast path takes the rest).
__device__ __noinline__ int clip_polygon(const float (*in)[4], float (*out)[4]) {
    float a_[5][4], b_[5][4];
    int n = 3;
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 4; ++k) a_[i][k] = in[i][k];
    for (int plane = 0; plane < 2; ++plane) {
        float (*src)[4] = plane == 0 ? a_ : b_;
        float (*dst)[4] = plane == 0 ? b_ : a_;
        int m = 0;
        for (int i = 0; i < n; ++i) {
            const float* a = src[i];
            const float* b = src[(i + 1) % n];
            const float da = plane == 0 ? a[2] : a[3] - a[2];
            const float db = plane == 0 ? b[2] : b[3] - b[2];
            if (da >= 0.0f) {
                for (int k = 0; k < 4; ++k) dst[m][k] = a[k];
                ++m;
            }
            if ((da >= 0.0f) != (db >= 0.0f)) {
                const float tt = da / (da - db);
                for (int k = 0; k < 4; ++k) dst[m][k] = fmaf(tt, b[k] - a[k], a[k]);
                ++m;
            }
        }
        n = m;
        if (n == 0) return 0;
    }
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 4; ++k) out[i][k] = a_[i][k];
    return n;
}

// The mesh program's setup geometry: vertex stage, clip, viewport, snap, facing
// of the clipped polygon (sum of its fan's A2), cull, then each fan triangle
// (p0, pk, pk+1) oriented and bounded on its own.  valid bit k: fan k may cover.
struct MeshFans {
    PrimGeom f[kMeshFans];
    uint32_t valid;
};

__device__ __forceinline__ bool mesh_geometry(const DrawParams& P, const PrimIn& in, MeshFans& m, int& ndropped) {
    m.valid = 0;
    if (!in.ok) return false;
    float c[3][4];
#pragma unroll
    for (int k = 0; k < 3; ++k) mesh_transform(view_matrix(P), in.p[k], c[k]);
    bool inside = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) inside = inside && c[k][2] >= 0.0f && c[k][3] - c[k][2] >= 0.0f;
    float poly[5][4];
    int n = 3;
    if (inside) {
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) poly[k][j] = c[k][j];
    } else {
        n = clip_polygon(c, poly);
        if (n == 0) {
            ++ndropped;
            return false;
        }
    }
    int32_t X[5], Y[5];
    float Z[5];
    for (int k = 0; k < n; ++k) {
        const float x = poly[k][0], y = poly[k][1], z = poly[k][2], w = poly[k][3];
        if (!(w > 0.0f)) { ++ndropped; return false; }
        const float xd = x / w, yd = y / w, zd = z / w;
        const float xf = fmaf(xd, P.hw, P.cx), yf = fmaf(yd, P.hh, P.cy);
        if (!(fabsf(xf) < 4194304.0f && fabsf(yf) < 4194304.0f)) { ++ndropped; return false; }
        X[k] = (int32_t)rintf(xf * 256.0f);
        Y[k] = (int32_t)rintf(yf * 256.0f);
        Z[k] = fmaf(zd, P.dr, P.dmin) + 0.0f;  // -0 -> +0
    }
    long long Asum = 0;
    for (int k = 1; k + 1 < n; ++k)
        Asum += (long long)(X[k] - X[0]) * (Y[k + 1] - Y[0]) - (long long)(X[k + 1] - X[0]) * (Y[k] - Y[0]);
    const bool ccw = Asum < 0;
    const bool front = (P.front_face == 0) ? ccw : !ccw;
    if (Asum == 0 || ((P.cull_mode & 1u) && front) || ((P.cull_mode & 2u) && !front)) return false;
    for (int k = 1; k + 1 < n; ++k) {
        PrimGeom& g = m.f[k - 1];
        g.X[0] = X[0]; g.X[1] = X[k]; g.X[2] = X[k + 1];
        g.Y[0] = Y[0]; g.Y[1] = Y[k]; g.Y[2] = Y[k + 1];
        g.z[0] = Z[0]; g.z[1] = Z[k]; g.z[2] = Z[k + 1];
        g.rv[0] = in.vid[0]; g.rv[1] = in.vid[1]; g.rv[2] = in.vid[2];
        const long long A2 = (long long)(g.X[1] - g.X[0]) * (g.Y[2] - g.Y[0]) -
                             (long long)(g.X[2] - g.X[0]) * (g.Y[1] - g.Y[0]);
        if (A2 != 0 && orient_and_bound(P, g, A2)) m.valid |= 1u << (k - 1);
    }
    return m.valid != 0;
}

// mesh_geometry for a primitive that needs no clipping (all vertices inside
// 0 <= z <= w): one fan, the same operations on fixed indices, so everything
// stays in registers (the general path's polygon arrays live in scratch).
__device__ __forceinline__ bool mesh_geometry_unclipped(const DrawParams& P, const PrimIn& in, const float c[3][4],
                                                        PrimGeom& g, int& ndropped) {
    int32_t X[3], Y[3];
    float Z[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float x = c[k][0], y = c[k][1], z = c[k][2], w = c[k][3];
        if (!(w > 0.0f)) { ++ndropped; return false; }
        const float xd = x / w, yd = y / w, zd = z / w;
        const float xf = fmaf(xd, P.hw, P.cx), yf = fmaf(yd, P.hh, P.cy);
        if (!(fabsf(xf) < 4194304.0f && fabsf(yf) < 4194304.0f)) { ++ndropped; return false; }
        X[k] = (int32_t)rintf(xf * 256.0f);
        Y[k] = (int32_t)rintf(yf * 256.0f);
        Z[k] = fmaf(zd, P.dr, P.dmin) + 0.0f;  // -0 -> +0
    }
    const long long A2 = (long long)(X[1] - X[0]) * (Y[2] - Y[0]) - (long long)(X[2] - X[0]) * (Y[1] - Y[0]);
    const bool ccw = A2 < 0;
    const bool front = (P.front_face == 0) ? ccw : !ccw;
    if (A2 == 0 || ((P.cull_mode & 1u) && front) || ((P.cull_mode & 2u) && !front)) return false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        g.X[k] = X[k];
        g.Y[k] = Y[k];
        g.z[k] = Z[k];
        g.rv[k] = in.vid[k];
    }
    return orient_and_bound(P, g, A2);
}

// Counts the owned (tile, primitive) pairs of a set-up triangle in the LDS
// histogram; returns how many there are.
// The first tile row at or after ty0 that this shard owns (ty % G == rank) and its
// index among the owned rows; the next owned row is G further.  One division per
// primitive, none when the target is not sharded (G == 1, wave-uniform).
__device__ __forceinline__ int first_owned_row(uint32_t G, uint32_t rank, int ty0, uint32_t& orow) {
    if (G == 1u) {
        orow = (uint32_t)ty0;
        return ty0;
    }
    const uint32_t q = (uint32_t)ty0 / G, m = (uint32_t)ty0 - q * G;
    orow = m <= rank ? q : q + 1u;
    return (int)(orow * G + rank);
}

// Calls fn(owned tile index, tx, ty) for every tile of [tx0, tx1] x [ty0, ty1]
// this shard owns (ShardGeom): its round-robin rows, then the leftover rows'
// tiles inside its run.  G == 1: every tile, index ty * tiles_x + tx.
template <typename Fn>
__device__ __forceinline__ void for_owned_tiles(uint32_t G, uint32_t rank, uint32_t tiles_x, uint32_t full_rows,
                                                uint32_t own_rows, uint32_t left_lo, uint32_t left_hi, int tx0, int ty0,
                                                int tx1, int ty1, Fn&& fn) {
    uint32_t orow;
    const int tyf = min(ty1, (int)full_rows - 1);
    for (int ty = first_owned_row(G, rank, ty0, orow); ty <= tyf; ty += (int)G, ++orow) {
        const uint32_t row = orow * tiles_x;
        for (int tx = tx0; tx <= tx1; ++tx) fn(row + (uint32_t)tx, tx, ty);
    }
    for (int ty = max(ty0, (int)full_rows); ty <= ty1; ++ty) {  // leftover rows (G > 1 only)
        const int i0 = (ty - (int)full_rows) * (int)tiles_x;
        const int c0 = max(tx0, (int)left_lo - i0), c1 = min(tx1, (int)left_hi - 1 - i0);
        const uint32_t base = own_rows * tiles_x + (uint32_t)(i0 - (int)left_lo);
        for (int tx = c0; tx <= c1; ++tx) fn(base + (uint32_t)tx, tx, ty);
    }
}

__device__ __forceinline__ uint32_t count_owned_box(const DrawParams& P, int px0, int py0, int px1, int py1,
                                                    uint32_t* s_hist) {
    const uint32_t tsh = P.tile_shift;
    const int tx0 = px0 >> tsh, tx1 = px1 >> tsh;
    const int ty0 = py0 >> tsh, ty1 = py1 >> tsh;
    uint32_t owned = 0;
    for_owned_tiles(P.shard_count, P.shard_rank, P.tiles_x, P.full_rows, P.own_rows, P.left_lo, P.left_hi, tx0, ty0,
                    tx1, ty1, [&](uint32_t t, int, int) {
                        atomicAdd(&s_hist[t], 1u);
                        ++owned;
                    });
    return owned;
}

__device__ __forceinline__ uint32_t count_owned(const DrawParams& P, const PrimGeom& g, uint32_t* s_hist) {
    return count_owned_box(P, g.px0, g.py0, g.px1, g.py1, s_hist);
}

// A compact record (as two 16-B words) whose primitive is too large for int16 deltas.
__device__ __forceinline__ bool compact_is_large(const int4 q0) { return (int16_t)(q0.z & 0xFFFF) == kCompactLarge; }
// A large primitive covering at most a quarter of its bbox (dy1 == 1 in its
// compact record; the lane walk takes it even in the last cost bucket, k_tile).
__device__ __forceinline__ bool compact_is_sliver(const int4 q0) { return (q0.z >> 16) == 1; }

// The compact record and the clipped pixel bbox of a set-up triangle.
__device__ __forceinline__ TriCompact make_compact(const PrimGeom& g, BBox& box) {
    const int32_t* X = g.X;
    const int32_t* Y = g.Y;
    const float invA2 = 1.0f / (float)g.A2;
    const bool small = (g.flags & kFlagSmall) != 0u;
    TriCompact c;
    c.X0 = X[0]; c.Y0 = Y[0];
    c.dx1 = small ? (int16_t)(X[1] - X[0]) : kCompactLarge;
    const long long bbox = (long long)(max(X[0], max(X[1], X[2])) - min(X[0], min(X[1], X[2]))) *
                           (max(Y[0], max(Y[1], Y[2])) - min(Y[0], min(Y[1], Y[2])));
    c.dy1 = small ? (int16_t)(Y[1] - Y[0]) : (int16_t)(bbox >= 2 * g.A2 ? 1 : 0);  // large: the sliver flag
    c.dx2 = small ? (int16_t)(X[2] - X[0]) : (int16_t)0;
    c.dy2 = small ? (int16_t)(Y[2] - Y[0]) : (int16_t)0;
    c.z0 = g.z[0];
    c.dz1 = g.z[1] - g.z[0];
    c.dz2 = g.z[2] - g.z[0];
    c.invA2s = (g.flags & kFlagSwapped) ? -invA2 : invA2;
    box.bb0 = (uint32_t)g.px0 | ((uint32_t)g.py0 << 16);
    box.bb1 = (uint32_t)g.px1 | ((uint32_t)g.py1 << 16);
    return c;
}

// Stores setup record `rec` (compact, plus the full record for a large
// triangle) and returns its tile bbox.
__device__ __forceinline__ BBox write_record(const DrawParams& P, uint32_t rec, const PrimGeom& g) {
    BBox box;
    const TriCompact c = make_compact(g, box);
    P.records[rec] = c;
    if (!(g.flags & kFlagSmall)) {
        TriRecord r;
        r.X0 = g.X[0]; r.Y0 = g.Y[0]; r.X1 = g.X[1]; r.Y1 = g.Y[1]; r.X2 = g.X[2]; r.Y2 = g.Y[2];
        r.z0 = c.z0; r.dz1 = c.dz1; r.dz2 = c.dz2;
        r.invA2 = fabsf(c.invA2s);
        r.v0 = g.rv[0]; r.v1 = g.rv[1]; r.v2 = g.rv[2];
        r.bb0 = box.bb0;
        r.bb1 = box.bb1;
        r.flags = g.flags;
        P.records_big[rec] = r;
    }
    return box;
}

// The mesh program's barycentric planes: with the homogeneous
// screen vertices h_i = (x_i hw + w_i cx, y_i hh + w_i cy, w_i) of the primitive
// (not of its clipped fans), E_i(p) = p . (h_j x h_k) = c0 fx + c1 fy + c2.
// Evaluated relative to a reference pixel r near the primitive (r = floor of
// vertex 0's screen position), E_i = c0 (px - rx) + c1 (py - ry) + c2r with c2r
// = E_i at r's centre: the plane constants are formed in double and rounded once,
// so the resolve's float32 evaluation has no cancellation between large terms.
// e = {c0_0, c1_0, c2r_0, c0_1, c1_1, c2r_1, c0_2, c1_2, c2r_2, rx, ry, 0}
// (zr_oracle.c mesh_planes, same operations).
__device__ __forceinline__ void mesh_edge_planes(const DrawParams& P, const float3 p[3], float e[12]) {
    double hX[3], hY[3], hW[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float c[4];
        mesh_transform(view_matrix(P), p[k], c);
        hX[k] = (double)c[0] * (double)P.hw + (double)c[3] * (double)P.cx;
        hY[k] = (double)c[1] * (double)P.hh + (double)c[3] * (double)P.cy;
        hW[k] = (double)c[3];
    }
    // (a primitive reaching here has w > 0 at vertex 0 unless it was clipped; the
    // reference pixel only has to be finite: clamped to the guard band)
    double rx = hW[0] > 0.0 ? floor(hX[0] / hW[0]) : 0.0, ry = hW[0] > 0.0 ? floor(hY[0] / hW[0]) : 0.0;
    rx = fmin(fmax(rx, -4194304.0), 4194304.0);
    ry = fmin(fmax(ry, -4194304.0), 4194304.0);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        const double c0 = hY[j] * hW[k] - hW[j] * hY[k];
        const double c1 = hW[j] * hX[k] - hX[j] * hW[k];
        const double c2 = hX[j] * hY[k] - hY[j] * hX[k];
        e[3 * i + 0] = (float)c0;
        e[3 * i + 1] = (float)c1;
        e[3 * i + 2] = (float)((c0 * (rx + 0.5) + c1 * (ry + 0.5)) + c2);
    }
    e[9] = (float)rx;
    e[10] = (float)ry;
    e[11] = 0.0f;
}

// E_i of pixel (px, py) from the stored planes (float32, see mesh_edge_planes).
__device__ __forceinline__ void mesh_plane_eval(const float* e, int px, int py, float E[3]) {
    const float dx = (float)px - e[9], dy = (float)py - e[10];  // exact: integers below 2^24
#pragma unroll
    for (int i = 0; i < 3; ++i) E[i] = fmaf(e[3 * i], dx, fmaf(e[3 * i + 1], dy, e[3 * i + 2]));
}

// Setup record index of fan k of mesh primitive p (zr_internal.h kMeshFans).
__device__ __forceinline__ uint32_t mesh_record(const DrawParams& P, uint32_t p, uint32_t k) {
    return k ? P.prims + 2u * p + k - 1u : p;
}

// The mesh program's setup of primitive `prim`: returns fan 0's bbox, stores fans
// 1 and 2's in their global slots (empty when absent).
__device__ __forceinline__ BBox setup_finish_mesh(const DrawParams& P, uint32_t prim, const PrimIn& in,
                                                  uint32_t* s_hist, int& nvalid, int& ndropped) {
    BBox box[kMeshFans];
#pragma unroll
    for (uint32_t k = 0; k < kMeshFans; ++k) box[k] = BBox{kEmptyBox, 0u};
    bool fast = in.ok;
    float c[3][4];
    if (fast) {
#pragma unroll
        for (int k = 0; k < 3; ++k) mesh_transform(view_matrix(P), in.p[k], c[k]);
#pragma unroll
        for (int k = 0; k < 3; ++k) fast = fast && c[k][2] >= 0.0f && c[k][3] - c[k][2] >= 0.0f;
    }
    if (fast) {
        PrimGeom g;
        if (mesh_geometry_unclipped(P, in, c, g, ndropped)) {
            ++nvalid;
            if (count_owned(P, g, s_hist)) {
                box[0] = write_record(P, prim, g);
                float e[12];
                mesh_edge_planes(P, in.p, e);
                float4* q = P.mesh_edges + (size_t)prim * 3u;
                q[0] = make_float4(e[0], e[1], e[2], e[3]);
                q[1] = make_float4(e[4], e[5], e[6], e[7]);
                q[2] = make_float4(e[8], e[9], e[10], e[11]);
            }
        }
    } else {  // clipped (or invalid): the general path
        MeshFans m;
        if (mesh_geometry(P, in, m, ndropped)) {
            ++nvalid;
            bool owned = false;
            for (uint32_t k = 0; k < kMeshFans; ++k) {
                if (!((m.valid >> k) & 1u)) continue;
                if (count_owned(P, m.f[k], s_hist)) {
                    box[k] = write_record(P, mesh_record(P, prim, k), m.f[k]);
                    owned = true;
                }
            }
            if (owned) {  // the resolve's barycentric planes (shade_mesh)
                float e[12];
                mesh_edge_planes(P, in.p, e);
                float4* q = P.mesh_edges + (size_t)prim * 3u;
                q[0] = make_float4(e[0], e[1], e[2], e[3]);
                q[1] = make_float4(e[4], e[5], e[6], e[7]);
                q[2] = make_float4(e[8], e[9], e[10], e[11]);
            }
        }
    }
    P.bboxes[mesh_record(P, prim, 1)] = box[1];
    P.bboxes[mesh_record(P, prim, 2)] = box[2];
    return box[0];
}

// A micro primitive: its clipped bbox is one pixel, so at most that pixel's
// centre is a sample, and it is small (extents <= 64 px), so its edge values
// there fit int32 (products below 2^28, as in k_tile's lane walk).  Whether it
// covers the sample, by k_tile's biased sign test: one that does not yields no
// fragment and needs neither a record nor a bin entry (DrawParams::micro; k_tile
// tests the covered ones again, with their depth).
__device__ __forceinline__ bool micro_covers(const PrimGeom& g) {
    const int Sx = g.px0 * 256 + 128, Sy = g.py0 * 256 + 128;
    const int* X = g.X;
    const int* Y = g.Y;
    const int w0 = (X[2] - X[1]) * (Sy - Y[1]) - (Y[2] - Y[1]) * (Sx - X[1]) - (int)((g.flags >> 1) & 1u);
    const int w1 = (X[0] - X[2]) * (Sy - Y[2]) - (Y[0] - Y[2]) * (Sx - X[2]) - (int)((g.flags >> 2) & 1u);
    const int w2 = (X[1] - X[0]) * (Sy - Y[0]) - (Y[1] - Y[0]) * (Sx - X[0]) - (int)((g.flags >> 3) & 1u);
    return (w0 | w1 | w2) >= 0;
}

// Setup of draw primitive `prim`; returns its tile bbox (empty when culled,
// owning no tile, or a micro primitive that misses its sample).
__device__ __forceinline__ BBox setup_finish(const DrawParams& P, uint32_t prim, const PrimIn& in, uint32_t* s_hist,
                                             int& nvalid, int& ndropped, int& nmicro) {
    BBox box{kEmptyBox, 0u};
    PrimGeom g;
    if (prim_geometry(P, in, g, ndropped)) {
        ++nvalid;
        if (P.micro && g.px0 == g.px1 && g.py0 == g.py1 && (g.flags & kFlagSmall)) {
            if (!micro_covers(g)) return box;  // no fragment: no record, no bin entry
            ++nmicro;
        }
        if (count_owned(P, g, s_hist)) box = write_record(P, prim, g);
    }
    return box;
}

// Records mode (partitioned setup): received entry `pos` of the
// blocks (s_pre: exclusive prefix of the blocks' counts, G + 1 entries, in LDS).
// The sender set the primitive up: its compact record is stored at its draw id
// and its bbox counted; a large primitive (no compact form) is set up again here
// from the vertices every rank holds.  Returns the bbox; *gid = the draw id.
__device__ __forceinline__ BBox receive_entry(const DrawParams& P, const uint32_t* s_pre, uint32_t pos, uint32_t* s_hist,
                                              int& nvalid, int& ndropped, uint32_t& gid) {
    uint32_t src = 0;
    while (src + 1u < P.shard_count && pos >= s_pre[src + 1u]) ++src;
    const int4* e = reinterpret_cast<const int4*>(P.rlist + (size_t)src * route_block_bytes(P.route_cap) +
                                                  sizeof(RouteHeader) + (size_t)(pos - s_pre[src]) * sizeof(RouteEntry));
    const int4 q0 = e[0], q1 = e[1], q2 = e[2];
    gid = (uint32_t)q2.z;
    BBox box{(uint32_t)q2.x, (uint32_t)q2.y};
    ++nvalid;
    if (!compact_is_large(q0)) {
        int4* r = reinterpret_cast<int4*>(P.records + gid);
        r[0] = q0;
        r[1] = q1;
        count_owned_box(P, (int)(box.bb0 & 0xFFFFu), (int)(box.bb0 >> 16), (int)(box.bb1 & 0xFFFFu), (int)(box.bb1 >> 16),
                        s_hist);
        return box;
    }
    PrimIn in;
    fetch_indices_gid(P, gid, in);
    fetch_positions(P, in);
    PrimGeom g;
    if (prim_geometry(P, in, g, ndropped) && count_owned(P, g, s_hist)) return write_record(P, gid, g);
    return BBox{kEmptyBox, 0u};
}

// ----------------------------------------------------------------- k_route
//
// Partitioned setup, step 1 (tile-row shards): one pass over this
// rank's primitive range [route_lo, route_hi).  Thread t of workgroup c sets up
// primitive route_lo + c * kRouteChunk + t (the same setup geometry k_setup_bin
// computes) and appends its RouteEntry -- compact record, bbox, draw id -- to the
// block of every rank owning a tile row the bbox touches (ty % G == rank).  A
// workgroup reserves its run in a block with one returning atomic per
// destination on the block header's `total` (zero before every route: this
// rank's previous records-mode setup on the scratch set, or the runtime, resets
// it), so runs land in any order -- the receiver keys records by the draw id,
// so block order carries no meaning.  Entries past a block's capacity are
// dropped; the receiver reads count = min(total, capacity) and sees the overflow.
__device__ __forceinline__ uint32_t dest_mask(const DrawParams& P, const PrimGeom& g) {
    const uint32_t G = P.shard_count;
    const uint32_t tsh = P.tile_shift;  // (kTileShift: shards bin 32-px tiles)
    const int ty0 = g.py0 >> tsh, ty1 = g.py1 >> tsh;
    const int tx0 = g.px0 >> tsh, tx1 = g.px1 >> tsh;
    const uint32_t all = G >= 32u ? 0xFFFFFFFFu : (1u << G) - 1u;
    const int tyf = min(ty1, (int)P.full_rows - 1);  // round-robin rows: owner ty % G
    uint32_t m = 0;
    if (tyf >= ty0) m = (uint32_t)(tyf - ty0) + 1u >= G ? all : 0u;
    if (!m)
        for (int ty = ty0; ty <= tyf; ++ty) m |= 1u << ((uint32_t)ty % G);
    if (ty1 >= (int)P.full_rows) {  // leftover rows: the owners of the bbox's columns, a contiguous rank range per row
        const uint64_t n = (uint64_t)(P.tiles_y - P.full_rows) * P.tiles_x;
        for (int ty = max(ty0, (int)P.full_rows); ty <= ty1; ++ty) {
            const uint64_t i0 = (uint64_t)(ty - (int)P.full_rows) * P.tiles_x;
            const uint32_t ra = (uint32_t)((i0 + (uint64_t)tx0) * G / n), rb = (uint32_t)((i0 + (uint64_t)tx1) * G / n);
            m |= (rb >= 31u ? 0xFFFFFFFFu : (2u << rb) - 1u) & ~((1u << ra) - 1u);
        }
    }
    return m & all;
}

__global__ __launch_bounds__(kRouteThreads) void k_route(DrawParams P) {
    constexpr uint32_t kWaves = kRouteThreads / 64;
    static_assert(kRouteChunk == kRouteThreads, "k_route: one primitive per thread");
    __shared__ uint32_t s_off[kWaves][kMaxShards];  // entries per (wave, destination) -> run offsets
    __shared__ uint32_t s_base[kMaxShards];
    const uint32_t G = P.shard_count, c = blockIdx.x, tid = threadIdx.x;
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    const uint32_t gid = P.route_lo + c * kRouteChunk + tid;
    PrimIn in;
    in.ok = gid < P.route_hi;
    if (in.ok) fetch_indices_gid(P, gid, in);
    fetch_positions(P, in);
    int ndropped = 0;
    PrimGeom g;
    const uint32_t m = prim_geometry(P, in, g, ndropped) ? dest_mask(P, g) : 0u;
    BBox box{kEmptyBox, 0u};
    TriCompact rec;
    if (m) rec = make_compact(g, box);
    for (uint32_t d = 0; d < G; ++d) {
        const uint32_t n = (uint32_t)__popcll(__ballot((m >> d) & 1u));
        if (lane == 0) s_off[wave][d] = n;
    }
    __syncthreads();
    const uint64_t block = route_block_bytes(P.route_cap);
    if (tid < G) {
        uint32_t run = 0;
        for (uint32_t i = 0; i < kWaves; ++i) {
            const uint32_t n = s_off[i][tid];
            s_off[i][tid] = run;
            run += n;
        }
        uint32_t* total = &reinterpret_cast<RouteHeader*>(P.route_out + (size_t)tid * block)->total;
        s_base[tid] = run ? atomicAdd(total, run) : 0u;
    }
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1ull;
    for (uint32_t d = 0; d < G; ++d) {
        const bool on = (m >> d) & 1u;
        const unsigned long long b = __ballot(on);
        const uint32_t k = s_base[d] + s_off[wave][d] + (uint32_t)__popcll(b & below);
        if (on && k < P.route_cap) {
            int4* e = reinterpret_cast<int4*>(P.route_out + (size_t)d * block + sizeof(RouteHeader) + (size_t)k * sizeof(RouteEntry));
            const int4* q = reinterpret_cast<const int4*>(&rec);
            e[0] = q[0];
            e[1] = q[1];
            e[2] = make_int4((int)box.bb0, (int)box.bb1, (int)gid, 0);
        }
    }
}

// XCD-aware tile order.  Blocks are dealt round-robin over the 8 XCDs, so blocks b
// and b + 8 share an XCD and its L2 (MI355X_MICROARCH.md; affinity only, nothing
// depends on it).  Runs of ZR_XCD_TILES consecutive (row-major) tiles go to one
// XCD, the runs round-robin over the XCDs: a primitive straddling two tiles of a
// run has its record and vertices read through one L2, and a dense screen region
// still spreads over every XCD.  A bijection: blocks past the last whole round of
// runs keep their own tile.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
    constexpr uint32_t K = ZR_XCD_TILES;
    if (K <= 1u || b >= n / (8u * K) * (8u * K)) return b;
    const uint32_t x = b & 7u, l = b >> 3;
    return ((l / K) * 8u + x) * K + l % K;
}

// The inverse of xcd_tile: the block that takes tile t in that order.
__device__ __forceinline__ uint32_t xcd_block(uint32_t t, uint32_t n) {
    constexpr uint32_t K = ZR_XCD_TILES;
    if (K <= 1u || t >= n / (8u * K) * (8u * K)) return t;
    const uint32_t R = t / K, o = t - R * K;
    return ((R >> 3) * K + o) * 8u + (R & 7u);
}

// Tile schedule (longest-processing-time first): built by the last k_setup_bin
// workgroup past phase 2, when every tile's count is final.  Each tile keeps the
// XCD xcd_tile gives it (block % 8), but within an XCD the blocks take its tiles
// heaviest list first, so the hardware, which dispatches blocks in order as slots
// free up, starts the long tiles first and ends the pass on short ones (the
// pass has ~2 tiles per wave slot at C2; without it its last ~15 us ran at 0.77
// occupancy, docs/EXPERIMENTS.md).  Counting sort over kSchedBuckets weight
// classes per XCD (s_sched: 8 x kSchedBuckets words of LDS).
__device__ void build_tile_schedule(const DrawParams& P, uint32_t nt, uint32_t* s_sched, uint32_t* order) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 8u * kSchedBuckets; i += kSetupThreads) s_sched[i] = 0u;
    const uint32_t top = __hip_atomic_fetch_max(&P.counters[kCtMaxTile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t shift = top >= kSchedBuckets ? 32u - __clz(top / kSchedBuckets) : 0u;  // top >> shift < 64
    __syncthreads();
    auto key = [&](uint32_t t, uint32_t& x) {  // XCD and descending-weight bucket of tile t
        const uint32_t c = __hip_atomic_fetch_add(&P.tile_counts[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kCountRuns;
        x = xcd_block(t, nt) & 7u;
        return kSchedBuckets - 1u - min(c >> shift, kSchedBuckets - 1u);
    };
    for (uint32_t t = tid; t < nt; t += kSetupThreads) {
        uint32_t x;
        const uint32_t k = key(t, x);
        atomicAdd(&s_sched[x * kSchedBuckets + k], 1u);
    }
    __syncthreads();
    if (tid < 8u * 64u) {  // one wave per XCD: exclusive scan of its 64 buckets
        static_assert(kSchedBuckets == 64, "one lane per bucket");
        const uint32_t c = s_sched[tid];
        uint32_t inc = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if ((int)(tid & 63u) >= d) inc += y;
        }
        s_sched[tid] = inc - c;
    }
    __syncthreads();
    for (uint32_t t = tid; t < nt; t += kSetupThreads) {
        uint32_t x;
        const uint32_t k = key(t, x);
        const uint32_t l = atomicAdd(&s_sched[x * kSchedBuckets + k], 1u);  // rank of t within its XCD
        order[l * 8u + x] = t;  // block l * 8 + x runs on XCD x (a bijection on [0, nt))
    }
}

// Tile jobs (DrawParams::job_entries), built by the same last workgroup.  A
// tile whose list is longer than J (and takes no record scan) becomes
// K = ceil(count / J) jobs, part p covering list entries [p J, (p + 1) J), with
// K key buffers from job_slot[t].  Part 0 keeps the tile's block in the usual
// order (blocks [job_pad, job_pad + nt)); parts 1.. take blocks of [0, job_pad)
// spread like their tile (block b % 8 = the tile's XCD in that order, for L2
// locality only); the blocks of [0, job_pad) left over get kJobNone.  (Every
// part among the first blocks, part 0 included, measured slower on c2x: 167.7 ->
// 172.0 us per frame, docs/EXPERIMENTS.md round 6.)  When the
// parts do not fit (an XCD's share of job_pad, or the key buffers) no tile is
// split and the draw is counted (kCtJobsDenied) for the runtime to size them up.  k_tile derives K from the
// same count and run word.
__device__ uint32_t tile_jobs(uint32_t count, uint32_t run_word, uint32_t J) {
    return (J && !(run_word & kRunDropped) && count > J) ? (count + J - 1u) / J : 1u;
}

__device__ __noinline__ void build_job_schedule(const DrawParams& P, uint32_t nt, uint32_t* s_buf) {
    const uint32_t tid = threadIdx.x, J = P.job_entries, per_xcd = P.job_pad / 8u;
    uint32_t* s_cnt = s_buf;       // [8] parts per XCD, then their cursors
    uint32_t* s_tot = s_buf + 8;   // [0] key buffers (jobs of split tiles), [1] buffer cursor, [2] denied, [3] split tiles
    if (tid < 16u) s_buf[tid] = 0u;
    __syncthreads();
    // pass 1: every tile's job count, kept in this thread's registers for pass 2
    // (tiles tid + k * kSetupThreads), and the parts each XCD gets; loads in
    // batches of kB in flight together (one tile at a time, and the counts parked
    // in job_slot and read back, kept this last workgroup ~11 us at 8160 tiles;
    // all 16 at once took 120 VGPRs, which every k_setup_bin instance reserves)
    constexpr uint32_t kPer = kMaxTilesPerPass / kSetupThreads, kB = 4;
    uint32_t K[kPer];
#pragma unroll
    for (uint32_t k0 = 0; k0 < kPer; k0 += kB) {
        uint32_t c[kB], rw[kB];
        if (tid + k0 * kSetupThreads >= nt) {
#pragma unroll
            for (uint32_t k = 0; k < kB; ++k) K[k0 + k] = 1u;
            continue;
        }
#pragma unroll
        for (uint32_t k = 0; k < kB; ++k) {
            const uint32_t t = tid + (k0 + k) * kSetupThreads;
            c[k] = t < nt ? __hip_atomic_load(&P.tile_counts[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kB; ++k) {
            const uint32_t t = tid + (k0 + k) * kSetupThreads;
            rw[k] = (c[k] & kCountRuns) ? __hip_atomic_load(&P.run_counts[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kB; ++k) {
            const uint32_t t = tid + (k0 + k) * kSetupThreads;
            K[k0 + k] = t < nt ? tile_jobs(c[k] & ~kCountRuns, rw[k], J) : 1u;
            if (K[k0 + k] > 1u) {
                atomicAdd(&s_cnt[xcd_block(t, nt) & 7u], K[k0 + k] - 1u);
                atomicAdd(&s_tot[0], K[k0 + k]);
                atomicAdd(&s_tot[3], 1u);
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        bool ok = s_tot[0] <= P.job_slots;
        uint32_t xmax = 0;
        for (uint32_t x = 0; x < 8u; ++x) {
            ok = ok && s_cnt[x] <= per_xcd;
            xmax = max(xmax, s_cnt[x]);
        }
        // what the split needs, fitting or not (the runtime sizes the shape's next
        // draws from it: key buffers and spare blocks per XCD)
        P.counters[kCtJobBufs] = s_tot[0];
        P.counters[kCtJobXcdMax] = xmax;
        s_tot[2] = ok ? 0u : 1u;
        P.draw_info[kInfoJobEntries] = ok ? J : 0u;
        if (!ok) atomicAdd(&P.counters[kCtJobsDenied], 1u);
    }
    __syncthreads();
    const bool ok = s_tot[2] == 0u;
    if (tid < 8u) {
        s_cnt[16 + tid] = ok ? s_cnt[tid] : 0u;  // (parts per XCD; s_cnt[0, 8) become the cursors)
        s_cnt[tid] = 0u;
    }
    if (tid == 0 && ok && s_tot[0]) atomicAdd(&P.counters[kCtJobs], s_tot[0] - s_tot[3]);  // (jobs beyond one per tile)
    __syncthreads();
    // pass 2: key slots (k_tile reads job_slot[t] of split tiles only) and part items
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t t = tid + k * kSetupThreads;
        if (!ok || K[k] <= 1u) continue;
        const uint32_t x = xcd_block(t, nt) & 7u;
        P.job_slot[t] = atomicAdd(&s_tot[1], K[k]);  // (K key buffers, one per job)
        const uint32_t l0 = atomicAdd(&s_cnt[x], K[k] - 1u);
        for (uint32_t p = 1; p < K[k]; ++p) P.tile_order[(l0 + p - 1u) * 8u + x] = t | (p << kJobTileBits);
    }
    for (uint32_t i = tid; i < P.job_pad; i += kSetupThreads)  // the spare part blocks
        if ((i >> 3) >= s_cnt[16 + (i & 7u)]) P.tile_order[i] = kJobNone;
    __syncthreads();  // (s_buf is build_tile_schedule's next)
}

// ----------------------------------------------------------- k_setup_bin
//
// One launch, one 1024-thread workgroup per CU (fewer for small draws), no grid
// barrier (workgroups never wait for each other, so nothing assumes they are
// co-resident):
//   phase 1  vertex stage + setup in units of 64 * KB * rounds primitives, one
//            wave per unit (units assigned statically); records and tile bboxes
//            to HBM (bboxes also to LDS when they fit), pairs counted in an LDS
//            histogram of all tiles
//   phase 2  the histogram is added into the global per-tile counters with
//            returning atomics (a wave's adds to consecutive tiles leave L2 as
//            64-B requests); the value returned is this workgroup's offset inside
//            the tile's list
//   phase 4  scatter the workgroup's (tile, primitive) pairs straight into the
//            tile's slab: tile t's list starts at bins[t * slab], so a list
//            start needs no scan of the totals (the round-1 design's grid
//            barrier + phase 3 scan cost ~6 us of a C2 frame).  A workgroup's
//            pairs that do not fit the rest of the slab go to a pool run
//            (pool_run); a run the pool cannot hold is dropped and counted:
//            k_tile rasterizes that tile exactly by scanning every record's
//            bbox, and the runtime grows the bin buffer at the next sync point
//            (DESIGN.md §4).
// Order inside a tile's list is arbitrary (whatever order the atomics returned),
// which is free: visibility keys carry the primitive sequence (k_tile).  The
// counters return to zero in k_tile, so a draw needs no memset.
#define ZR_STAMP(i)                                                                         \
    do {                                                                                    \
        if ((P.debug & kDebugStamps) && tid == 0) P.dbg_ts[w * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// Phase 2's overflow run (DrawParams::runs): this workgroup's c pairs for tile t,
// reserved at offset o (ov: the count the atomic returned) of the tile's list, do not fit the rest of its slab; they
// go to the pool.  The run takes slot w (this workgroup) of t's run table and an
// offset inside the workgroup's pool allocation (an LDS counter, s_pool[0]); the
// allocation itself is one atomic per workgroup after the tile loop
// (pool_commit), which turns the returned kPoolPending | offset into the run's
// bin position.  No returning global atomic per run: one per run on the pool
// counter queued the clustered c2x scene's ~31k runs on that address (setup
// 772 us), and a slot counter per tile cost cerberus' ~100 runs ~4 us of setup.
// Returns kDropCursor for a workgroup beyond the run table (run_cap).
constexpr uint32_t kPoolPending = 0x40000000u;
__device__ __noinline__ uint32_t pool_run(const DrawParams& P, uint32_t t, uint32_t ov, uint32_t c, uint32_t* s_pool,
                                          uint32_t w) {
    if (!(ov & kCountRuns)) atomicOr(&P.tile_counts[t], kCountRuns);  // (the first run of the tile, as far as this workgroup saw)
    const uint32_t o = ov & ~kCountRuns;
    if (o < P.slab) atomicOr(&P.run_counts[t], kRunFill | (o << kRunFillShift));  // the slab holds [0, o) of the list
    if (w >= P.run_cap) {
        atomicOr(&P.run_counts[t], kRunDropped);
        return kDropCursor;
    }
    P.runs[(size_t)t * P.run_cap + w].y = c;  // (the position once the workgroup's allocation is known)
    atomicAdd(&s_pool[1], 1u);
    return kPoolPending | atomicAdd(&s_pool[0], c);
}

// After phase 2's tile loop: the workgroup's pool runs take one allocation of
// s_pool[0] entries from its sub-pool (pool_subs); each pending cursor becomes its
// run's position, or kDropCursor (and the tile's kRunDropped) when the sub-pool is
// full.
__device__ __forceinline__ uint32_t pool_subs(const DrawParams& P) { return min(kPoolSubs, max(P.setup_wgs, 1u)); }

// The pool is kPoolSubs regions of pool_cap / subs entries (the remainder unused),
// region k the bump allocator of workgroups w % subs: one allocator for all 256
// workgroups queued their returning atomics on one word (c2x: phase 2 +8.7 us on
// average, the last workgroup's ticket 22 us late).  A workgroup's draw is a
// random sample of the primitives, so the regions fill alike; k_tile reports subs
// x the fullest region's requests as the pool the draw needs.
__device__ __noinline__ void pool_commit(const DrawParams& P, uint32_t* s_hist, uint32_t* s_pool, uint32_t rot,
                                         uint32_t w) {
    const uint32_t nt = P.ntiles, tid = threadIdx.x;
    if (tid == 0) {
        const uint32_t subs = pool_subs(P), k = w % subs, size = P.pool_cap / subs;
        const unsigned long long base = atomicAdd(
            reinterpret_cast<unsigned long long*>(&P.counters[kCtPoolSub0 + k * kCtSpread]), (unsigned long long)s_pool[0]);
        s_pool[2] = base + s_pool[0] <= size ? P.pool_off + k * size + (uint32_t)base : kDropCursor;
        atomicAdd(&P.counters[kCtPoolRuns], s_pool[1]);
    }
    __syncthreads();
    const uint32_t pb = s_pool[2];
    for (uint32_t i = tid; i < nt; i += kSetupThreads) {
        const uint32_t t = i + rot < nt ? i + rot : i + rot - nt;
        const uint32_t v = s_hist[t];
        if ((v >> 30) != 1u) continue;  // not pending
        if (pb != kDropCursor) {
            const uint32_t x = pb + (v & ~kPoolPending);
            P.runs[(size_t)t * P.run_cap + w].x = x;
            s_hist[t] = x;
        } else {
            atomicOr(&P.run_counts[t], kRunDropped);
            s_hist[t] = kDropCursor;
        }
    }
}

// i-th unit of primitives owned by workgroup w: interleaved (unit u -> workgroup
// u mod G), so every workgroup streams from the whole input at once (contiguous
// blocks per workgroup measured slower: C4 setup 286 vs 339 us).
__device__ __forceinline__ uint32_t own_unit(uint32_t w, uint32_t G, uint32_t i) { return w + i * G; }

template <uint32_t KB, bool MESH>
__global__ __launch_bounds__(kSetupThreads) void k_setup_bin(DrawParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_lds[];  // [ntiles (16-B padded) + kSetupMiscWords] + bboxes
    const uint32_t nt = P.ntiles, G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
    uint32_t* s_hist = s_lds;                       // histogram -> cursors
    uint32_t* s_misc = s_hist + ((nt + 3u) & ~3u);  // [32]
    uint32_t* s_pre = s_misc + 32;       // records mode: exclusive prefix of the received blocks' counts
    uint32_t* s_sched = s_misc + 96;     // [8 x kSchedBuckets] the tile schedule (last workgroup)
    // this workgroup's primitives' tile bboxes, indexed like phase 4's flattened
    // (own unit, primitive in unit) space, when they fit (P.bbox_lds)
    BBox* s_bbox = reinterpret_cast<BBox*>(s_misc + kSetupMiscWords);
    // phase 4's staging (P.bin_stage): per-tile local cursors, then (bin position,
    // entry) pairs grouped by tile
    uint32_t* s_lcur = reinterpret_cast<uint32_t*>(s_bbox + P.bbox_lds);
    uint2* s_stage = reinterpret_cast<uint2*>(s_lcur + ((nt + 3u) & ~3u));
    ZR_STAMP(0);
    for (uint32_t t = tid; t < nt; t += kSetupThreads) s_hist[t] = 0;
    if (tid < 32) s_misc[tid] = 0;
    // Partitioned draws (records mode): the received blocks' counts, and whether
    // any block overflowed -- then this workgroup, like every other (they all read
    // the same headers), sets up every primitive of the draw instead.
    if (P.rlist && tid < 64) {  // one lane per source block (G <= 32): the headers' loads in flight together
        const uint32_t src = tid;
        uint32_t total = 0;
        if (src < P.shard_count)
            total = reinterpret_cast<const RouteHeader*>(P.rlist + (size_t)src * route_block_bytes(P.route_cap))->total;
        const uint32_t cnt = min(total, P.route_cap);
        uint32_t inc = cnt, top = total;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if ((int)tid >= d) inc += y;
            top = max(top, (uint32_t)__shfl_xor((int)top, d, 64));
        }
        if (src <= P.shard_count) s_pre[src] = inc - cnt;  // exclusive prefix; s_pre[G] = all entries
        const bool over = __ballot(total > cnt) != 0ull;
        if (tid == 0) s_misc[4] = over ? 0u : 1u;
        if (tid == 0 && w == 0) {  // the draw's route statistics (one writer: workgroup 0)
            volatile uint32_t* st = P.status;
            if (over) st[kStRouteFallback] += 1u;
            if (top > st[kStRouteMax]) st[kStRouteMax] = top;
        }
    }
    __syncthreads();
    // This rank's own send headers are k_route's counters: the exchange has
    // consumed them (it precedes this kernel on the setup stream), so they are
    // zeroed here for the next route into this scratch set.
    if (P.rlist && w == 0 && tid < P.shard_count)
        reinterpret_cast<RouteHeader*>(P.route_out + (size_t)tid * route_block_bytes(P.route_cap))->total = 0u;
    const bool rec_mode = s_misc[4] != 0u;
    // setup records: the draw's primitives, or (records mode) the dense positions
    // of the received entries, in units of 2^unit_shift
    const uint32_t n_pos = rec_mode ? min(s_pre[P.shard_count], P.prims) : P.rlist ? P.draw_prims : P.prims;
    const uint32_t units = rec_mode || P.rlist ? (n_pos + (1u << P.unit_shift) - 1u) >> P.unit_shift : P.units;
    // records k_tile's overflow scan covers, and how their bboxes are indexed
    if (w == 0 && tid == 0) {
        P.draw_info[kInfoRecords] = MESH ? kMeshFans * n_pos : n_pos;
        P.draw_info[kInfoByPosition] = rec_mode ? 1u : 0u;
        // (kInfoJobEntries: build_job_schedule's alone.  A store of 0 here raced with
        // it -- plain stores of two workgroups, possibly in two XCDs' L2s, written
        // back at the kernel's end in either order -- and k_tile reads it only for
        // draws with tile jobs, whose schedule always writes it.)
    }

    // ---- phase 1
    int nvalid = 0, ndropped = 0, nmicro = 0;
    if (rec_mode) {  // the received entries: records stored at their draw ids, bboxes counted
        const DrawParams& P = kernarg_params();
        const uint32_t lane = tid & 63u, wave = tid >> 6;
        const uint32_t usz = 1u << P.unit_shift;
        for (uint32_t i = 0;; ++i) {
            const uint32_t u = own_unit(w, G, wave + i * (kSetupThreads / 64u));
            if (u >= units) break;
            const uint32_t jw = wave + i * (kSetupThreads / 64u);  // own-unit ordinal
            for (uint32_t r = lane; r < usz; r += 64u) {
                const uint32_t pos = (u << P.unit_shift) + r;
                if (pos >= n_pos) break;
                uint32_t gid;
                const BBox box = receive_entry(P, s_pre, pos, s_hist, nvalid, ndropped, gid);
                P.gids[pos] = gid;
                P.bboxes[pos] = box;
                if (P.bbox_lds) s_bbox[(jw << P.unit_shift) + r] = box;
            }
        }
    } else {
        const DrawParams& P = kernarg_params();  // phase 1's own loads of the parameters (SGPR pressure)
        const uint32_t lane = tid & 63u, wave = tid >> 6;
        const uint32_t rounds = (1u << P.unit_shift) / (64u * KB);
        for (uint32_t i = 0;; ++i) {
            const uint32_t u = own_unit(w, G, wave + i * (kSetupThreads / 64u));
            if (u >= units) break;
            const uint32_t jw = wave + i * (kSetupThreads / 64u);  // own-unit ordinal
            for (uint32_t r = 0; r < rounds; ++r) {
                const uint32_t pb = (u << P.unit_shift) + r * 64u * KB + lane;
                const uint32_t lb = (jw << P.unit_shift) + r * 64u * KB + lane;
                PrimIn in[KB];
#pragma unroll
                for (uint32_t b = 0; b < KB; ++b) fetch_indices(P, pb + b * 64u, n_pos, in[b]);
#pragma unroll
                for (uint32_t b = 0; b < KB; ++b) fetch_positions(P, in[b]);
#pragma unroll
                for (uint32_t b = 0; b < KB; ++b) {
                    const uint32_t prim = pb + b * 64u;
                    if (prim >= n_pos) continue;
                    BBox box;
                    if constexpr (MESH)
                        box = setup_finish_mesh(P, prim, in[b], s_hist, nvalid, ndropped);
                    else
                        box = setup_finish(P, prim, in[b], s_hist, nvalid, ndropped, nmicro);
                    // global: the overflow scan of any tile may need it; LDS: phase 4
                    P.bboxes[prim] = box;
                    if (P.bbox_lds) s_bbox[lb + b * 64u] = box;
                }
            }
        }
    }
    if (nvalid) atomicAdd(&s_misc[0], (uint32_t)nvalid);
    if (ndropped) atomicAdd(&s_misc[1], (uint32_t)ndropped);
    if (nmicro) atomicAdd(&s_misc[6], (uint32_t)nmicro);
    __syncthreads();
    ZR_STAMP(1);
    if (P.debug & kDebugPhase1Only) return;

    // ---- phase 2: reserve this workgroup's slots in every tile's list; the
    // cursor of tile t becomes t * slab + the offset the atomic returned.  Each
    // workgroup starts at a different 64-tile block so that the workgroups' adds
    // spread over the counter lines instead of all queueing on the same ones.
    {
        const DrawParams& P = kernarg_params();
        const uint32_t rot = nt ? ((w * 64u) % nt) : 0u;
        uint32_t top = 0, sum = 0;  // the largest tile count this workgroup saw, its pairs
        for (uint32_t i = tid; i < nt; i += kSetupThreads) {
            const uint32_t t = i + rot < nt ? i + rot : i + rot - nt;
            const uint32_t c = s_hist[t];
            const uint32_t ov = c ? __hip_atomic_fetch_add(&P.tile_counts[t], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            const uint32_t o = ov & ~kCountRuns;
            s_hist[t] = o + c <= P.slab ? t * P.slab + o : pool_run(P, t, ov, c, s_misc + 8, w);
            if (P.bin_stage) s_lcur[t] = c;
            top = max(top, o + c);
            sum += c;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            top = max(top, (uint32_t)__shfl_xor((int)top, o, 64));
            sum += (uint32_t)__shfl_xor((int)sum, o, 64);
        }
        if ((tid & 63u) == 0) {
            if (top) atomicMax(&s_misc[2], top);
            if (sum) atomicAdd(&s_misc[3], sum);
        }
        __syncthreads();
        if (tid == 0) {
            if (s_misc[0]) atomicAdd(&P.counters[kCtSetup], s_misc[0]);
            if (s_misc[1]) atomicAdd(&P.counters[kCtDropped], s_misc[1]);
            if (s_misc[6]) atomicAdd(&P.counters[kCtMicro], s_misc[6]);
            if (s_misc[2]) atomicMax(&P.counters[kCtMaxTile], s_misc[2]);
            if (s_misc[3]) atomicAdd(reinterpret_cast<unsigned long long*>(&P.counters[kCtPairs]), (unsigned long long)s_misc[3]);
        }
        if (s_misc[8]) {  // (the barrier above: every pool_run of this workgroup is done)
            pool_commit(P, s_hist, s_misc + 8, rot, w);
            __syncthreads();
        }
        if (P.tile_order) {  // (the tile schedule and / or tile jobs)
            // The last workgroup to take a ticket sees every tile's final count: the
            // counts and the max are only ever changed by atomics, which execute at
            // the memory side, and every one of this workgroup's has completed before
            // its ticket (returned, or drained by the wait below); the schedule reads
            // them back with atomics too, so no L2 holds a stale copy in between.
            // Tickets in two levels: a workgroup takes one in its group of
            // kTicketGroup (w / kTicketGroup, a word of its own), the group's last
            // one a ticket of the groups; the last group's last workgroup builds.
            // (One word for all 256 queued their returning atomics on it.)  The
            // chain keeps the order argument: every workgroup's atomics precede its
            // group ticket, which precedes its group's ticket of the groups.
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                const uint32_t g = w / kTicketGroup, gsize = min(kTicketGroup, G - g * kTicketGroup);
                const uint32_t gt = __hip_atomic_fetch_add(&P.counters[kCtTicketGroup0 + g * kCtSpread], 1u,
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint32_t last = 0u;
                if (gt == gsize - 1u)
                    last = __hip_atomic_fetch_add(&P.counters[kCtSchedTicket], 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) == (G + kTicketGroup - 1u) / kTicketGroup - 1u;
                s_misc[5] = last;
            }
            __syncthreads();
            if (s_misc[5]) {
                if (P.job_entries) build_job_schedule(P, nt, s_sched);
                if (P.tile_sched) build_tile_schedule(P, nt, s_sched, P.tile_order + (P.job_entries ? P.job_pad : 0u));
            }
        }
    }
    ZR_STAMP(2);
    if (!P.bbox_lds || rec_mode) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // phase 4 reads global bboxes / gids
    __syncthreads();

    // ---- phase 4: scatter the pairs of this workgroup's units, flattened over
    // (own unit, primitive in unit) so every thread has work
    {
        const DrawParams& P = kernarg_params();
        const uint32_t usz = 1u << P.unit_shift;
        // appends (tile, record) pairs of one setup record to its owned tiles' slabs
        // (the parameters the loops use, read once: kernarg_params() would reload them
        // per iteration)
        uint32_t* const bins = P.bins;
        const uint32_t sG = P.shard_count, srank = P.shard_rank, tiles_x = P.tiles_x;
        const uint32_t full_rows = P.full_rows, own_rows = P.own_rows, left_lo = P.left_lo, left_hi = P.left_hi;
        const uint32_t tsh = P.tile_shift;
        const int tl = 1 << tsh;
        auto scatter = [&](uint32_t rec, const BBox bb) {
            if (bb.bb0 == kEmptyBox) return;
            const int tx0 = (int)(bb.bb0 & 0xFFFFu) >> tsh, tx1 = (int)(bb.bb1 & 0xFFFFu) >> tsh;
            const int ty0 = (int)(bb.bb0 >> 16) >> tsh, ty1 = (int)(bb.bb1 >> 16) >> tsh;
            for_owned_tiles(sG, srank, tiles_x, full_rows, own_rows, left_lo, left_hi, tx0, ty0, tx1, ty1,
                            [&](uint32_t t, int tx, int ty) {
                const int cy0 = max((int)(bb.bb0 >> 16), ty << tsh);
                const int cy1 = min((int)(bb.bb1 >> 16), (ty << tsh) + tl - 1);
                const int cx0 = max((int)(bb.bb0 & 0xFFFFu), tx << tsh);
                const int cx1 = min((int)(bb.bb1 & 0xFFFFu), (tx << tsh) + tl - 1);
                // cost class: the lane walk's pair steps over bbox ∩ tile, ceil(w / 2)
                // per row (sorting by steps instead of area: C3 tile pass -1 %, C2 -0.8 %)
                const uint32_t steps = (uint32_t)(((cx1 - cx0 + 2) >> 1) * (cy1 - cy0 + 1));
                const uint32_t bucket = min((steps - 1u) >> 1, kSortBuckets - 1u);
                const uint32_t pos = atomicAdd(&s_hist[t], 1u);
                if (pos < 0x80000000u) bins[pos] = rec | (bucket << kBinPrimBits);  // (not a dropped run)
            });
        };
        uint32_t nown = 0;
        while (own_unit(w, G, nown) < units) ++nown;
        // Staged (the workgroup's pairs fit P.bin_stage): the pairs go to LDS grouped
        // by tile -- local offsets from an exclusive scan of this workgroup's
        // per-tile counts -- with their bin positions, and are then stored in that
        // order, so the lanes of a store instruction write a tile's run side by
        // side (one request per run and line instead of one per pair).
        const uint32_t npairs = s_misc[3];
        const bool staged = P.bin_stage && npairs <= P.bin_stage;
        if (staged) {
            const uint32_t per = (nt + kSetupThreads - 1u) / kSetupThreads;
            const uint32_t t0 = min(tid * per, nt), t1 = min(t0 + per, nt);
            uint32_t sum = 0;
            for (uint32_t t = t0; t < t1; ++t) sum += s_lcur[t];
            uint32_t inc = sum;  // exclusive scan of the threads' sums: waves, then the 16 wave totals
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(inc, d, 64);
                if ((int)(tid & 63u) >= d) inc += y;
            }
            if ((tid & 63u) == 63u) s_misc[16 + (tid >> 6)] = inc;
            __syncthreads();
            uint32_t base = 0;
            for (uint32_t q = 0; q < (tid >> 6); ++q) base += s_misc[16 + q];
            uint32_t run = base + inc - sum;
            for (uint32_t t = t0; t < t1; ++t) {
                const uint32_t c = s_lcur[t];
                s_lcur[t] = run;   // the tile's local cursor
                s_hist[t] -= run;  // bin position - local slot
                run += c;
            }
            __syncthreads();
        }
        auto scatter_staged = [&](uint32_t rec, const BBox bb) {
            if (bb.bb0 == kEmptyBox) return;
            const int tx0 = (int)(bb.bb0 & 0xFFFFu) >> tsh, tx1 = (int)(bb.bb1 & 0xFFFFu) >> tsh;
            const int ty0 = (int)(bb.bb0 >> 16) >> tsh, ty1 = (int)(bb.bb1 >> 16) >> tsh;
            for_owned_tiles(sG, srank, tiles_x, full_rows, own_rows, left_lo, left_hi, tx0, ty0, tx1, ty1,
                            [&](uint32_t t, int tx, int ty) {
                const int cy0 = max((int)(bb.bb0 >> 16), ty << tsh);
                const int cy1 = min((int)(bb.bb1 >> 16), (ty << tsh) + tl - 1);
                const int cx0 = max((int)(bb.bb0 & 0xFFFFu), tx << tsh);
                const int cx1 = min((int)(bb.bb1 & 0xFFFFu), (tx << tsh) + tl - 1);
                const uint32_t steps = (uint32_t)(((cx1 - cx0 + 2) >> 1) * (cy1 - cy0 + 1));
                const uint32_t bucket = min((steps - 1u) >> 1, kSortBuckets - 1u);
                const uint32_t l = atomicAdd(&s_lcur[t], 1u);
                const uint32_t pos = s_hist[t] + l;
                s_stage[l] = make_uint2(pos < 0x80000000u ? pos : 0xFFFFFFFFu, rec | (bucket << kBinPrimBits));
            });
        };
        for (uint32_t j = tid; staged && j < (nown << P.unit_shift); j += kSetupThreads) {
            const uint32_t prim = (own_unit(w, G, j >> P.unit_shift) << P.unit_shift) + (j & (usz - 1u));
            if (prim >= n_pos) continue;
            const BBox bb = P.bbox_lds ? s_bbox[j] : P.bboxes[prim];
            scatter_staged(rec_mode && bb.bb0 != kEmptyBox ? P.gids[prim] : prim, bb);
            if (MESH) {
                scatter_staged(mesh_record(P, prim, 1), P.bboxes[mesh_record(P, prim, 1)]);
                scatter_staged(mesh_record(P, prim, 2), P.bboxes[mesh_record(P, prim, 2)]);
            }
        }
        if (staged) {
            __syncthreads();
            for (uint32_t i = tid; i < npairs; i += kSetupThreads) {
                const uint2 v = s_stage[i];
                if (v.x != 0xFFFFFFFFu) bins[v.x] = v.y;
            }
        }
        for (uint32_t j = tid; !staged && j < (nown << P.unit_shift); j += kSetupThreads) {
            const uint32_t prim = (own_unit(w, G, j >> P.unit_shift) << P.unit_shift) + (j & (usz - 1u));
            if (prim >= n_pos) continue;
            const BBox bb = P.bbox_lds ? s_bbox[j] : P.bboxes[prim];
            scatter(rec_mode && bb.bb0 != kEmptyBox ? P.gids[prim] : prim, bb);
            if (MESH) {  // fans 1 and 2 (bboxes stored by this workgroup in phase 1)
                scatter(mesh_record(P, prim, 1), P.bboxes[mesh_record(P, prim, 1)]);
                scatter(mesh_record(P, prim, 2), P.bboxes[mesh_record(P, prim, 2)]);
            }
        }
    }
    ZR_STAMP(5);
}

// ------------------------------------------------------------------- k_tile

// T: the sRGB threshold table (LDS copy in k_tile).
__device__ __forceinline__ void store_color(const DrawParams& P, int px, int py, bool have, const float c[4],
                                            const float* T) {
    const size_t idx = (size_t)py * P.fb_w + (size_t)px;
    if (P.color_bpp == 4) {
        uint32_t* cp = (uint32_t*)P.color + idx;
        const uint32_t m = rgba8_write_mask(P.write_mask, P.color_format);
        if (have) {
            const uint32_t texel = pack_rgba8_fast(c, P.color_format, T);
            if (m == 0xFFFFFFFFu) {
                *cp = texel;
            } else {
                const uint32_t base = P.clear_color_enable ? P.clear_color_packed : *cp;
                *cp = (base & ~m) | (texel & m);
            }
        } else if (P.clear_color_enable) {
            *cp = P.clear_color_packed;
        }
    } else if (P.color_bpp == 16) {
        float4* cp = (float4*)P.color + idx;
        float4 v = P.clear_color_enable ? make_float4(P.clear_color[0], P.clear_color[1], P.clear_color[2],
                                                      P.clear_color[3])
                                        : *cp;
        if (have) {
            if (P.write_mask & 1u) v.x = c[0];
            if (P.write_mask & 2u) v.y = c[1];
            if (P.write_mask & 4u) v.z = c[2];
            if (P.write_mask & 8u) v.w = c[3];
        }
        if (have || P.clear_color_enable) *cp = v;
    }
}

__device__ __forceinline__ int rl(int v, uint32_t lane) { return __builtin_amdgcn_readlane(v, lane); }

// Rasterize one primitive (wave-uniform record) into the tile's LDS keys: lanes
// sweep the primitive's bbox ∩ tile, packed power-of-two rows per pass.
// Expands a compact record (two 16-B words, TriCompact) into the TriRecord fields
// the raster and resolve use: vertices, depth terms, |1/A2|, kFlagSmall/Swapped,
// and with `full` also the top-left bias flags and the clipped pixel bbox, computed
// exactly as k_setup_bin computed them.  v0..v2 are not part of the compact form.
// The top-left bias flags and the clipped pixel bbox of a record's vertices,
// computed exactly as k_setup_bin computed them.
__device__ __forceinline__ void finish_record(const DrawParams& P, TriRecord& r) {
    const int X[3] = {r.X0, r.X1, r.X2}, Y[3] = {r.Y0, r.Y1, r.Y2};
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // top-left rule (y-down), edge i opposite vertex i
        const int a = (i + 1) % 3, b = (i + 2) % 3;
        const int dx = X[b] - X[a], dy = Y[b] - Y[a];
        if (!((dy < 0) || (dy == 0 && dx > 0))) r.flags |= (kFlagBias0 << i);
    }
    const int minX = min(X[0], min(X[1], X[2])), maxX = max(X[0], max(X[1], X[2]));
    const int minY = min(Y[0], min(Y[1], Y[2])), maxY = max(Y[0], max(Y[1], Y[2]));
    const int px0 = max((minX - 128 + 255) >> 8, P.clip_x0), px1 = min((maxX - 128) >> 8, P.clip_x1);
    const int py0 = max((minY - 128 + 255) >> 8, P.clip_y0), py1 = min((maxY - 128) >> 8, P.clip_y1);
    r.bb0 = (uint32_t)px0 | ((uint32_t)py0 << 16);
    r.bb1 = (uint32_t)px1 | ((uint32_t)py1 << 16);
}

__device__ __forceinline__ TriRecord decode_compact(const DrawParams& P, const int4 q0, const int4 q1, bool full) {
    TriRecord r;
    r.X0 = q0.x; r.Y0 = q0.y;
    r.X1 = q0.x + (int)(int16_t)(q0.z & 0xFFFF); r.Y1 = q0.y + (q0.z >> 16);
    r.X2 = q0.x + (int)(int16_t)(q0.w & 0xFFFF); r.Y2 = q0.y + (q0.w >> 16);
    r.z0 = __int_as_float(q1.x); r.dz1 = __int_as_float(q1.y); r.dz2 = __int_as_float(q1.z);
    r.invA2 = fabsf(__int_as_float(q1.w));
    r.flags = kFlagSmall | ((q1.w < 0) ? kFlagSwapped : 0u);
    r.v0 = r.v1 = r.v2 = 0u;
    r.bb0 = r.bb1 = 0u;
    if (full) finish_record(P, r);
    return r;
}

// A compact record for the lane walk; for a large primitive (large: its compact
// record holds vertex 0, the depth terms and |1/A2|, the same values as its full
// record) with vertices 1 and 2 from records_big (X1, Y1, X2, Y2: bytes 8-23).
// Biases and bbox as setup computed them.
__device__ __forceinline__ TriRecord decode_large(const DrawParams& P, const int4 q0, const int4 q1, bool large,
                                                  const int2 v1, const int2 v2) {
    TriRecord r;
    r.X0 = q0.x; r.Y0 = q0.y;
    r.X1 = large ? v1.x : q0.x + (int)(int16_t)(q0.z & 0xFFFF); r.Y1 = large ? v1.y : q0.y + (q0.z >> 16);
    r.X2 = large ? v2.x : q0.x + (int)(int16_t)(q0.w & 0xFFFF); r.Y2 = large ? v2.y : q0.y + (q0.w >> 16);
    r.z0 = __int_as_float(q1.x); r.dz1 = __int_as_float(q1.y); r.dz2 = __int_as_float(q1.z);
    r.invA2 = fabsf(__int_as_float(q1.w));
    r.flags = (q1.w < 0) ? kFlagSwapped : 0u;
    r.v0 = r.v1 = r.v2 = 0u;
    finish_record(P, r);
    return r;
}

// Whether the lane walk (raster_lane) is exact for a large primitive in this
// tile: every edge value it tests, over bbox ∩ tile widened by the walk's
// kLaneStep - 1 columns on either side, must fit int32.  The edge functions are linear, so
// their extremes are at the rectangle's corners: |w| <= |w(corner)| + |dy| 256 W
// + |dx| 256 H, bounded in int64 against 2^31 - 1.
template <int TS>
__device__ __forceinline__ bool lane_walk_fits(const TriRecord& r, int x0, int y0) {
    constexpr int T = 1 << TS;
    const int bx0 = max((int)(r.bb0 & 0xFFFFu), x0) - (kLaneStep - 1), by0 = max((int)(r.bb0 >> 16), y0);
    const int bx1 = min((int)(r.bb1 & 0xFFFFu), x0 + T - 1) + (kLaneStep - 1);
    const int by1 = min((int)(r.bb1 >> 16), y0 + T - 1);
    const long long Sx = (long long)bx0 * 256 + 128, Sy = (long long)by0 * 256 + 128;
    const long long Wd = (long long)(bx1 - bx0) * 256, Hd = (long long)max(by1 - by0, 0) * 256;
    auto edge = [&](int Xa, int Ya, int Xb, int Yb) {
        const long long dx = (long long)Xb - Xa, dy = (long long)Yb - Ya;
        const long long w = dx * (Sy - Ya) - dy * (Sx - Xa);
        return llabs(w) + llabs(dy) * Wd + llabs(dx) * Hd;
    };
    const long long m = max(edge(r.X1, r.Y1, r.X2, r.Y2), max(edge(r.X2, r.Y2, r.X0, r.Y0), edge(r.X0, r.Y0, r.X1, r.Y1)));
    return m < 0x7FFFFFFFll;
}

// A wave-uniform full record, moved to scalar registers right after the load so
// the wave path does not hold 16 more VGPRs.
__device__ __forceinline__ TriRecord uniform_record(const int4 a, const int4 b, const int4 c, const int4 d) {
    auto u = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
    TriRecord r;
    r.X0 = u(a.x); r.Y0 = u(a.y); r.X1 = u(a.z); r.Y1 = u(a.w);
    r.X2 = u(b.x); r.Y2 = u(b.y);
    r.z0 = __int_as_float(u(b.z)); r.dz1 = __int_as_float(u(b.w));
    r.dz2 = __int_as_float(u(c.x)); r.invA2 = __int_as_float(u(c.y));
    r.v0 = (uint32_t)u(c.z); r.v1 = (uint32_t)u(c.w); r.v2 = (uint32_t)u(d.x);
    r.bb0 = (uint32_t)u(d.y); r.bb1 = (uint32_t)u(d.z); r.flags = (uint32_t)u(d.w);
    return r;
}

__device__ __forceinline__ TriRecord load_uniform_record(const TriRecord* p) {
    const int4* q = reinterpret_cast<const int4*>(p);
    return uniform_record(q[0], q[1], q[2], q[3]);
}


// Row sweeps raster_prim makes over a record's bbox ∩ tile (kDebugStamps).
template <int TS>
__device__ __forceinline__ uint32_t prim_sweeps(const TriRecord& r, int x0, int y0) {
    constexpr int T = 1 << TS;
    const int bw = min((int)(r.bb1 & 0xFFFFu), x0 + T - 1) - max((int)(r.bb0 & 0xFFFFu), x0) + 1;
    const int bh = min((int)(r.bb1 >> 16), y0 + T - 1) - max((int)(r.bb0 >> 16), y0) + 1;
    if (bw <= 0 || bh <= 0) return 0u;
    const int sh = bw <= 1 ? 0 : 32 - __clz(bw - 1);
    const int rows = 64 >> sh;
    return (uint32_t)((bh + rows - 1) / rows);
}

template <int MODE, bool INITD, int TS>
__device__ __forceinline__ void raster_prim(const DrawParams& P, const TriRecord& r, uint32_t seq, int x0, int y0,
                                            int lane, unsigned long long* s_key, const float* s_initd) {
    constexpr int T = 1 << TS;
    const int bx0 = max((int)(r.bb0 & 0xFFFFu), x0), by0 = max((int)(r.bb0 >> 16), y0);
    const int bx1 = min((int)(r.bb1 & 0xFFFFu), x0 + T - 1), by1 = min((int)(r.bb1 >> 16), y0 + T - 1);
    const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
    if (bw <= 0 || bh <= 0) return;
    const int sh = bw <= 1 ? 0 : 32 - __clz(bw - 1);
    const int rows = 64 >> sh;
    const int lx = lane & ((1 << sh) - 1), lyo = lane >> sh;
    const long long bias0 = (r.flags >> 1) & 1, bias1 = (r.flags >> 2) & 1, bias2 = (r.flags >> 3) & 1;
    const DepthPlane dp = depth_plane(r.z0, r.dz1, r.dz2, r.invA2, (int)bias1, (int)bias2);
    const float dlo = P.dlo, dhi = P.dhi;  // (held: a per-pass kernarg reload waits on the scalar cache)
    // The lane's biased edge values at its first pixel, then stepped by `rows`
    // pixel rows per pass in int64 (exact; a pass was two int64 products per edge.
    // Stepping in double measured slower: cerberus 48.5 -> 51.3 us)
    const EdgeEval e = eval_edges(r, bx0 + lx, by0 + lyo);
    long long w0 = e.w0 - bias0, w1 = e.w1 - bias1, w2 = e.w2 - bias2;
    const long long s0 = (long long)(r.X2 - r.X1) * (256 * rows), s1 = (long long)(r.X0 - r.X2) * (256 * rows);
    const long long s2 = (long long)(r.X1 - r.X0) * (256 * rows);
    for (int ry = 0; ry < bh; ry += rows) {
        const int ly = ry + lyo;
        if (lx < bw && ly < bh && (w0 | w1 | w2) >= 0) {
            const float z = plane_z(dp, (float)w1, (float)w2);
            if (z >= dlo && z <= dhi) {
                const int li = (by0 + ly - y0) * T + (bx0 + lx - x0);
                if (!INITD || depth_pass(P.depth_op, z, s_initd[li])) atomicMin(&s_key[li], frag_key<MODE>(z, seq));
            }
        }
        w0 += s0;
        w1 += s1;
        w2 += s2;
    }
}

// Lane-parallel path for small primitives (kFlagSmall): each lane walks its own
// primitive's bbox ∩ tile in row order, stepping the three edge functions
// incrementally in int32 (exact: |w| <= 2^29 inside a small primitive's bbox).
// With k = 2^ksh lanes per primitive (sparse tiles), lane `sub` of the
// primitive's group takes the bbox rows sub, sub + k, ...
template <int MODE, bool INITD, int TS>
__device__ __forceinline__ void raster_lane(const DrawParams& P, const TriRecord& r, uint32_t seq, int x0, int y0,
                                            unsigned long long* s_key, const float* s_initd, int sub, int ksh) {
    constexpr int T = 1 << TS;
    const int k = 1 << ksh;
    const int X0 = r.X0, Y0 = r.Y0, X1 = r.X1, Y1 = r.Y1, X2 = r.X2, Y2 = r.Y2;
    const float z0 = r.z0, dz1 = r.dz1, dz2 = r.dz2, invA2 = r.invA2;
    const uint32_t bb0 = r.bb0, bb1 = r.bb1, flags = r.flags;
    int bx0 = max((int)(bb0 & 0xFFFFu), x0);
    const int by0 = max((int)(bb0 >> 16), y0);
    const int bx1 = min((int)(bb1 & 0xFFFFu), x0 + T - 1), by1 = min((int)(bb1 >> 16), y0 + T - 1);
    int bw = bx1 - bx0 + 1;
    const int bh = by1 - by0 + 1;
    if (bw <= 0 || bh <= sub) return;
    // S pixels of a row per step (kLaneStep).  A row whose width is not a multiple
    // of S leaves samples of its last step past the bbox.  When the bbox's right
    // side is the primitive's own x extent (not cut by the tile or the scissor)
    // they lie right of every vertex, so they are never covered; else, when the
    // left side is its own extent, the steps start that many columns further left
    // (left of every vertex).  Only when both sides are cut does the step test
    // for them (chk: pixels j >= rem of the row's last step).
    constexpr int S = kLaneStep;
    bool chk = false;
    int rem = S;
    if (bw & (S - 1)) {
        const int minX = min(X0, min(X1, X2)), maxX = max(X0, max(X1, X2));
        if (bx1 != (maxX - 128) >> 8) {
            if (bx0 == (minX - 128 + 255) >> 8) {
                const int e = S - (bw & (S - 1));
                bx0 -= e;
                bw += e;
            } else {
                chk = true;
                rem = bw & (S - 1);
            }
        }
    }
    // Edge values and steps in arithmetic mod 2^32 (u32 products and sums): exact
    // wherever the true value fits int32, which holds at every sample the walk
    // tests -- a small primitive's |w| <= 2^29, a large one is sent here only when
    // lane_walk_fits bounds its values over bbox ∩ tile -- whatever the steps'
    // own magnitudes (a row wrap's jump may exceed int32; the sum it lands on does not).
    auto wr = [](uint32_t a) { return (int)a; };
    const int Sx = bx0 * 256 + 128, Sy = (by0 + sub) * 256 + 128;
    const uint32_t dx0 = X2 - X1, dy0 = Y2 - Y1, dx1 = X0 - X2, dy1 = Y0 - Y2, dx2 = X1 - X0, dy2 = Y1 - Y0;
    int r0 = wr(dx0 * (uint32_t)(Sy - Y1) - dy0 * (uint32_t)(Sx - X1));
    int r1 = wr(dx1 * (uint32_t)(Sy - Y2) - dy1 * (uint32_t)(Sx - X2));
    int r2 = wr(dx2 * (uint32_t)(Sy - Y0) - dy2 * (uint32_t)(Sx - X0));
    const int sx0 = wr(0u - dy0 * 256u), sx1 = wr(0u - dy1 * 256u), sx2 = wr(0u - dy2 * 256u);  // +1 pixel in x
    const int sy0 = wr(dx0 * 256u), sy1 = wr(dx1 * 256u), sy2 = wr(dx2 * 256u);                 // +1 pixel in y
    const int b0 = (int)((flags >> 1) & 1u), b1 = (int)((flags >> 2) & 1u), b2 = (int)((flags >> 3) & 1u);
    // Sweep the bbox in row order, stepping the edge values: +sx per pixel, and at
    // the end of a row the jump back to the next row's first pixel, chosen with
    // selects (no divergent branch: a nested row / column loop, or a wrap branch,
    // idles the lanes of narrower primitives and measured slower).  The top-left
    // bias is folded into the edge values, so coverage is one sign test, and the
    // depth plane is defined on the biased values (§3.6).  Fragment depth is never
    // -0 here: setup canonicalised the vertex depths to +0 (the oracle's
    // per-fragment -0 -> +0 rule therefore gives the same bits).  The sweep ends when the key address reaches the row after the
    // last one (no separate step counter).
    const int rows = (bh - sub + k - 1) >> ksh;
    int w0 = wr((uint32_t)r0 - b0), w1 = wr((uint32_t)r1 - b1), w2 = wr((uint32_t)r2 - b2);
    int ex = 0;
    uint32_t la = (uint32_t)(((by0 + sub - y0) * T + (bx0 - x0)) * 8);  // byte offset of the key
    const uint32_t la_end = la + (uint32_t)(rows * k * T * 8);
    // The depth-range test (fragments outside [dlo, dhi] are discarded, §3) is
    // dropped from the loop when every lane's vertex depths lie inside the range
    // by a margin far above the interpolation's rounding (a few ulp of 1): then
    // no fragment can fall outside.  NaN depths fail the comparisons, so keep it.
    const float z1v = z0 + dz1, z2v = z0 + dz2, zlo = P.dlo + 1e-4f, zhi = P.dhi - 1e-4f;
    const bool zsafe = z0 >= zlo && z0 <= zhi && z1v >= zlo && z1v <= zhi && z2v >= zlo && z2v <= zhi;
    // one covered sample: depth from the (un-biased) edge values, test, key
    const DepthPlane dp = depth_plane(z0, dz1, dz2, invA2, b1, b2);
    auto frag = [&](auto ztest, int e1, int e2, uint32_t a) {
        const float z = plane_z(dp, (float)e1, (float)e2);  // e1, e2: the biased values
        if ((!decltype(ztest)::value || (z >= P.dlo && z <= P.dhi)) &&
            (!INITD || depth_pass(P.depth_op, z, s_initd[a >> 3])))
            atomicMin(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(s_key) + a), frag_key<MODE>(z, seq));
    };
    // S pixels of a row per step (VALU and loop-control SALU are what the lane
    // walk spends: one step's wrap selects and branch bookkeeping serve S
    // samples).  Pixels j >= rem of a row's last step (index lastB) lie past a
    // bbox cut on both sides and are skipped.
    const int hw = (bw + S - 1) / S, lastB = chk ? hw - 1 : hw;
    const int t0 = wr((uint32_t)S * sx0), t1 = wr((uint32_t)S * sx1), t2 = wr((uint32_t)S * sx2);
    const uint32_t kk = (uint32_t)k, hh = (uint32_t)S * (uint32_t)(hw - 1);
    const int q0 = wr(kk * sy0 - hh * sx0), q1 = wr(kk * sy1 - hh * sx1), q2 = wr(kk * sy2 - hh * sx2);
    const uint32_t lq = (uint32_t)((k * T - S * (hw - 1)) * 8);
    auto sweep = [&](auto ztest, auto wchk) {
        do {
            int a0 = w0, a1 = w1, a2 = w2;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                if (j) {
                    a0 = wr((uint32_t)a0 + sx0);
                    a1 = wr((uint32_t)a1 + sx1);
                    a2 = wr((uint32_t)a2 + sx2);
                }
                if ((j == 0 || !decltype(wchk)::value || ex != lastB || j < rem) && (a0 | a1 | a2) >= 0)
                    frag(ztest, a1, a2, la + 8u * (uint32_t)j);
            }
            const bool wrap = ++ex == hw;
            ex = wrap ? 0 : ex;
            w0 = wr((uint32_t)w0 + (wrap ? q0 : t0));
            w1 = wr((uint32_t)w1 + (wrap ? q1 : t1));
            w2 = wr((uint32_t)w2 + (wrap ? q2 : t2));
            la += wrap ? lq : 8u * (uint32_t)S;
        } while (la != la_end);
    };
    const bool wchk = __ballot(chk) != 0ull;
    const bool wz = __ballot(!zsafe) != 0ull;
    if (!wz && !wchk)
        sweep(std::false_type{}, std::false_type{});
    else if (!wz)
        sweep(std::false_type{}, std::true_type{});
    else if (!wchk)
        sweep(std::true_type{}, std::false_type{});
    else
        sweep(std::true_type{}, std::true_type{});
}

// Visibility sequence of setup record e (API order): e + 1, or for the mesh
// program 4p + k + 1 for fan k of primitive p (zr_internal.h kMeshFans).
template <int PROG>
__device__ __forceinline__ uint32_t entry_seq(const DrawParams& P, uint32_t e) {
    if (PROG != kProgMesh) return e + 1u;
    if (e < P.prims) return 4u * e + 1u;
    const uint32_t q = e - P.prims;
    return 4u * (q >> 1) + (q & 1u) + 2u;
}
// ... and back: the setup record and the draw primitive of sequence s + 1.
template <int PROG>
__device__ __forceinline__ uint32_t seq_record(const DrawParams& P, uint32_t s) {
    if (PROG != kProgMesh) return s;
    const uint32_t p = s >> 2, k = s & 3u;
    return k ? P.prims + 2u * p + k - 1u : p;
}
template <int PROG>
__device__ __forceinline__ uint32_t seq_prim(uint32_t s) { return PROG == kProgMesh ? s >> 2 : s; }
template <int PROG>
__device__ __forceinline__ uint32_t record_prim(const DrawParams& P, uint32_t e) {
    return (PROG == kProgMesh && e >= P.prims) ? (e - P.prims) >> 1 : e;
}

template <int PROG>
__device__ __forceinline__ void shade_winner(const DrawParams& P, const TriRecord& r, const EdgeEvalF& e, float out[4]) {
    if (PROG == kProgFlat) {
        const float* c = attr_ptr(P, r.v0, 1);  // provoking vertex = first (flat)
        out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = 1.0f;
        return;
    }
    // perspective-correct weights b_i / w_i with w_i = 1 for every built-in vertex stage
    const float pw0 = e.f0 * r.invA2, pw1 = e.f1 * r.invA2, pw2 = e.f2 * r.invA2;
    const float inv = 1.0f / ((pw0 + pw1) + pw2);
    const float* a0 = attr_ptr(P, r.v0, 1);
    const float* a1 = attr_ptr(P, r.v1, 1);
    const float* a2 = attr_ptr(P, r.v2, 1);
    float f[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) f[i] = ((pw0 * a0[i] + pw1 * a1[i]) + pw2 * a2[i]) * inv;
    if (PROG == kProgTriangle) {
        const float t3 = (P.time_ptr ? *P.time_ptr : 0.0f) * 3.0f;
        out[0] = shade_triangle_channel(f[0], t3);
        out[1] = shade_triangle_channel(f[1], t3);
        out[2] = shade_triangle_channel(f[2], t3);
        out[3] = 1.0f;
        return;
    }
    const float* k0 = attr_ptr(P, r.v0, 2);
    const float* k1 = attr_ptr(P, r.v1, 2);
    const float* k2 = attr_ptr(P, r.v2, 2);
    float kd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) kd[i] = ((pw0 * k0[i] + pw1 * k1[i]) + pw2 * k2[i]) * inv;
    shade_blinn_phong(f[0], f[1], f[2], kd[0], kd[1], kd[2], out);
}

// mesh.slang psmain: perspective-correct barycentrics of the primitive (not of
// its clipped fan triangle) from its homogeneous screen vertices
// h_i = (x_i hw + w_i cx, y_i hh + w_i cy, w_i): b_i = E_i / sum E with
// E_i = p . (h_j x h_k) at the pixel centre (the planes setup stored,
// mesh_edge_planes); then normal and uv interpolated and lit like blinn_phong.slang with kd = (0.35 + 0.3 u, 0.35 + 0.3 v, 0.7)
// (zr_oracle.c shade, same operation order).
__device__ __forceinline__ void shade_mesh(const DrawParams& P, uint32_t prim, const uint32_t vid[3], int px, int py,
                                           float out[4]) {
    const float4* q = P.mesh_edges + (size_t)prim * 3u;
    const float4 qa = q[0], qb = q[1], qc = q[2];
    const float c[12] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w, qc.x, qc.y, qc.z, qc.w};
    float E[3];
    mesh_plane_eval(c, px, py, E);
    const float einv = 1.0f / ((E[0] + E[1]) + E[2]);
    const float b0 = E[0] * einv, b1 = E[1] * einv, b2 = E[2] * einv;
    const float* n0 = attr_ptr(P, vid[0], 1);
    const float* n1 = attr_ptr(P, vid[1], 1);
    const float* n2 = attr_ptr(P, vid[2], 1);
    const float* u0 = attr_ptr(P, vid[0], 2);
    const float* u1 = attr_ptr(P, vid[1], 2);
    const float* u2 = attr_ptr(P, vid[2], 2);
    float n[3], uv[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) n[i] = (b0 * n0[i] + b1 * n1[i]) + b2 * n2[i];
#pragma unroll
    for (int i = 0; i < 2; ++i) uv[i] = (b0 * u0[i] + b1 * u1[i]) + b2 * u2[i];
    shade_blinn_phong(n[0], n[1], n[2], fmaf(uv[0], 0.3f, 0.35f), fmaf(uv[1], 0.3f, 0.35f), 0.7f, out);
}

// Vertex ids of a winning primitive; IDX32: u32 index buffer (one 12-B load).
template <bool IDX32>
__device__ __forceinline__ void resolve_vids(const DrawParams& P, uint32_t prim, uint32_t v[3]) {
    if (IDX32) {
        const uint32_t tri = tri_of(P, prim);
        const uint3 ix = *reinterpret_cast<const uint3*>(P.ib + (uint64_t)(P.first + tri * 3u) * 4);
        const uint32_t off = (uint32_t)P.vertex_offset;
        v[0] = ix.x + off; v[1] = ix.y + off; v[2] = ix.z + off;
    } else {
        winner_vids(P, prim, v);
    }
}

// Record table of a 512-thread tile (LDS): the small primitives of its current
// segment, with the part of the compact record the resolve reads (vertex 0
// relative to the tile origin as int16 pairs, the deltas, +-1/A2), stored at the
// entry's sorted position j (no collisions), and a 2048-slot hash from the setup
// record to j + 1 (load factor <= 1/2: short probes).  A lookup is valid when the
// sorted array still holds that record at j (a later segment reuses positions).
// The raster inserts each entry as it loads it; the resolve looks its winners up
// and gathers the record only when that fails (a table overwritten by a later
// segment, a long probe, a large primitive).  A large primitive is not hashed, but
// its position's slot gets the large marker, so a stale hash slot an earlier
// segment left for that position decodes as large (records_big), never as the
// earlier segment's small record.  Every winner request the pass saves
// is worth ~20 ns of a C2 tile pass (docs/EXPERIMENTS.md).
constexpr uint32_t kRecHashSlots = 2048;
constexpr uint32_t kRecTabProbes = 8;
__device__ __forceinline__ uint32_t rec_hash(uint32_t rec) { return (rec * 0x9E3779B1u) >> 21; }  // 11 bits
// Vertex 0 of a small primitive (extents <= 64 px) whose bbox meets the tile lies
// within [-64 px, tile edge + 64 px) of the tile origin: stored as u16 offsets (24.8
// fixed point) from 64 px above-left of the origin.
constexpr int kRelBias = 64 * 256;
static_assert((64 + 128) * 256 <= 65536, "tile-relative vertex 0 fits u16 (tiles up to 64 px)");

__device__ __forceinline__ void rec_table_insert(uint32_t* s_thash, int4* s_trec, uint32_t rec, uint32_t j,
                                                 const int4 q0, const int4 q1, int x0, int y0) {
    const uint32_t rel = ((uint32_t)(q0.x - x0 * 256 + kRelBias) & 0xFFFFu) | ((uint32_t)(q0.y - y0 * 256 + kRelBias) << 16);
    s_trec[j] = make_int4((int)rel, q0.z, q0.w, q1.w);
    uint32_t h = rec_hash(rec);
    for (uint32_t p = 0; p < kRecTabProbes; ++p) {
        if (atomicCAS(&s_thash[h], 0u, j + 1u) == 0u) return;
        h = (h + 1u) & (kRecHashSlots - 1u);
    }
}

// The compact record words (q1: only 1/A2) of setup record `rec`.
__device__ __forceinline__ bool rec_table_find(const uint32_t* s_thash, const int4* s_trec, const uint32_t* s_sorted,
                                               uint32_t rec, int x0, int y0, int4& q0, int4& q1) {
    uint32_t h = rec_hash(rec);
    for (uint32_t p = 0; p < kRecTabProbes; ++p) {
        const uint32_t v = s_thash[h];
        if (v == 0u) return false;
        if (s_sorted[v - 1u] == rec) {
            const int4 e = s_trec[v - 1u];
            q0 = make_int4(x0 * 256 - kRelBias + (int)((uint32_t)e.x & 0xFFFFu), y0 * 256 - kRelBias + (int)((uint32_t)e.x >> 16),
                           e.y, e.z);
            q1 = make_int4(0, 0, 0, e.w);
            return true;
        }
        h = (h + 1u) & (kRecHashSlots - 1u);
    }
    return false;
}

// Per-pixel resolve (512-thread tiles: two pixels per thread, one batch): per
// pixel the winning primitive is read from its key, its compact record and vertex
// ids are gathered, its edges evaluated once and the program shaded once
// (deferred shading); colour and depth are stored.  The batch's gathers are in
// flight together, and a tile's records are still L2-resident from its raster
// phase.  Measured faster than resolve_tile at 512 threads (C2: ~78 vs 80-84 us:
// no barriers, two dependent round trips), slower at 256 threads (4 pixels per
// thread in two batches; C1 49 vs 44 us, C3 223 vs 204 us).  A wave with no
// winner skips the gathers; other pixels without a winner load the wave's first
// winner (in-bounds addresses) and discard it.
template <int PROG, int MODE, bool IDX32, int NT, bool TAB, int TS>
__device__ __forceinline__ void resolve_pixels(const DrawParams& P, int x0, int y0, const unsigned long long* s_key,
                                               const float* s_srgb, const uint32_t* s_thash, const int4* s_trec,
                                               const uint32_t* s_sorted) {
    constexpr int T = 1 << TS, TP = T * T;
    constexpr int kPer = TP / NT;
    constexpr int kB = kPer < (int)kResolveBatch ? kPer : (int)kResolveBatch;
    // recomputed here, not reused from the tile's init: a pixel coordinate kept
    // live across the raster loop spills at 64 VGPRs
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
#pragma unroll 1
    for (int k0 = 0; k0 < kPer; k0 += kB) {
        int px[kB], py[kB];
        bool have[kB], inside[kB];
        unsigned long long key[kB];
        uint32_t prim[kB], gp[kB], vid[kB][3];  // setup record, draw primitive, its vertex ids
        int4 c0[kB], c1[kB];
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const int i = tid + (k0 + b) * NT;
            px[b] = x0 + (i & (T - 1));
            py[b] = y0 + (i >> TS);
            inside[b] = !(px[b] < P.ra_x0 || px[b] > P.ra_x1 || py[b] < P.ra_y0 || py[b] > P.ra_y1);
            key[b] = s_key[i];
            const uint32_t seq = inside[b] ? winner_seq<MODE>(key[b]) : 0u;
            have[b] = seq != 0;
            prim[b] = have[b] ? seq_record<PROG>(P, seq - 1u) : 0u;
            gp[b] = have[b] ? seq_prim<PROG>(seq - 1u) : 0u;
        }
        if (P.win_bits) {  // winner census (profiling level 2 only; never in a timed pass)
#pragma unroll
            for (int b = 0; b < kB; ++b)
                if (have[b]) atomicOr(&P.win_bits[gp[b] >> 5], 1u << (gp[b] & 31u));
        }
        unsigned long long anyw = 0;
#pragma unroll
        for (int b = 0; b < kB; ++b) anyw |= __ballot(have[b]);
        if (anyw) {  // wave-uniform: some pixel of the wave has a winner, lend it to the others
            const int src = (int)__builtin_ctzll(anyw);
            uint32_t fb = 0, fg = 0;
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const unsigned long long hb = __ballot(have[b]);
                const uint32_t pb = (uint32_t)__builtin_amdgcn_readlane((int)prim[b], src);
                const uint32_t gb = (uint32_t)__builtin_amdgcn_readlane((int)gp[b], src);
                if (!fb && ((hb >> src) & 1ull)) { fb = pb + 1u; fg = gb; }
            }
#pragma unroll
            for (int b = 0; b < kB; ++b)
                if (!have[b]) { prim[b] = fb - 1u; gp[b] = fg; }
        }
        float col[kB][4];
        float zw[kB];
        if (anyw) {
#pragma unroll
            for (int b = 0; b < kB; ++b) {  // the index gathers first: the table lookups run under them
                if (tile_debug(P) & kDebugIdentityVids) {
                    const uint32_t v = P.first + tri_of(P, gp[b]) * 3u + (uint32_t)P.vertex_offset;
                    vid[b][0] = v; vid[b][1] = v + 1u; vid[b][2] = v + 2u;
                } else {
                    resolve_vids<IDX32>(P, gp[b], vid[b]);
                }
                if (tile_debug(P) & kDebugSameVids) vid[b][0] = vid[b][1] = vid[b][2] = 0u;
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                // the record: from the tile's record table, else gathered (mesh
                // programs read it only for a last-wins depth)
                bool tab = false;
                if (TAB && P.rec_table) tab = rec_table_find(s_thash, s_trec, s_sorted, prim[b], x0, y0, c0[b], c1[b]);
                if (!tab && (PROG != kProgMesh || MODE == kDepthLastWins)) {
                    const int4* cp = reinterpret_cast<const int4*>(P.records + ((tile_debug(P) & kDebugSameRecord) ? 0u : prim[b]));
                    c0[b] = cp[0];
                    c1[b] = cp[1];
                } else if (!tab) {
                    c0[b] = c1[b] = make_int4(0, 0, 1, 1);
                }
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                TriRecord r = decode_compact(P, c0[b], c1[b], false);
                if (__ballot(compact_is_large(c0[b]))) {  // rare, wave-uniform: a winner is a large primitive
                    if (compact_is_large(c0[b])) r = P.records_big[prim[b]];
                }
                const bool sw = (r.flags & kFlagSwapped) != 0u;
                r.v0 = vid[b][0];
                r.v1 = sw ? vid[b][2] : vid[b][1];
                r.v2 = sw ? vid[b][1] : vid[b][2];
                const EdgeEvalF e = eval_edges_f(r, px[b], py[b]);
                col[b][0] = col[b][1] = col[b][2] = col[b][3] = 0.0f;
                if (P.color_bpp && !(tile_debug(P) & kDebugSkipShade)) {
                    if constexpr (PROG == kProgMesh) shade_mesh(P, gp[b], vid[b], px[b], py[b], col[b]);
                    else shade_winner<PROG>(P, r, e, col[b]);
                }
                zw[b] = (MODE == kDepthLastWins) ? winner_depth(r, px[b], py[b]) : key_depth<MODE>(key[b]);
            }
        } else {
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                col[b][0] = col[b][1] = col[b][2] = col[b][3] = 0.0f;
                zw[b] = 0.0f;
            }
        }
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            if (!inside[b]) continue;
            if (P.color_bpp) store_color(P, px[b], py[b], have[b], col[b], s_srgb);
            if (P.depth) {
                float* dp = P.depth + (size_t)py[b] * P.fb_w + px[b];
                if (have[b] && P.depth_write_out) *dp = zw[b];
                else if (P.clear_depth_enable) *dp = P.clear_depth;
            }
        }
    }
}


// ------------------------------------------------------------ tile resolve
//
// The resolve shades each pixel's winner once, but fetches each *distinct*
// winner of the tile once (C2: ~280 winners for 1024 pixels): the pixels' winning
// records go into an LDS hash table that hands out dense winner ids, then the
// workgroup loads every winner's record, vertex ids and shading attributes with
// one cooperative pass into an LDS array (AoS, WinLayout), and each pixel shades
// from LDS.  A tile with more winners than the array holds runs it in batches.

// Per-winner words in LDS, 16-B aligned records (zr_kernels.hip resolve):
//   geometry  X0, Y0, (dx1 | dy1 << 16), (dx2 | dy2 << 16), |1/A2|   -- the compact
//             record (vertex 1/2 in record order); a large primitive keeps dx1 ==
//             kCompactLarge and its setup-record index in X0 (full record from HBM)
//   depth     z0, dz1, dz2                      (last-wins modes only)
//   attrs     flat: provoking colour (3); triangle: colour of v0..v2 (9); Blinn:
//             normals then colours (18); mesh: barycentric planes and their
//             reference pixel (12), normals (9), uvs (6).  Triangle/Blinn in record order, mesh/flat in API order.
template <int PROG, int MODE>
struct WinLayout {
    static constexpr bool kGeo = PROG == kProgTriangle || PROG == kProgBlinn || MODE == kDepthLastWins;
    static constexpr bool kZ = MODE == kDepthLastWins;
    static constexpr int kZOff = kGeo ? 5 : 0;
    static constexpr int kAttrOff = kZOff + (kZ ? 3 : 0);
    static constexpr int kAttrW = PROG == kProgFlat ? 3 : PROG == kProgTriangle ? 9 : PROG == kProgBlinn ? 18 : 27;
    static constexpr int kWords = (kAttrOff + kAttrW + 3) & ~3;
};

// Resolve hash table: TP setup-record ids (kWinEmpty = free), then the
// dense winner list (TP record ids); both live where the keys were.
// (TP = the tile's pixels, 1 << 2 TS)
constexpr uint32_t kWinEmpty = 0xFFFFFFFFu;
template <int TS>
__device__ __forceinline__ uint32_t win_hash(uint32_t rec) { return (rec * 0x9E3779B1u) >> (32 - 2 * TS); }  // log2(TP) bits

__device__ __forceinline__ void copy3(float* dst, const float* src) {
    dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2];
}

// Loads winner `rec` (a setup record) into w[0 .. WinLayout::kWords).
template <int PROG, int MODE, bool IDX32>
__device__ __forceinline__ void fetch_winner(const DrawParams& P, uint32_t rec, float* w) {
    using L = WinLayout<PROG, MODE>;
    uint32_t v[3];
    const uint32_t gp = record_prim<PROG>(P, rec);  // draw primitive (mesh: of the fan record)
    {
        const uint32_t tri = tri_of(P, gp);
        const uint32_t e0 = P.first + tri * 3u;
        if (IDX32) {
            const uint3 ix = *reinterpret_cast<const uint3*>(P.ib + (uint64_t)e0 * 4);
            const uint32_t off = (uint32_t)P.vertex_offset;  // two's complement: id + offset wraps to the valid id
            v[0] = ix.x + off; v[1] = ix.y + off; v[2] = ix.z + off;
        } else {
            winner_vids(P, gp, v);
        }
    }
    int4 q0 = make_int4(0, 0, 0, 0), q1 = q0;
    if (L::kGeo) {
        const int4* cp = reinterpret_cast<const int4*>(P.records + rec);
        q0 = cp[0];
        q1 = cp[1];
    }
    if (L::kGeo) {
        int* wi = reinterpret_cast<int*>(w);
        wi[0] = compact_is_large(q0) ? (int)rec : q0.x;
        wi[1] = q0.y;
        wi[2] = q0.z;
        wi[3] = q0.w;
        w[4] = fabsf(__int_as_float(q1.w));
    }
    if (L::kZ) {
        w[L::kZOff + 0] = __int_as_float(q1.x);
        w[L::kZOff + 1] = __int_as_float(q1.y);
        w[L::kZOff + 2] = __int_as_float(q1.z);
    }
    float* a = w + L::kAttrOff;
    if (PROG == kProgFlat) {
        copy3(a, attr_ptr(P, v[0], 1));  // provoking vertex = first (flat)
    } else if (PROG == kProgMesh) {
        const float4* q = P.mesh_edges + (size_t)gp * 3u;
        const float4 qa = q[0], qb = q[1], qc = q[2];
        a[0] = qa.x; a[1] = qa.y; a[2] = qa.z; a[3] = qa.w;
        a[4] = qb.x; a[5] = qb.y; a[6] = qb.z; a[7] = qb.w;
        a[8] = qc.x; a[9] = qc.y; a[10] = qc.z; a[11] = qc.w;
#pragma unroll
        for (int k = 0; k < 3; ++k) copy3(a + 12 + 3 * k, attr_ptr(P, v[k], 1));
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float* u = attr_ptr(P, v[k], 2);
            a[21 + 2 * k] = u[0];
            a[22 + 2 * k] = u[1];
        }
    } else {
        // record order: setup swapped v1 / v2 when it oriented the primitive (sign of 1/A2)
        const bool sw = q1.w < 0;
        const uint32_t r1 = sw ? v[2] : v[1], r2 = sw ? v[1] : v[2];
        copy3(a + 0, attr_ptr(P, v[0], 1));
        copy3(a + 3, attr_ptr(P, r1, 1));
        copy3(a + 6, attr_ptr(P, r2, 1));
        if (PROG == kProgBlinn) {
            copy3(a + 9, attr_ptr(P, v[0], 2));
            copy3(a + 12, attr_ptr(P, r1, 2));
            copy3(a + 15, attr_ptr(P, r2, 2));
        }
    }
}

// Colour (and for last-wins modes the depth) of pixel (px, py) from its winner's
// LDS words; the same operations as the oracle's per-fragment shading
// (zr_oracle.c shade), only fetched from LDS instead of the vertex buffer.
template <int PROG, int MODE>
__device__ __forceinline__ void shade_from_lds(const DrawParams& P, const float* w, int px, int py, float t3,
                                               float out[4], float& zw) {
    using L = WinLayout<PROG, MODE>;
    TriRecord r;
    EdgeEvalF e{0.0f, 0.0f, 0.0f};
    if (L::kGeo) {
        const int4 g = *reinterpret_cast<const int4*>(w);
        const bool large = compact_is_large(g);
        int4 q1 = make_int4(0, 0, 0, __float_as_int(w[4]));
        if (L::kZ) {
            q1.x = __float_as_int(w[L::kZOff + 0]);
            q1.y = __float_as_int(w[L::kZOff + 1]);
            q1.z = __float_as_int(w[L::kZOff + 2]);
        }
        r = decode_compact(P, g, q1, false);
        if (__ballot(large)) {  // rare, wave-uniform: a winner too large for the compact form
            if (large) r = P.records_big[g.x];
        }
        e = eval_edges_f(r, px, py);
        if (L::kZ) zw = winner_depth(r, px, py);
    }
    const float* a = w + L::kAttrOff;
    out[3] = 1.0f;
    if (PROG == kProgFlat) {
        out[0] = a[0]; out[1] = a[1]; out[2] = a[2];
        return;
    }
    if (PROG == kProgMesh) {
        // mesh.slang psmain: b_i = E_i / sum E with E_i = p . (h_j x h_k) at the pixel
        // centre, from the planes setup stored (mesh_edge_planes); then normal and uv
        // interpolated and lit like blinn_phong.slang, kd = (0.35 + 0.3 u, 0.35 + 0.3 v, 0.7)
        float E[3];
        mesh_plane_eval(a, px, py, E);
        const float einv = 1.0f / ((E[0] + E[1]) + E[2]);
        const float b0 = E[0] * einv, b1 = E[1] * einv, b2 = E[2] * einv;
        float n[3], uv[2];
#pragma unroll
        for (int i = 0; i < 3; ++i) n[i] = (b0 * a[12 + i] + b1 * a[15 + i]) + b2 * a[18 + i];
#pragma unroll
        for (int i = 0; i < 2; ++i) uv[i] = (b0 * a[21 + i] + b1 * a[23 + i]) + b2 * a[25 + i];
        shade_blinn_phong(n[0], n[1], n[2], fmaf(uv[0], 0.3f, 0.35f), fmaf(uv[1], 0.3f, 0.35f), 0.7f, out);
        return;
    }
    // perspective-correct weights b_i / w_i with w_i = 1 for every built-in vertex stage
    const float pw0 = e.f0 * r.invA2, pw1 = e.f1 * r.invA2, pw2 = e.f2 * r.invA2;
    const float inv = 1.0f / ((pw0 + pw1) + pw2);
    float f[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) f[i] = ((pw0 * a[i] + pw1 * a[3 + i]) + pw2 * a[6 + i]) * inv;
    if (PROG == kProgTriangle) {
        out[0] = shade_triangle_channel(f[0], t3);
        out[1] = shade_triangle_channel(f[1], t3);
        out[2] = shade_triangle_channel(f[2], t3);
        return;
    }
    float kd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) kd[i] = ((pw0 * a[9 + i] + pw1 * a[12 + i]) + pw2 * a[15 + i]) * inv;
    shade_blinn_phong(f[0], f[1], f[2], kd[0], kd[1], kd[2], out);
}

// Resolve of one tile (after the raster phase; s_key holds the final keys).
//   1  per pixel: key -> winning setup record; pixels no fragment won store the
//      clear, and the key's depth is stored now (depth-writing min/max modes).
//      The key array's upper half becomes the hash table: each thread empties the
//      slots lying over the keys it owns (so no barrier is needed before that).
//   2  winners into the hash table (LDS CAS, linear probing); the inserting lane
//      takes a dense id (one LDS add per wave) and records it beside the slot and
//      the winner in the dense list (the key array's lower half)
//   3  per batch of <= cap winners: cooperative fetch into LDS, then every pixel
//      whose winner is in the batch shades from LDS and stores its colour
// Three barriers in all.  s_u: the dense-id map (u16 per slot), then (kPer > 2)
// each pixel's dense id (u16), then the per-winner words (cap * kWords floats).
template <int PROG, int MODE, bool IDX32, int NT, int TS>
__device__ __forceinline__ void resolve_tile(const DrawParams& P, int x0, int y0, unsigned long long* s_key,
                                             uint32_t* s_u, uint32_t u_words, uint32_t* s_nwin,
                                             const float* s_srgb, unsigned long long* ts = nullptr) {
    constexpr int T = 1 << TS, TP = T * T;
    using L = WinLayout<PROG, MODE>;
    constexpr int kPer = TP / NT;
    constexpr bool kPixLds = kPer > 2;  // per-pixel ids in LDS (registers at 512 threads)
    uint32_t* s_list = reinterpret_cast<uint32_t*>(s_key);              // [TP] over keys 0..511
    uint32_t* s_tab = s_list + TP;                               // [TP] over keys 512..1023
    uint16_t* s_dmap = reinterpret_cast<uint16_t*>(s_u);                // [TP]
    uint32_t* s_pix = s_tab;  // [TP] (kPixLds): the table is free once every dense id is known
    float* s_win = reinterpret_cast<float*>(s_u + TP / 2u);
    const uint32_t cap = min((u_words - TP / 2u) / (uint32_t)L::kWords, TP);
    // recomputed here, not reused from the tile's init: a pixel coordinate kept
    // live across the raster loop spills at 64 VGPRs
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    uint32_t rec[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = tid + k * NT;
        const int px = x0 + (i & (T - 1)), py = y0 + (i >> TS);
        const bool inside = !(px < P.ra_x0 || px > P.ra_x1 || py < P.ra_y0 || py > P.ra_y1);
        const unsigned long long key = s_key[i];
        if (i >= (int)(TP / 2)) {  // this key's bytes hold hash slots 2(i - 512) and 2(i - 512) + 1
            s_tab[2 * (i - TP / 2)] = kWinEmpty;
            s_tab[2 * (i - TP / 2) + 1] = kWinEmpty;
        }
        const uint32_t seq = inside ? winner_seq<MODE>(key) : 0u;
        rec[k] = seq ? seq_record<PROG>(P, seq - 1u) : kWinEmpty;
        if (!inside) continue;
        if (!seq && P.color_bpp) {
            const float c[4] = {0.f, 0.f, 0.f, 0.f};
            store_color(P, px, py, false, c, s_srgb);
        }
        if (P.depth) {
            float* dp = P.depth + (size_t)py * P.fb_w + px;
            if (seq && P.depth_write_out) {
                if (MODE != kDepthLastWins) *dp = key_depth<MODE>(key);  // last-wins: interpolated in step 3
            } else if (P.clear_depth_enable) {
                *dp = P.clear_depth;
            }
        }
    }
    if (threadIdx.x == 0) *s_nwin = 0u;
    __syncthreads();  // every key read, every slot empty
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t hs[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        bool fresh = false;
        uint32_t h = win_hash<TS>(rec[k]);
        if (rec[k] != kWinEmpty) {
            for (;;) {  // linear probing; at most TP distinct records, so it ends
                const uint32_t old = atomicCAS(&s_tab[h], kWinEmpty, rec[k]);
                if (old == kWinEmpty) { fresh = true; break; }
                if (old == rec[k]) break;
                h = (h + 1u) & (TP - 1u);
            }
        }
        hs[k] = h;
        const unsigned long long b = __ballot(fresh);
        uint32_t base = 0;
        if (lane == 0 && b) base = atomicAdd(s_nwin, (uint32_t)__popcll(b));
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
        if (fresh) {
            const uint32_t d = base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
            s_list[d] = rec[k];
            s_dmap[h] = (uint16_t)d;
        }
    }
    __syncthreads();  // every winner has its dense id
    uint32_t did[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        did[k] = rec[k] != kWinEmpty ? (uint32_t)s_dmap[hs[k]] : kWinEmpty;
    }
    if (kPixLds) {
        __syncthreads();  // every lookup of the table done before it holds pixel ids
#pragma unroll
        for (int k = 0; k < kPer; ++k) s_pix[tid + k * NT] = did[k];  // read back by this thread only
    }
    const uint32_t nwin = *s_nwin;
    if (ts) ts[5] = __builtin_amdgcn_s_memrealtime();  // kDebugStamps: winners known
    const float t3 = PROG == kProgTriangle ? (P.time_ptr ? *P.time_ptr : 0.0f) * 3.0f : 0.0f;
    for (uint32_t base = 0; base < nwin; base += cap) {
        const uint32_t nb = min(cap, nwin - base);
        if (base) __syncthreads();  // the previous batch's pixels are done with s_win
        for (uint32_t j = threadIdx.x; j < nb; j += NT) {
            fetch_winner<PROG, MODE, IDX32>(P, s_list[base + j], s_win + (size_t)j * L::kWords);
            if (P.win_bits) {  // winner census (profiling level 2 only)
                const uint32_t g = record_prim<PROG>(P, s_list[base + j]);
                atomicOr(&P.win_bits[g >> 5], 1u << (g & 31u));
            }
        }
        __syncthreads();
        if (ts && !base) ts[6] = __builtin_amdgcn_s_memrealtime();  // first batch fetched
        auto shade_pixel = [&](int k, uint32_t dk) {
            const uint32_t j = dk - base;
            if (dk == kWinEmpty || j >= nb) return;
            const int i = tid + k * NT;
            const int px = x0 + (i & (T - 1)), py = y0 + (i >> TS);
            float col[4] = {0.f, 0.f, 0.f, 0.f};
            float zw = 0.0f;
            if (!(tile_debug(P) & kDebugSkipShade))
                shade_from_lds<PROG, MODE>(P, s_win + (size_t)j * L::kWords, px, py, t3, col, zw);
            if (P.color_bpp) store_color(P, px, py, true, col, s_srgb);
            if (MODE == kDepthLastWins && P.depth && P.depth_write_out) P.depth[(size_t)py * P.fb_w + px] = zw;
        };
        if (kPixLds) {
#pragma unroll 1
            for (int k = 0; k < kPer; ++k) shade_pixel(k, s_pix[tid + k * NT]);
        } else {
#pragma unroll
            for (int k = 0; k < kPer; ++k) shade_pixel(k, did[k]);
        }
    }
}

// NT threads per tile: 256 when the pass has several tiles per CU, 512 when it
// has few (tile-row shards, small attachments), so a tile's primitives spread
// over more waves (P.tile_threads, tile_threads_for).
template <int PROG, int MODE, bool INITD, int NT, int TS>
// (launch bounds: the second argument is the minimum waves per SIMD -- 8, i.e.
// 64 VGPRs, for both sizes; 8 x 256 or 4 x 512 threads per CU)
__global__ __launch_bounds__(NT, kTileWgs * kTileThreads / 256) void k_tile(DrawParams P) {
    constexpr int T = 1 << TS, TP = T * T;
    // LDS: a workgroup's share of the CU's 160 KiB at the occupancy the launch
    // bounds ask for (8 x 256 or 4 x 512 threads: 20 or 40 KiB).  The keys (8 KiB)
    // become the resolve's hash table; one union holds the raster scratch (sorted
    // segment, wave-path queue, bucket counts, initial depths) and then the
    // resolve's per-winner array.
    constexpr uint32_t kWgsPerCu = kTileWgs * (uint32_t)kTileThreads / (uint32_t)NT;
    constexpr uint32_t kBudget = 160u * 1024u / kWgsPerCu;
    constexpr uint32_t kMiscWords = 16;
    constexpr uint32_t kUnionWords = (kBudget - TP * 8u - 256u * 4u - kMiscWords * 4u) / 4u;
    static_assert(kSortCap + kBigQueue + kSortBuckets + (INITD ? TP : 0u) +
                          ((NT >= 512 && MODE != kDepthLastWins && PROG != kProgMesh && !INITD && (TS <= 5 || NT >= 1024))
                               ? 4u * kSortCap + kRecHashSlots
                               : 0u) <=
                      kUnionWords,
                  "k_tile raster scratch exceeds the workgroup's LDS share");
    __shared__ unsigned long long s_key[TP];
    __shared__ float s_srgb[256];
    __shared__ __attribute__((aligned(16))) uint32_t s_u[kUnionWords];
    __shared__ uint32_t s_misc[kMiscWords];
    uint32_t* s_sorted = s_u;                       // [kSortCap]
    // wave-path (large) primitives of the segment, rasterized after its
    // chunks by whichever wave claims them next: the area sort groups them, so the
    // wave owning their chunk would otherwise sweep them all alone
    uint32_t* s_big = s_u + kSortCap;               // [kBigQueue]
    uint32_t* s_bucket = s_big + kBigQueue;         // [kSortBuckets]
    float* s_initd = reinterpret_cast<float*>(s_bucket + kSortBuckets);  // [TP] (INITD)
    // 512-thread tiles: the record table of the resolve (rec_table_insert); last-wins
    // modes need the records' depth terms, which it does not hold
    // (64-px tiles: only 1024-thread workgroups have the LDS for it beside 32 KiB of keys)
    constexpr bool kTab = ZR_TAB && !ZR_RESOLVE_DEDUP512 && NT >= 512 && MODE != kDepthLastWins && PROG != kProgMesh &&
                          !INITD && (TS <= 5 || NT >= 1024);
    int4* s_trec = reinterpret_cast<int4*>(s_bucket + kSortBuckets);        // [kSortCap]
    uint32_t* s_thash = reinterpret_cast<uint32_t*>(s_trec + kSortCap);      // [kRecHashSlots]
    uint32_t& s_claim = s_misc[0];   // next 64-entry chunk of the segment to rasterize
    uint32_t& s_nbig = s_misc[1];
    uint32_t& s_bclaim = s_misc[2];
    uint32_t* s_dbg = s_misc + 3;    // [2] kDebugStamps: lane-walk steps of the chunks, wave-path sweeps
    uint32_t* s_nwin = s_misc + 5;   // resolve: distinct winners of the tile
    // a tile_order item: tile | job part << kJobTileBits, or a job grid's spare block
    const uint32_t jp = P.job_entries ? P.job_pad : 0u;  // (tile jobs: part blocks first)
    // (reversed timing runs reverse the tile blocks only, so block jp -- the
    // reporter below -- still holds a tile, never a spare part block)
    const uint32_t b = ((tile_debug(P) & kDebugReverseTiles) && blockIdx.x >= jp) ? jp + (gridDim.x - 1u - blockIdx.x)
                                                                                   : blockIdx.x;
    const uint32_t item = (b < jp || P.tile_sched) ? P.tile_order[b] : xcd_tile(b - jp, P.ntiles);
    // (a tile past the draw's would be a schedule bug: a wrong image the parity
    // tests see, not an access outside the buffers)
    if (item == kJobNone || (item & kJobTileMask) >= P.ntiles) return;
    const uint32_t t = item & kJobTileMask, part = item >> kJobTileBits;
    uint32_t tx, ty;
    shard_tile_xy(shard_geom(P), t, tx, ty);
    const int x0 = (int)tx * T, y0 = (int)ty * T;
    const bool stamp = (tile_debug(P) & kDebugStamps) && threadIdx.x == 0 && t < kMaxTilesPerPass;
    unsigned long long* ts = P.dbg_ts + 8192 * 8 + (size_t)t * 8;
    if (stamp) ts[0] = __builtin_amdgcn_s_memrealtime();

    // The tile's first segment of bin entries is requested before anything else
    // (workgroups dispatched last would otherwise queue these loads behind the
    // record gathers of every tile that started earlier), in parallel with its
    // count: the list lives at a fixed slab, bins[t * slab, ...), so the loads need
    // not wait for it; entries past the count are never used.
    const uint32_t slab = P.slab;
    const uint32_t lbeg = t * slab;
    constexpr uint32_t kPerThread = kSortCap / NT;
    uint32_t ent[kPerThread];
    auto load_segment = [&](uint32_t seg, uint32_t n) {
        // the segment's base as a uniform (scalar) pointer: lane addresses then come
        // from threadIdx alone instead of per-lane bases held (spilled) across the pass
        const uint32_t* bp = P.bins + lbeg + seg;
        asm volatile("" : "+s"(bp));
#pragma unroll
        for (uint32_t k = 0; k < kPerThread; ++k) {
            const uint32_t i = threadIdx.x + k * NT;
            ent[k] = i < n ? bp[i] : 0u;  // prim | cost bucket (k_setup_bin phase 4)
        }
    };
    // A list with pool runs (rare: crowded tiles) is loaded through the run table,
    // held in the wave-path queue's LDS (free between segments): run bases in
    // s_big[0, 256), exclusive pair offsets in s_big[256, 512); a position past the
    // slab part finds its run by binary search.
    static_assert(NT >= (int)kMaxRunsPerTile && 2u * kMaxRunsPerTile <= kBigQueue, "run table staging");
    auto load_segment_runs = [&](uint32_t seg, uint32_t n, uint32_t slab_len, uint32_t nruns) {
        const DrawParams& P = kernarg_params();  // (re-loaded here, not held across the pass)
        // one descriptor per thread (the loads in flight together), then wave 0's
        // exclusive scan of the run lengths
        if (threadIdx.x < nruns) {
            const uint2 r = P.runs[(size_t)t * P.run_cap + threadIdx.x];
            s_big[threadIdx.x] = r.x;
            s_big[kMaxRunsPerTile + threadIdx.x] = r.y;
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            uint32_t carry = 0;
            for (uint32_t i0 = 0; i0 < nruns; i0 += 64u) {
                const uint32_t i = i0 + threadIdx.x;
                const uint32_t len = i < nruns ? s_big[kMaxRunsPerTile + i] : 0u;
                uint32_t inc = len;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = __shfl_up(inc, d, 64);
                    if ((int)threadIdx.x >= d) inc += y;
                }
                if (i < nruns) s_big[kMaxRunsPerTile + i] = carry + inc - len;
                carry += (uint32_t)__shfl((int)inc, 63, 64);
            }
        }
        __syncthreads();
        // the segment's entries to s_sorted (free until the sort rewrites [0, n)),
        // then to the registers load_segment fills
        for (uint32_t i = threadIdx.x; i < n; i += NT) {
            const uint32_t p = seg + i;
            uint32_t e;
            if (p < slab_len) {
                e = P.bins[lbeg + p];
            } else {
                const uint32_t q = p - slab_len;
                uint32_t lo = 0, hi = nruns;  // the last run whose offset is <= q
                while (hi - lo > 1u) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_big[kMaxRunsPerTile + mid] <= q) lo = mid; else hi = mid;
                }
                e = P.bins[s_big[lo] + (q - s_big[kMaxRunsPerTile + lo])];
            }
            s_sorted[i] = e;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < kPerThread; ++k) {
            const uint32_t i = threadIdx.x + k * NT;
            ent[k] = i < n ? s_sorted[i] : 0u;
        }
    };
    if (!(tile_debug(P) & kDebugSkipRaster) && part == 0) load_segment(0, min(kSortCap, slab));
    const uint32_t count_v = P.tile_counts[t];
    const uint32_t count = count_v & ~kCountRuns;
    // The list: the slab's first slab_len entries, then the tile's pool runs
    // (k_setup_bin pool_run), count entries in all.  A tile with a dropped run (the
    // pool was full; the runtime grows the bin buffer for later draws) is
    // rasterized exactly but slowly: it scans every record's bbox (k_setup_bin
    // stored them all) instead.  Only a tile with kCountRuns reads its run word.

    for (int i = threadIdx.x; i < TP; i += NT) {
        const int px = x0 + (i & (T - 1)), py = y0 + (i >> TS);
        float d = P.clear_depth;
        if (P.load_depth && px < (int)P.fb_w && py < (int)P.fb_h) d = P.depth[(size_t)py * P.fb_w + px];
        s_key[i] = init_key<MODE>(d);
        if (INITD) s_initd[i] = d;
    }
    if (threadIdx.x < 255) s_srgb[threadIdx.x] = c_srgbT[threadIdx.x];
    const bool tab = kTab && P.rec_table != 0u;  // (runtime: draws dense enough to gain from it)
    if (tab)
        for (uint32_t i = threadIdx.x; i < kRecHashSlots; i += NT) s_thash[i] = 0u;
    if (threadIdx.x < 2) s_dbg[threadIdx.x] = 0u;
    // The first tile block dispatched reports the draw's setup and binning stats
    // (k_setup_bin's counters, complete before this launch) to the runtime's status
    // words: plain stores, no read of host memory unless a run was dropped
    // (volatile accesses wait for each one to cross the bus).  Draws run in stream
    // order; the host reads the words after a stream sync.
    if (blockIdx.x == jp && threadIdx.x == 0) {  // (jp: the first tile block; part blocks before it may be spare)
        uint32_t* st = P.status;
        const unsigned long long pairs = *reinterpret_cast<const unsigned long long*>(&P.counters[kCtPairs]);
        // pool: what the runs asked for; need: subs x the fullest sub-pool's asks,
        // which passes pool_cap exactly when a sub-pool dropped a run (pool_commit)
        unsigned long long pool = 0ull, need_sub = 0ull;
        const uint32_t subs = pool_subs(P);
        for (uint32_t k = 0; k < subs; ++k) {
            const unsigned long long a = *reinterpret_cast<const unsigned long long*>(&P.counters[kCtPoolSub0 + k * kCtSpread]);
            pool += a;
            need_sub = max(need_sub, a);
        }
        const unsigned long long pool_need = need_sub * subs;
        st[kStTrianglesSetup] = P.counters[kCtSetup];
        st[kStDroppedClip] = P.counters[kCtDropped];
        st[kStMicro] = P.counters[kCtMicro];
        st[kStTotalPairs] = pairs > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)pairs;
        st[kStPoolPairs] = pool > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)pool;
        st[kStPoolRuns] = P.counters[kCtPoolRuns];
        st[kStJobs] = P.counters[kCtJobs];
        if (P.counters[kCtJobsDenied]) {
            const uint32_t jd = st[kStJobsDenied];
            st[kStJobsDenied] = jd + 1u;
        }
        const uint32_t target = bin_slab_target(pairs, P.ntiles);
        if (pool_need > P.pool_cap) {  // a dropped run: the buffer this draw asks for (read-modify-write only here)
            const unsigned long long need = (unsigned long long)P.ntiles * target + pool_need;
            const uint32_t need32 = need > 0x80000000ull ? 0x80000000u : (uint32_t)need;
            const uint32_t ov = st[kStOverflow], bn = st[kStBinNeed];
            st[kStOverflow] = ov + 1u;
            if (need32 > bn) st[kStBinNeed] = need32;
        }
        if (P.stat_slot < kSlabSlots) {  // (the runtime derives the buffer the draw asks for from these)
            st[kStSlabSlot0 + P.stat_slot] = target;
            st[kStPoolSlot0 + P.stat_slot] = pool_need > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)pool_need;
            st[kStMaxSlot0 + P.stat_slot] = P.counters[kCtMaxTile];
            st[kStJobBufSlot0 + P.stat_slot] = P.counters[kCtJobBufs];
            st[kStJobPartSlot0 + P.stat_slot] = P.counters[kCtJobXcdMax];
        }
    }
    __syncthreads();
    const bool has_runs = (__builtin_amdgcn_readfirstlane((int)count_v) & (int)kCountRuns) != 0;
    const uint32_t rcw = has_runs ? (uint32_t)__builtin_amdgcn_readfirstlane((int)P.run_counts[t]) : 0u;
    const bool spill = (rcw & kRunDropped) != 0u;
    // this block's part of the list: all of it, or job `part` of K (build_job_schedule)
    const uint32_t J = P.job_entries ? (uint32_t)__builtin_amdgcn_readfirstlane((int)P.draw_info[kInfoJobEntries]) : 0u;
    const uint32_t K = tile_jobs(count, rcw, J);
    const uint32_t seg_lo = K > 1u ? part * J : 0u;
    const uint32_t cnt = spill ? 0u : K > 1u ? min(count, seg_lo + J) : count;
    // (the segment loop reads slab_len and the run count back from LDS, each wave
    // its own leader's copy: held in registers across the pass they cost the C2
    // instance VGPR spills; likewise the job count and key slot after it)
    if ((threadIdx.x & 63u) == 0) {
        s_misc[8] = (rcw & kRunFill) ? (rcw & ~(kRunFill | kRunDropped)) >> kRunFillShift : min(count, slab);
        s_misc[9] = has_runs ? P.run_cap : 0u;  // (one run slot per setup workgroup, empty ones of length 0)
        s_misc[10] = K;
        s_misc[11] = K > 1u ? P.job_slot[t] : 0u;
    }
    // k_setup_bin's counters back to zero for the next draw on this scratch set:
    // each tile its own count (every wave has read it: the barrier above) and, at
    // the end of the tile, its run word (read after that barrier), block 0 the draw
    // counters
    if (threadIdx.x == 0 && K == 1u) P.tile_counts[t] = 0u;  // (a split tile: its resolving job)
    if (blockIdx.x == jp)
        for (uint32_t i = threadIdx.x; i < kCtWords; i += NT) P.counters[i] = 0u;

    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (stamp) ts[1] = __builtin_amdgcn_s_memrealtime();
    if (!(tile_debug(P) & kDebugSkipRaster)) {
        // The list is processed in segments of kSortCap entries.  Each segment is
        // counting-sorted in LDS by the lane walk's pair steps over bbox ∩ tile
        // so that a 64-lane chunk holds primitives of similar cost (the lane loop runs
        // as long as its largest member).  Then each wave takes every 4th chunk: one
        // lane per entry loads the 64-B record, and the wave walks the chunk.
        for (uint32_t seg = seg_lo; seg < cnt; seg += kSortCap) {
            const uint32_t n = min(kSortCap, cnt - seg);
            // a list with pool runs loads its segments past the slab part through
            // the run table (s_misc[9]: runs, s_misc[8]: the slab part's length)
            const uint32_t nr = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_misc[9]);
            const uint32_t slab_len = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_misc[8]);
            if (nr && seg + n > slab_len) {
                load_segment_runs(seg, n, slab_len, nr);
            } else if (seg) {
                load_segment(seg, n);
            }
            const DrawParams& P = kernarg_params();  // re-loaded per segment, not held across the pass
            if (threadIdx.x < kSortBuckets) s_bucket[threadIdx.x] = 0u;
            if (threadIdx.x < 3) s_misc[threadIdx.x] = 0u;  // s_claim, s_nbig, s_bclaim
            __syncthreads();
            uint32_t pr[kPerThread], bk[kPerThread], sl[kPerThread];
#pragma unroll
            for (uint32_t k = 0; k < kPerThread; ++k) {
                const uint32_t i = threadIdx.x + k * NT;
                pr[k] = bk[k] = sl[k] = 0u;
                if (i < n) {
                    pr[k] = ent[k] & kBinPrimMask;
                    bk[k] = ent[k] >> kBinPrimBits;
                    sl[k] = atomicAdd(&s_bucket[bk[k]], 1u);
                }
            }
            __syncthreads();
            if (threadIdx.x < 64) {  // exclusive scan of the 64 bucket counts (one wave)
                const uint32_t c = s_bucket[threadIdx.x];
                uint32_t inc = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = __shfl_up(inc, d, 64);
                    if ((int)threadIdx.x >= d) inc += y;
                }
                s_bucket[threadIdx.x] = inc - c;
            }
            __syncthreads();
#pragma unroll
            for (uint32_t k = 0; k < kPerThread; ++k) {
                const uint32_t i = threadIdx.x + k * NT;
                if (i < n) s_sorted[s_bucket[bk[k]] + sl[k]] = pr[k];
            }
            __syncthreads();
            if (stamp && seg == 0) ts[2] = __builtin_amdgcn_s_memrealtime();
            // Waves claim 64-entry chunks from an LDS counter, largest bboxes first
            // (the sort put them last): longest-processing-time-first balances the
            // waves of a tile.  One lane per entry loads its 32-B compact record.
            // A sparse segment (fewer entries than lanes) gives each entry k lanes,
            // which split its bbox rows.  With no more chunks than waves each wave
            // takes one statically (measured faster there: C1 78 vs 85 us, C3 299
            // vs 304 us; LPT: C2 80 vs 82 us).
            const uint32_t kl = min(8u, max(1u, (uint32_t)NT / max(n, 1u)));
            const uint32_t ksh_s = 31u - __clz(kl);  // lanes per entry: 1, 2, 4 or 8
            // entries of the last bucket (127+ pair steps, ~253+ pixels) get at least
            // kBigLanes lanes: one lane would walk up to 1024 steps and hold
            // its whole chunk (and the tile) for that long.  Chunks are 64 lanes of
            // this lane space: the first off63 entries kl lanes each, then the rest.
            // Likewise buckets from kMidBucket up (bbox ∩ tile > 4 * kMidBucket px) get at
            // least kMidLanes lanes.  Three runs of the sorted segment, each a
            // fixed number of lanes per entry.
            const uint32_t ksh_b = max(ksh_s, (uint32_t)(31 - __clz(kBigLanes)));
            // (2 lanes from 129 px, 4 from 253: C3 tile pass 262 -> 219 us, cerberus 68
            // -> 60 us, C1 / C2 within noise; 4 lanes from 97 px, 8 from 253: C1 58 ->
            // 51 us, cerberus 60 -> 57, C3 219 -> 226, C2 equal -- the default.
            // Gating it on the middle run's length lost the gains: a few mid-size
            // entries already make the chunk that ends the tile.)
            const uint32_t off63 = s_bucket[kSortBuckets - 1];
            const uint32_t offm = s_bucket[kMidBucket];
            const uint32_t ksh_m = max(ksh_s, (uint32_t)(31 - __clz(kMidLanes)));
            const uint32_t lsp_s = offm << ksh_s;                      // lane space of buckets < MIDB
            const uint32_t lsp_m = lsp_s + ((off63 - offm) << ksh_m);  // ... and up to the last bucket
            const uint32_t lanes_all = lsp_m + ((n - off63) << ksh_b);
            const uint32_t nch = (lanes_all + 63u) / 64u;
            const bool lpt = nch > NT / 64u;
            for (uint32_t it = 0;; ++it) {
                uint32_t claim = wave + it * (NT / 64u);  // static: wave w takes chunks w, w + waves, ...
                if (lpt) {
                    if (lane == 0) claim = atomicAdd(&s_claim, 1u);
                    claim = (uint32_t)__builtin_amdgcn_readfirstlane((int)claim);
                }
                if (claim >= nch) break;
                const uint32_t g = (lpt ? nch - 1u - claim : claim) * 64u + (uint32_t)lane;  // lane-space slot
                const bool gb = g >= lsp_m, gm = g >= lsp_s;
                const uint32_t ksh = gb ? ksh_b : gm ? ksh_m : ksh_s;
                const uint32_t g0 = gb ? g - lsp_m : gm ? g - lsp_s : g;  // slot within its run
                const uint32_t j = (gb ? off63 : gm ? offm : 0u) + (g0 >> ksh);
                const int sub = (int)(g0 & ((1u << ksh) - 1u));
                uint32_t my_prim = 0;
                int4 q0 = make_int4(0, 0, 0, 0), q1 = q0;
                if (j < n) {
                    my_prim = s_sorted[j];
                    const int4* rp = reinterpret_cast<const int4*>(P.records + my_prim);
                    q0 = rp[0];
                    q1 = rp[1];
                }
                const bool valid = j < n && !(tile_debug(P) & kDebugLoadOnly);
                if (tile_debug(P) & kDebugLoadOnly) asm volatile("" ::"v"(q0.x), "v"(q1.x), "v"(my_prim));
                const bool large = compact_is_large(q0);
                // A large primitive below the last cost bucket (bbox ∩ tile under ~253
                // px) takes the lane walk too when its edge values there fit int32
                // (lane_walk_fits): a wave-path sweep spends ~100 instructions of setup
                // per primitive, and sliver-heavy tiles queue hundreds of primitives with
                // a few dozen covered pixels each (cerberus: tile pass 42.6 -> 26.9 us).
                // Its other two vertices come from records_big.  The last bucket stays on
                // the wave path, which covers a large part of the tile in fewer
                // instructions (all large primitives walked: C3 tile pass +4.7 us).
                bool walk = valid && !large;
                int2 v1 = make_int2(0, 0), v2 = v1;
                if (valid && large && (!gb || compact_is_sliver(q0) || ZR_LARGE_LANES >= 2) && ZR_LARGE_LANES) {
                    const int2* vp = reinterpret_cast<const int2*>(P.records_big + my_prim) + 1;
                    v1 = vp[0];
                    v2 = vp[1];
                    walk = lane_walk_fits<TS>(decode_large(P, q0, q1, true, v1, v2), x0, y0);
                }
                if (tab && valid && sub == 0) {
                    if (!large) {
                        rec_table_insert(s_thash, s_trec, my_prim, j, q0, q1, x0, y0);
                    } else {
                        // not hashed, but position j must not keep an earlier segment's
                        // small record: a hash slot that segment inserted for j would
                        // pass rec_table_find's s_sorted[j] check for this primitive.
                        // The large marker (dx1 == kCompactLarge in q0.z) sends such a
                        // lookup to records_big.
                        s_trec[j] = make_int4(0, q0.z, 0, 0);
                    }
                }
                if (walk && !(tile_debug(P) & kDebugSkipLanePath))
                    raster_lane<MODE, INITD, TS>(P, decode_large(P, q0, q1, large, v1, v2), entry_seq<PROG>(P, my_prim), x0, y0,
                                             s_key, s_initd, sub, (int)ksh);
                if (ZR_TILE_WORK_STATS && (tile_debug(P) & kDebugStamps)) {  // work of the chunk: its longest lane walk
                    int steps = 0;
                    if (valid && !large) {
                        const TriRecord r = decode_compact(P, q0, q1, true);
                        const int bw = min((int)(r.bb1 & 0xFFFFu), x0 + T - 1) - max((int)(r.bb0 & 0xFFFFu), x0) + 1;
                        const int bh = min((int)(r.bb1 >> 16), y0 + T - 1) - max((int)(r.bb0 >> 16), y0) + 1;
                        steps = (bw > 0 && bh > sub) ? bw * ((bh - sub + (1 << ksh) - 1) >> ksh) : 0;
                    }
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) steps = max(steps, __shfl_xor(steps, o, 64));
                    if (lane == 0) atomicAdd(&s_dbg[0], (uint32_t)steps);
                }
                // large primitives: queued for the segment's wave pass; the whole
                // wave sweeps them itself only when the queue is full
                const bool is_big = valid && large && !walk && sub == 0;
                unsigned long long big = __ballot(is_big);
                if (big) {
                    // The wave's batch takes the queue's free slots from `base` on; the
                    // part past its end stays with this wave.  (s_nbig counts every
                    // primitive offered, so the wave pass reads min(s_nbig, kBigQueue)
                    // slots, and each of them must be filled: a batch straddling the end
                    // fills the last slots.)
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&s_nbig, (uint32_t)__popcll(big));
                    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
                    const uint32_t room = base < kBigQueue ? min((uint32_t)__popcll(big), kBigQueue - base) : 0u;
                    const uint32_t rank = (uint32_t)__popcll(big & ((1ull << lane) - 1ull));
                    if (is_big && rank < room) s_big[base + rank] = my_prim;
                    for (uint32_t q = 0; q < room; ++q) big &= big - 1ull;  // the queued ones (lowest lanes)
                }
                while (big) {
                    const uint32_t i = (uint32_t)__builtin_ctzll(big);
                    big &= big - 1ull;
                    const uint32_t prim = (uint32_t)rl((int)my_prim, i);
                    const TriRecord r = load_uniform_record(P.records_big + prim);
                    raster_prim<MODE, INITD, TS>(P, r, entry_seq<PROG>(P, prim), x0, y0, lane, s_key, s_initd);
                    if (ZR_TILE_WORK_STATS && (tile_debug(P) & kDebugStamps) && lane == 0) atomicAdd(&s_dbg[1], prim_sweeps<TS>(r, x0, y0));
                }
            }
            __syncthreads();
            const uint32_t nbig = min(s_nbig, kBigQueue);
            if (stamp && NT >= 512 && seg == 0) {  // first segment: chunks done, wave-path queue length
                ts[5] = __builtin_amdgcn_s_memrealtime();
                ts[6] = (unsigned long long)s_nbig << 32;
            }
            for (;;) {  // the segment's queued wave-path primitives, two per claim
                uint32_t i = 0;
                if (lane == 0) i = atomicAdd(&s_bclaim, 2u);
                i = (uint32_t)__builtin_amdgcn_readfirstlane((int)i);
                if (i >= nbig || (tile_debug(P) & kDebugSkipWavePath)) break;
                const bool two = i + 1u < nbig;
                const uint32_t e0 = s_big[i], e1 = two ? s_big[i + 1u] : e0;
                // both full records' loads in flight at once (one exposed latency per
                // claim), the second held in scalar registers.  (Staging the segment's
                // queued records in LDS with one workgroup-wide load: cerberus -0.8 us,
                // C2 +0.9, C3 +2.6.)
                const int4* a = reinterpret_cast<const int4*>(P.records_big + e0);
                const int4* b = reinterpret_cast<const int4*>(P.records_big + e1);
                const int4 a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
                const int4 b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3];
                const TriRecord ra = uniform_record(a0, a1, a2, a3);
                const TriRecord rb = uniform_record(b0, b1, b2, b3);
                raster_prim<MODE, INITD, TS>(P, ra, entry_seq<PROG>(P, e0), x0, y0, lane, s_key, s_initd);
                if (two) raster_prim<MODE, INITD, TS>(P, rb, entry_seq<PROG>(P, e1), x0, y0, lane, s_key, s_initd);
            }
            __syncthreads();
        }
        if (spill) {
            const uint32_t r0 = 0u, n_rec = P.draw_info[kInfoRecords];  // setup records of the draw
            const bool by_pos = P.draw_info[kInfoByPosition] != 0u;
            for (uint32_t cb = r0 + wave * 64u; cb < n_rec; cb += NT) {
                const uint32_t j = cb + (uint32_t)lane;
                bool hit = false;
                int4 q0 = make_int4(0, 0, 0, 0), q1 = q0;
                if (j < n_rec) {
                    const BBox bb = P.bboxes[j];
                    hit = bb.bb0 != kEmptyBox && (int)(bb.bb0 & 0xFFFFu) < x0 + T && (int)(bb.bb1 & 0xFFFFu) >= x0 &&
                          (int)(bb.bb0 >> 16) < y0 + T && (int)(bb.bb1 >> 16) >= y0;
                }
                uint32_t rec = j;  // bboxes by position; records by draw primitive (records mode: gids)
                if (hit) {
                    if (by_pos) rec = P.gids[j];
                    const int4* rp = reinterpret_cast<const int4*>(P.records + rec);
                    q0 = rp[0];
                    q1 = rp[1];
                }
                const bool large = compact_is_large(q0);
                if (hit && !large)
                    raster_lane<MODE, INITD, TS>(P, decode_compact(P, q0, q1, true), entry_seq<PROG>(P, rec), x0, y0, s_key,
                                             s_initd, 0, 0);
                unsigned long long big = __ballot(hit && large);
                while (big) {
                    const uint32_t i = (uint32_t)__builtin_ctzll(big);
                    big &= big - 1ull;
                    const uint32_t prim = (uint32_t)rl((int)rec, i);
                    raster_prim<MODE, INITD, TS>(P, load_uniform_record(P.records_big + prim), entry_seq<PROG>(P, prim), x0, y0, lane,
                                             s_key, s_initd);
                }
            }
        }
    }
    __syncthreads();
    // A split tile (tile jobs): every job stores its keys to a buffer of its own
    // (job_keys[job_slot[t] + part]) and takes a ticket; the last job to arrive
    // folds the others' keys into its own with a min (every job started from the
    // same initial keys) and resolves the tile, the others end here.  (Plain
    // system-coherent stores and loads: merging with 64-bit atomic mins at device
    // scope ran c2x's tile pass at 281 us with jobs of 2048 entries, 639 with 512;
    // their blocks are not reliably on one XCD, so L2-local atomics lost keys.)
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)s_misc[10]) > 1u) {
        const uint32_t Kj = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_misc[10]);
        const uint32_t buf0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_misc[11]);
        unsigned long long* mine = P.job_keys + (size_t)(buf0 + part) * TP;
        int i0 = threadIdx.x;  // (opaque: the key addresses of the init loop, held across the pass, spilled)
        asm volatile("" : "+v"(i0));
        for (int i = i0; i < TP; i += NT)
            __hip_atomic_store(&mine[i], s_key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (each thread's stores done before the ticket)
        __syncthreads();
        if (threadIdx.x == 0)
            s_misc[12] = __hip_atomic_fetch_add(&P.job_tickets[buf0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)s_misc[12]) != Kj - 1u) return;
        // (eight buffers' loads in flight per pixel: one buffer at a time, the fold
        // of a 15-job tile was ~15 memory round trips on the pass's critical path)
        const unsigned long long* keys0 = P.job_keys + (size_t)buf0 * TP;
        for (int i = i0; i < TP; i += NT) {
            unsigned long long m = s_key[i];
            for (uint32_t j0 = 0; j0 < Kj; j0 += 8u) {
                unsigned long long v[8];
#pragma unroll
                for (uint32_t k = 0; k < 8u; ++k) {
                    const uint32_t j = j0 + k;
                    v[k] = (j < Kj && j != part)
                               ? __hip_atomic_load(&keys0[(size_t)j * TP + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : ~0ull;
                }
#pragma unroll
                for (uint32_t k = 0; k < 8u; ++k) m = v[k] < m ? v[k] : m;
            }
            s_key[i] = m;
        }
        if (threadIdx.x == 0) {
            __hip_atomic_store(&P.job_tickets[buf0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            P.tile_counts[t] = 0u;  // (every job of the tile read it before its ticket)
        }
        __syncthreads();
    }
    if (stamp) ts[3] = __builtin_amdgcn_s_memrealtime();

    // Resolve (the index width is a template parameter so a winner's record and
    // index loads are issued back to back).
    if constexpr (NT >= 512 && !ZR_RESOLVE_DEDUP512) {
        if (P.index_size == 4)
            resolve_pixels<PROG, MODE, true, NT, kTab, TS>(kernarg_params(), x0, y0, s_key, s_srgb, s_thash, s_trec, s_sorted);
        else
            resolve_pixels<PROG, MODE, false, NT, kTab, TS>(kernarg_params(), x0, y0, s_key, s_srgb, s_thash, s_trec, s_sorted);
    } else if (P.index_size == 4) {
        resolve_tile<PROG, MODE, true, NT, TS>(kernarg_params(), x0, y0, s_key, s_u, kUnionWords, s_nwin, s_srgb,
                                          stamp ? ts : nullptr);
    } else {
        resolve_tile<PROG, MODE, false, NT, TS>(kernarg_params(), x0, y0, s_key, s_u, kUnionWords, s_nwin, s_srgb,
                                           stamp ? ts : nullptr);
    }
    // A tile with pool runs (s_misc[9]: its run slots) clears its run table and run
    // word for the next draw (every wave read them before the segment loop; a
    // split tile: its resolving job, after every job's loop)
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)s_misc[9])) {
        const DrawParams& Q = kernarg_params();  // (loaded here, not held across the pass)
        uint2* rt = Q.runs + (size_t)t * Q.run_cap;
        for (uint32_t i = threadIdx.x; i < Q.run_cap; i += NT) rt[i] = make_uint2(0u, 0u);
        if (threadIdx.x == 0) Q.run_counts[t] = 0u;
    }
    if (stamp) {
        ts[4] = __builtin_amdgcn_s_memrealtime();
        ts[7] = ((unsigned long long)s_dbg[1] << 32) | s_dbg[0];
        if (NT >= 512) {  // (resolve_tile's own stamps use these two at 256 threads)
            if (!count) {  // no segment ran: no wave-path queue either (dbg_ts persists across draws)
                ts[5] = ts[2] = ts[1];
                ts[6] = 0ull;
            } else {
                ts[6] = (ts[6] & ~0xFFFFFFFFull) | count;  // the tile's list length (tools/tile_stamps.py)
            }
        }
    }
}

__global__ __launch_bounds__(kTileThreads) void k_clear(DrawParams P) {
    const uint32_t t = blockIdx.x;
    uint32_t tx, ty;
    shard_tile_xy(shard_geom(P), t, tx, ty);
    const int x0 = (int)tx * kTile, y0 = (int)ty * kTile;
    const float c[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < kTilePixels; i += kTileThreads) {
        const int px = x0 + (i & (kTile - 1)), py = y0 + (i >> kTileShift);
        if (px < P.ra_x0 || px > P.ra_x1 || py < P.ra_y0 || py > P.ra_y1) continue;
        if (P.color_bpp && P.clear_color_enable) store_color(P, px, py, false, c, c_srgbT);
        if (P.depth && P.clear_depth_enable) P.depth[(size_t)py * P.fb_w + px] = P.clear_depth;
    }
}

// ---------------------------------------------------------------- launchers

static inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

size_t setup_bin_lds_bytes(uint32_t ntiles, uint32_t bbox_entries, uint32_t stage_pairs) {
    const size_t nt4 = ((size_t)ntiles + 3u) / 4u * 4u;
    return (nt4 + kSetupMiscWords) * sizeof(uint32_t) + (size_t)bbox_entries * sizeof(BBox) +
           (stage_pairs ? nt4 * sizeof(uint32_t) + (size_t)stage_pairs * 8u : 0u);
}

const void* setup_bin_kernel(uint32_t batch, bool mesh) {
    if (mesh) return reinterpret_cast<const void*>(&k_setup_bin<1, true>);
    switch (batch) {
    case 1: return reinterpret_cast<const void*>(&k_setup_bin<1, false>);
    case 2: return reinterpret_cast<const void*>(&k_setup_bin<2, false>);
    default: return reinterpret_cast<const void*>(&k_setup_bin<4, false>);
    }
}

void launch_setup_bin(const DrawParams& p, void* stream) {
    const size_t lds = setup_bin_lds_bytes(p.ntiles, p.bbox_lds, p.bin_stage);
    const hipStream_t s = (hipStream_t)stream;
    if (p.program == kProgMesh) {  // batch 1: the clip path is heavy
        hipLaunchKernelGGL((k_setup_bin<1, true>), dim3(p.setup_wgs), dim3(kSetupThreads), lds, s, p);
        return;
    }
    switch (p.setup_batch) {
    case 1: hipLaunchKernelGGL((k_setup_bin<1, false>), dim3(p.setup_wgs), dim3(kSetupThreads), lds, s, p); break;
    case 2: hipLaunchKernelGGL((k_setup_bin<2, false>), dim3(p.setup_wgs), dim3(kSetupThreads), lds, s, p); break;
    default: hipLaunchKernelGGL((k_setup_bin<4, false>), dim3(p.setup_wgs), dim3(kSetupThreads), lds, s, p); break;
    }
}

template <int PROG, int MODE, int NT, int TS>
static void launch_tile_pmt(const DrawParams& p, hipStream_t s, bool initd) {
    const uint32_t blocks = p.ntiles + (p.job_entries ? p.job_pad : 0u);  // (tile jobs: part blocks first)
    if constexpr (MODE == kDepthLastWins) {  // (initial depths: last-wins modes only)
        if (initd) {
            hipLaunchKernelGGL((k_tile<PROG, MODE, true, NT, TS>), dim3(blocks), dim3(NT), 0, s, p);
            return;
        }
    }
    hipLaunchKernelGGL((k_tile<PROG, MODE, false, NT, TS>), dim3(blocks), dim3(NT), 0, s, p);
}

// Tile-edge instances (tile_variant_built): every program and mode at 32 px, with
// 256 or 512 threads (tile_threads_for); 16- and 64-px tiles (256 / 512 or 1024
// threads) for the flat and Blinn-Phong programs under the depth-writing modes, the draws
// tile_shift_for picks them for (dense soups, crowded scenes).
template <int PROG, int MODE>
static void launch_tile_pm(const DrawParams& p, hipStream_t s, bool initd) {
    if constexpr (tile_variant_built(PROG, MODE)) {
        if (p.tile_shift == 6u)
            return p.tile_threads == 1024u ? launch_tile_pmt<PROG, MODE, 1024, 6>(p, s, initd)
                                           : launch_tile_pmt<PROG, MODE, 512, 6>(p, s, initd);
        if (p.tile_shift == 4u) return launch_tile_pmt<PROG, MODE, kTileThreads, 4>(p, s, initd);
    }
    switch (p.tile_threads) {
    case 512: launch_tile_pmt<PROG, MODE, 512, kTileShift>(p, s, initd); break;
    default: launch_tile_pmt<PROG, MODE, kTileThreads, kTileShift>(p, s, initd); break;
    }
}

template <int PROG>
static void launch_tile_p(const DrawParams& p, hipStream_t s, bool initd) {
    switch (p.depth_mode) {
    case kDepthMinStrict: launch_tile_pm<PROG, kDepthMinStrict>(p, s, false); break;
    case kDepthMinNonStrict: launch_tile_pm<PROG, kDepthMinNonStrict>(p, s, false); break;
    case kDepthMaxStrict: launch_tile_pm<PROG, kDepthMaxStrict>(p, s, false); break;
    case kDepthMaxNonStrict: launch_tile_pm<PROG, kDepthMaxNonStrict>(p, s, false); break;
    default: launch_tile_pm<PROG, kDepthLastWins>(p, s, initd); break;
    }
}

void launch_tile(const DrawParams& p, void* stream) {
    if (p.ntiles == 0) return;
    const bool initd = p.depth_mode == kDepthLastWins && p.depth != nullptr && p.depth_op != 7;
    hipStream_t s = (hipStream_t)stream;
    switch (p.program) {
    case kProgTriangle: launch_tile_p<kProgTriangle>(p, s, initd); break;
    case kProgFlat: launch_tile_p<kProgFlat>(p, s, initd); break;
    case kProgMesh: launch_tile_p<kProgMesh>(p, s, initd); break;
    default: launch_tile_p<kProgBlinn>(p, s, initd); break;
    }
}

void launch_route(const DrawParams& p, void* stream) {
    hipLaunchKernelGGL(k_route, dim3(p.route_chunks), dim3(kRouteThreads), 0, (hipStream_t)stream, p);
}

void launch_clear(const DrawParams& p, void* stream) {
    if (p.ntiles == 0) return;
    hipLaunchKernelGGL(k_clear, dim3(p.ntiles), dim3(kTileThreads), 0, (hipStream_t)stream, p);
}

}  // namespace zr
