// zr_kernels.hip — the MI355X (gfx950) draw path: setup -> scan -> bin -> tile.
//
// Pass structure:
//   k_setup  one thread per primitive: index + vertex fetch, vertex stage
//            (triangle.slang:19-25: SV_Position = float4(position, 1)), viewport
//            transform, 8-bit sub-pixel snap, facing/cull, orientation, top-left
//            biases, clipped pixel bbox -> 64-B TriRecord; per-tile overlap counts.
//   k_scan   one workgroup: exclusive scan of the per-tile counts.
//   k_bin    one thread per primitive: scatter primitive ids into per-tile lists.
//   k_tile   one 256-thread workgroup per 32x32 screen tile: LDS-resident 64-bit
//            visibility keys (depth | primitive sequence) updated with ds_min_u64
//            by a wave per primitive (lanes over the primitive's bbox ∩ tile),
//            then a resolve that shades each pixel's winner once (psmain),
//            encodes to the attachment format and writes colour + depth with
//            coalesced row stores.  The attachment CLEAR is fused into the resolve.
//
// Coverage/depth arithmetic is exact integer + explicitly ordered float math,
// bit-identical to the in-order CPU oracle (oracle/zr_oracle.c).
#include <hip/hip_runtime.h>

#include "zr_internal.h"
#include "zr_shading.h"

namespace zr {

__constant__ float c_srgbT[255] = ZR_SRGB_THRESHOLDS_INIT;

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

__device__ __forceinline__ const float* attr_ptr(const DrawParams& P, uint32_t vid, uint32_t loc) {
    return (const float*)(P.vb + (uint64_t)vid * P.stride + P.attr_offset[loc]);
}

__device__ __forceinline__ void prim_vids(const DrawParams& P, uint32_t prim, uint32_t flags, uint32_t vid[3]) {
    const uint32_t tri = (P.tris_per_instance == P.prims) ? prim : prim % P.tris_per_instance;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        int64_t v;
        fetch_index(P, (uint64_t)P.first + (uint64_t)tri * 3u + (uint64_t)k, v);
        vid[k] = (uint32_t)v;
    }
    if (flags & kFlagSwapped) {
        const uint32_t t = vid[1];
        vid[1] = vid[2];
        vid[2] = t;
    }
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

__device__ __forceinline__ float interp_depth(const TriRecord& r, long long w1, long long w2) {
    const float b1 = (float)w1 * r.invA2, b2 = (float)w2 * r.invA2;
    float z = fmaf(b2, r.dz2, fmaf(b1, r.dz1, r.z0));
    return z == 0.0f ? 0.0f : z;
}

// ------------------------------------------------------------------ k_setup

__global__ __launch_bounds__(kSetupThreads) void k_setup(DrawParams P) {
    const uint32_t prim = blockIdx.x * kSetupThreads + threadIdx.x;
    uint32_t ntiles = 0;
    int valid = 0, dropped = 0;
    if (prim < P.prims) {
        const uint32_t tri = (P.tris_per_instance == P.prims) ? prim : prim % P.tris_per_instance;
        uint32_t vid[3];
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            int64_t v = 0;
            ok = ok && fetch_index(P, (uint64_t)P.first + (uint64_t)tri * 3u + (uint64_t)k, v);
            ok = ok && v >= 0 && v <= 0xFFFFFFFFll;
            vid[k] = (uint32_t)v;
            for (uint32_t a = 0; a < P.nattr; ++a)
                ok = ok && ((uint64_t)vid[k] * P.stride + P.attr_offset[a] + 12 <= P.vb_bytes);
        }
        int32_t X[3], Y[3];
        float z[3], invw[3];
        if (ok) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float* pos = attr_ptr(P, vid[k], 0);
                const float x = pos[0], y = pos[1], zc = pos[2], w = 1.0f;  // vsmain
                if (!(w > 0.0f)) { dropped = 1; ok = false; break; }
                const float xd = x / w, yd = y / w, zd = zc / w;
                const float xf = fmaf(xd, P.hw, P.cx), yf = fmaf(yd, P.hh, P.cy);
                if (!(fabsf(xf) < 4194304.0f && fabsf(yf) < 4194304.0f)) { dropped = 1; ok = false; break; }
                X[k] = (int32_t)rintf(xf * 256.0f);
                Y[k] = (int32_t)rintf(yf * 256.0f);
                z[k] = fmaf(zd, P.dr, P.dmin);
                invw[k] = 1.0f / w;
            }
        }
        if (ok) {
            long long A2 = (long long)(X[1] - X[0]) * (Y[2] - Y[0]) - (long long)(X[2] - X[0]) * (Y[1] - Y[0]);
            const bool ccw = A2 < 0;  // Vulkan: a = -A2/2 > 0 is counter-clockwise
            const bool front = (P.front_face == 0) ? ccw : !ccw;
            ok = A2 != 0 && !((P.cull_mode & 1u) && front) && !((P.cull_mode & 2u) && !front);
            uint32_t flags = 0;
            if (ok && A2 < 0) {
                int32_t t = X[1]; X[1] = X[2]; X[2] = t;
                t = Y[1]; Y[1] = Y[2]; Y[2] = t;
                float f = z[1]; z[1] = z[2]; z[2] = f;
                f = invw[1]; invw[1] = invw[2]; invw[2] = f;
                A2 = -A2;
                flags |= kFlagSwapped;
            }
            int32_t px0 = 0, py0 = 0, px1 = -1, py1 = -1;
            if (ok) {
                // top-left rule (y-down): edge i is opposite vertex i
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const int a = (i + 1) % 3, b = (i + 2) % 3;
                    const int32_t dx = X[b] - X[a], dy = Y[b] - Y[a];
                    const bool tl = (dy < 0) || (dy == 0 && dx > 0);
                    if (!tl) flags |= (kFlagBias0 << i);
                }
                const int32_t minX = min(X[0], min(X[1], X[2])), maxX = max(X[0], max(X[1], X[2]));
                const int32_t minY = min(Y[0], min(Y[1], Y[2])), maxY = max(Y[0], max(Y[1], Y[2]));
                px0 = max((minX - 128 + 255) >> 8, P.clip_x0);
                px1 = min((maxX - 128) >> 8, P.clip_x1);
                py0 = max((minY - 128 + 255) >> 8, P.clip_y0);
                py1 = min((maxY - 128) >> 8, P.clip_y1);
                ok = px0 <= px1 && py0 <= py1;
            }
            if (ok) {
                valid = 1;
                const int tx0 = px0 >> kTileShift, tx1 = px1 >> kTileShift;
                const int ty0 = py0 >> kTileShift, ty1 = py1 >> kTileShift;
                for (int ty = ty0; ty <= ty1; ++ty) {
                    if ((uint32_t)ty % P.shard_count != P.shard_rank) continue;
                    const uint32_t row = ((uint32_t)ty / P.shard_count) * P.tiles_x;
                    for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&P.tile_counts[row + tx], 1u);
                    ntiles += (uint32_t)(tx1 - tx0 + 1);
                }
                if (ntiles) {
                    TriRecord r;
                    r.X0 = X[0]; r.Y0 = Y[0]; r.X1 = X[1]; r.Y1 = Y[1]; r.X2 = X[2]; r.Y2 = Y[2];
                    r.z0 = z[0];
                    r.dz1 = z[1] - z[0];
                    r.dz2 = z[2] - z[0];
                    r.invA2 = 1.0f / (float)A2;
                    r.invw0 = invw[0]; r.invw1 = invw[1]; r.invw2 = invw[2];
                    r.bb0 = (uint32_t)px0 | ((uint32_t)py0 << 16);
                    r.bb1 = (uint32_t)px1 | ((uint32_t)py1 << 16);
                    r.flags = flags;
                    P.records[prim] = r;
                }
            }
        }
        P.tri_ntiles[prim] = ntiles;
    }
    const int nvalid = __syncthreads_count(valid);
    const int ndropped = __syncthreads_count(dropped);
    if (threadIdx.x == 0) {
        uint32_t* ct = P.tile_counts + P.ntiles;
        if (nvalid) atomicAdd(&ct[kCtSetup], (uint32_t)nvalid);
        if (ndropped) atomicAdd(&ct[kCtDropped], (uint32_t)ndropped);
    }
}

// ------------------------------------------------------------------- k_scan

__global__ __launch_bounds__(1024) void k_scan(DrawParams P) {
    __shared__ uint32_t s_wave[16];
    const uint32_t n = P.ntiles, tid = threadIdx.x;
    const uint32_t per = (n + 1023u) / 1024u;
    const uint32_t beg = min(tid * per, n), end = min(beg + per, n);
    uint32_t sum = 0;
    for (uint32_t i = beg; i < end; ++i) sum += P.tile_counts[i];
    // wave-level inclusive scan
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    if (tid < 16) {
        uint32_t w = s_wave[tid], wi = w;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t v = __shfl_up(wi, d, 16);
            if ((int)tid >= d) wi += v;
        }
        s_wave[tid] = wi - w;  // exclusive wave base
    }
    __syncthreads();
    uint32_t run = s_wave[wave] + incl - sum;
    for (uint32_t i = beg; i < end; ++i) {
        P.tile_offsets[i] = run;
        run += P.tile_counts[i];
    }
    if (tid == 1023) {
        const uint32_t total = run;
        volatile uint32_t* st = P.status;
        st[kStTotalPairs] = total;
        if (total > P.bin_capacity) st[kStOverflow] = 1u;
        if (total > st[kStMaxPairs]) st[kStMaxPairs] = total;
        const uint32_t* ct = P.tile_counts + P.ntiles;
        st[kStTrianglesSetup] = ct[kCtSetup];
        st[kStDroppedClip] = ct[kCtDropped];
    }
}

// -------------------------------------------------------------------- k_bin

__global__ __launch_bounds__(kSetupThreads) void k_bin(DrawParams P) {
    const uint32_t prim = blockIdx.x * kSetupThreads + threadIdx.x;
    if (prim >= P.prims || P.tri_ntiles[prim] == 0) return;
    const uint32_t bb0 = P.records[prim].bb0, bb1 = P.records[prim].bb1;
    const int tx0 = (int)(bb0 & 0xFFFFu) >> kTileShift, tx1 = (int)(bb1 & 0xFFFFu) >> kTileShift;
    const int ty0 = (int)(bb0 >> 16) >> kTileShift, ty1 = (int)(bb1 >> 16) >> kTileShift;
    for (int ty = ty0; ty <= ty1; ++ty) {
        if ((uint32_t)ty % P.shard_count != P.shard_rank) continue;
        const uint32_t row = ((uint32_t)ty / P.shard_count) * P.tiles_x;
        for (int tx = tx0; tx <= tx1; ++tx) {
            const uint32_t pos = atomicAdd(&P.tile_offsets[row + tx], 1u);
            if (pos < P.bin_capacity) P.bins[pos] = prim;
        }
    }
}

// ------------------------------------------------------------------- k_tile

template <int PROG>
__device__ __forceinline__ void shade_winner(const DrawParams& P, const TriRecord& r, uint32_t prim, const EdgeEval& e,
                                             float out[4]) {
    uint32_t vid[3];
    prim_vids(P, prim, r.flags, vid);
    if (PROG == kProgFlat) {
        const float* c = attr_ptr(P, vid[0], 1);
        out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = 1.0f;
        return;
    }
    const float b0 = (float)e.w0 * r.invA2, b1 = (float)e.w1 * r.invA2, b2 = (float)e.w2 * r.invA2;
    const float pw0 = b0 * r.invw0, pw1 = b1 * r.invw1, pw2 = b2 * r.invw2;
    const float inv = 1.0f / ((pw0 + pw1) + pw2);
    const float* a0 = attr_ptr(P, vid[0], 1);
    const float* a1 = attr_ptr(P, vid[1], 1);
    const float* a2 = attr_ptr(P, vid[2], 1);
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
    const float* k0 = attr_ptr(P, vid[0], 2);
    const float* k1 = attr_ptr(P, vid[1], 2);
    const float* k2 = attr_ptr(P, vid[2], 2);
    float kd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) kd[i] = ((pw0 * k0[i] + pw1 * k1[i]) + pw2 * k2[i]) * inv;
    shade_blinn_phong(f[0], f[1], f[2], kd[0], kd[1], kd[2], out);
}

__device__ __forceinline__ void store_color(const DrawParams& P, int px, int py, bool have, const float c[4]) {
    const size_t idx = (size_t)py * P.fb_w + (size_t)px;
    if (P.color_bpp == 4) {
        uint32_t* cp = (uint32_t*)P.color + idx;
        const uint32_t m = rgba8_write_mask(P.write_mask, P.color_format);
        if (have) {
            const uint32_t texel = pack_rgba8(c, P.color_format, c_srgbT);
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

template <int PROG, int MODE, bool INITD>
__global__ __launch_bounds__(kTileThreads) void k_tile(DrawParams P) {
    __shared__ unsigned long long s_key[kTilePixels];
    __shared__ float s_initd[INITD ? kTilePixels : 1];
    const uint32_t t = blockIdx.x;
    const uint32_t oy = t / P.tiles_x, tx = t - oy * P.tiles_x;
    const uint32_t ty = oy * P.shard_count + P.shard_rank;
    const int x0 = (int)tx * kTile, y0 = (int)ty * kTile;

    for (int i = threadIdx.x; i < kTilePixels; i += kTileThreads) {
        const int px = x0 + (i & (kTile - 1)), py = y0 + (i >> kTileShift);
        float d = P.clear_depth;
        if (P.load_depth && px < (int)P.fb_w && py < (int)P.fb_h) d = P.depth[(size_t)py * P.fb_w + px];
        s_key[i] = init_key<MODE>(d);
        if (INITD) s_initd[i] = d;
    }
    __syncthreads();

    const uint32_t cnt = P.tile_counts[t];
    const uint32_t begin = P.tile_offsets[t] - cnt;  // offsets hold list ends after k_bin
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    for (uint32_t j = wave; j < cnt; j += kTileThreads / 64) {
        const uint32_t slot = begin + j;
        if (slot >= P.bin_capacity) break;  // overflowed draw: replayed by the runtime
        const uint32_t prim = __builtin_amdgcn_readfirstlane(P.bins[slot]);
        const TriRecord r = P.records[prim];
        const int bx0 = max((int)(r.bb0 & 0xFFFFu), x0), by0 = max((int)(r.bb0 >> 16), y0);
        const int bx1 = min((int)(r.bb1 & 0xFFFFu), x0 + kTile - 1), by1 = min((int)(r.bb1 >> 16), y0 + kTile - 1);
        const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
        if (bw <= 0 || bh <= 0) continue;
        const int sh = bw <= 1 ? 0 : 32 - __clz(bw - 1);
        const int rows = 64 >> sh;
        const int lx = lane & ((1 << sh) - 1), lyo = lane >> sh;
        const long long bias0 = (r.flags >> 1) & 1, bias1 = (r.flags >> 2) & 1, bias2 = (r.flags >> 3) & 1;
        for (int ry = 0; ry < bh; ry += rows) {
            const int ly = ry + lyo;
            if (lx < bw && ly < bh) {
                const int px = bx0 + lx, py = by0 + ly;
                const EdgeEval e = eval_edges(r, px, py);
                if (e.w0 >= bias0 && e.w1 >= bias1 && e.w2 >= bias2) {
                    const float z = interp_depth(r, e.w1, e.w2);
                    if (z >= P.dlo && z <= P.dhi) {
                        const int li = (py - y0) * kTile + (px - x0);
                        if (!INITD || depth_pass(P.depth_op, z, s_initd[li]))
                            atomicMin(&s_key[li], frag_key<MODE>(z, prim + 1u));
                    }
                }
            }
        }
    }
    __syncthreads();

    for (int i = threadIdx.x; i < kTilePixels; i += kTileThreads) {
        const int px = x0 + (i & (kTile - 1)), py = y0 + (i >> kTileShift);
        if (px < P.ra_x0 || px > P.ra_x1 || py < P.ra_y0 || py > P.ra_y1) continue;
        const unsigned long long key = s_key[i];
        const uint32_t seq = winner_seq<MODE>(key);
        float c[4] = {0.f, 0.f, 0.f, 0.f};
        float zw = 0.0f;
        if (seq) {
            const uint32_t prim = seq - 1u;
            const TriRecord r = P.records[prim];
            const EdgeEval e = eval_edges(r, px, py);
            if (P.color_bpp) shade_winner<PROG>(P, r, prim, e, c);
            zw = (MODE == kDepthLastWins) ? interp_depth(r, e.w1, e.w2) : key_depth<MODE>(key);
        }
        if (P.color_bpp) store_color(P, px, py, seq != 0, c);
        if (P.depth) {
            float* dp = P.depth + (size_t)py * P.fb_w + px;
            if (seq && P.depth_write_out) *dp = zw;
            else if (P.clear_depth_enable) *dp = P.clear_depth;
        }
    }
}

__global__ __launch_bounds__(kTileThreads) void k_clear(DrawParams P) {
    const uint32_t t = blockIdx.x;
    const uint32_t oy = t / P.tiles_x, tx = t - oy * P.tiles_x;
    const uint32_t ty = oy * P.shard_count + P.shard_rank;
    const int x0 = (int)tx * kTile, y0 = (int)ty * kTile;
    const float c[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < kTilePixels; i += kTileThreads) {
        const int px = x0 + (i & (kTile - 1)), py = y0 + (i >> kTileShift);
        if (px < P.ra_x0 || px > P.ra_x1 || py < P.ra_y0 || py > P.ra_y1) continue;
        if (P.color_bpp && P.clear_color_enable) store_color(P, px, py, false, c);
        if (P.depth && P.clear_depth_enable) P.depth[(size_t)py * P.fb_w + px] = P.clear_depth;
    }
}

// ---------------------------------------------------------------- launchers

static inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

void launch_setup(const DrawParams& p, void* stream) {
    if (p.prims == 0) return;
    hipLaunchKernelGGL(k_setup, dim3(blocks_for(p.prims, kSetupThreads)), dim3(kSetupThreads), 0,
                       (hipStream_t)stream, p);
}

void launch_scan(const DrawParams& p, void* stream) {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, (hipStream_t)stream, p);
}

void launch_bin(const DrawParams& p, void* stream) {
    if (p.prims == 0) return;
    hipLaunchKernelGGL(k_bin, dim3(blocks_for(p.prims, kSetupThreads)), dim3(kSetupThreads), 0,
                       (hipStream_t)stream, p);
}

template <int PROG, int MODE>
static void launch_tile_pm(const DrawParams& p, hipStream_t s, bool initd) {
    if (initd)
        hipLaunchKernelGGL((k_tile<PROG, MODE, true>), dim3(p.ntiles), dim3(kTileThreads), 0, s, p);
    else
        hipLaunchKernelGGL((k_tile<PROG, MODE, false>), dim3(p.ntiles), dim3(kTileThreads), 0, s, p);
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
    default: launch_tile_p<kProgBlinn>(p, s, initd); break;
    }
}

void launch_clear(const DrawParams& p, void* stream) {
    if (p.ntiles == 0) return;
    hipLaunchKernelGGL(k_clear, dim3(p.ntiles), dim3(kTileThreads), 0, (hipStream_t)stream, p);
}

}  // namespace zr
