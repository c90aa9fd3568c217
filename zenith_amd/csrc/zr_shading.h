// zr_shading.h — fragment-stage arithmetic of the built-in programs and the colour
// output encodings.  Host+device: the runtime uses the
// encoders for clear values, the kernels for fragments.  Every float op is
// written out (explicit fmaf, -ffp-contract=off) so results are bit-identical to
// the CPU oracle's independent restatement (oracle/zr_oracle.c).
#pragma once
#include <stdint.h>
#include <math.h>

#include "zr_srgb_table.h"

#if defined(__HIPCC__)
#define ZR_HD __host__ __device__ __forceinline__
#else
#define ZR_HD inline
#endif

namespace zr {

enum : int32_t {
    kFmtR8G8B8A8Unorm = 37,
    kFmtR8G8B8A8Srgb = 43,
    kFmtB8G8R8A8Unorm = 44,
    kFmtB8G8R8A8Srgb = 50,
    kFmtR32G32B32A32Sfloat = 109,
    kFmtD32Sfloat = 126,
};

// sin() of triangle.slang:36 (content/shaders).  Pinned implementation: 3-part
// Cody-Waite reduction by pi/2 + Taylor polynomials on [-pi/4, pi/4].
ZR_HD float zr_sinf(float x) {
    const float q = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(q, -0x1.921fb6p+0f, x);
    r = fmaf(q, 0x1.777a5cp-25f, r);
    r = fmaf(q, 0x1.0p-49f, r);
    const int qi = ((int)q) & 3;
    const float r2 = r * r;
    float s = fmaf(r2, -0x1.ae64568p-26f, 0x1.71de3a6p-19f);
    s = fmaf(r2, s, -0x1.a01a01ap-13f);
    s = fmaf(r2, s, 0x1.111112p-7f);
    s = fmaf(r2, s, -0x1.555556p-3f);
    s = fmaf(r2 * r, s, r);
    float c = fmaf(r2, 0x1.1ee9ebp-29f, -0x1.27e4fbp-22f);
    c = fmaf(r2, c, 0x1.a01a01ap-16f);
    c = fmaf(r2, c, -0x1.6c16c16p-10f);
    c = fmaf(r2, c, 0x1.555556p-5f);
    c = fmaf(r2, c, -0.5f);
    c = fmaf(r2, c, 1.0f);
    const float v = (qi & 1) ? c : s;
    return (qi & 2) ? -v : v;
}

ZR_HD float clamp01(float c) {
    if (!(c > 0.0f)) return 0.0f;  // NaN -> 0
    return c > 1.0f ? 1.0f : c;
}

ZR_HD uint32_t encode_unorm8(float c) { return (uint32_t)rintf(clamp01(c) * 255.0f); }

// Correctly-rounded sRGB encode: count of thresholds <= c (8-step bisection).
ZR_HD uint32_t encode_srgb8(float c, const float* T) {
    c = clamp01(c);
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 128; step > 0; step >>= 1) {
        const uint32_t probe = lo + step - 1;  // thresholds T[0..probe] all <= c ?
        if (probe < 255 && c >= T[probe]) lo += step;
    }
    return lo;
}

ZR_HD bool format_is_srgb(int32_t f) { return f == kFmtB8G8R8A8Srgb || f == kFmtR8G8B8A8Srgb; }
ZR_HD bool format_is_bgra(int32_t f) { return f == kFmtB8G8R8A8Srgb || f == kFmtB8G8R8A8Unorm; }
ZR_HD uint32_t format_bpp(int32_t f) {
    switch (f) {
    case kFmtR8G8B8A8Unorm: case kFmtR8G8B8A8Srgb: case kFmtB8G8R8A8Unorm: case kFmtB8G8R8A8Srgb: return 4;
    case kFmtR32G32B32A32Sfloat: return 16;
    default: return 0;
    }
}

// Packs RGBA (linear float) into one 32-bit texel of an 8-bit format.
ZR_HD uint32_t pack_rgba8(const float c[4], int32_t fmt, const float* T) {
    const bool srgb = format_is_srgb(fmt);
    uint32_t r = srgb ? encode_srgb8(c[0], T) : encode_unorm8(c[0]);
    uint32_t g = srgb ? encode_srgb8(c[1], T) : encode_unorm8(c[1]);
    uint32_t b = srgb ? encode_srgb8(c[2], T) : encode_unorm8(c[2]);
    uint32_t a = encode_unorm8(c[3]);  // sRGB formats keep alpha linear
    return format_is_bgra(fmt) ? (b | (g << 8) | (r << 16) | (a << 24)) : (r | (g << 8) | (b << 16) | (a << 24));
}

#if defined(__HIPCC__)
// Device fast path with the same result as encode_srgb8: estimate the code with
// the hardware log2/exp2, then move it onto the threshold table (T in LDS) until
// T[k-1] <= c < T[k].  The estimate is within one code of the exact result; two
// fix-up rounds make the result exact by construction (the table defines it).
__device__ __forceinline__ uint32_t encode_srgb8_fast(float c, const float* T) {
    c = clamp01(c);
    const float e = c <= 0.0031308f ? c * 12.92f : fmaf(1.055f, __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(c) * (1.0f / 2.4f)), -0.055f);
    int k = (int)fmaf(e, 255.0f, 0.5f);
    k = k < 0 ? 0 : (k > 255 ? 255 : k);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const float lo = k > 0 ? T[k - 1] : -1.0f;
        const float hi = k < 255 ? T[k] : 2.0f;
        k += (c >= hi) ? 1 : 0;
        k -= (c < lo) ? 1 : 0;
    }
    return (uint32_t)k;
}

__device__ __forceinline__ uint32_t pack_rgba8_fast(const float c[4], int32_t fmt, const float* T) {
    const bool srgb = format_is_srgb(fmt);
    const uint32_t r = srgb ? encode_srgb8_fast(c[0], T) : encode_unorm8(c[0]);
    const uint32_t g = srgb ? encode_srgb8_fast(c[1], T) : encode_unorm8(c[1]);
    const uint32_t b = srgb ? encode_srgb8_fast(c[2], T) : encode_unorm8(c[2]);
    const uint32_t a = encode_unorm8(c[3]);
    return format_is_bgra(fmt) ? (b | (g << 8) | (r << 16) | (a << 24)) : (r | (g << 8) | (b << 16) | (a << 24));
}
#endif

// Byte mask of the 32-bit texel selected by a VkColorComponentFlags write mask.
ZR_HD uint32_t rgba8_write_mask(uint32_t mask, int32_t fmt) {
    const uint32_t rpos = format_is_bgra(fmt) ? 16u : 0u, bpos = format_is_bgra(fmt) ? 0u : 16u;
    uint32_t m = 0;
    if (mask & 1u) m |= 0xFFu << rpos;
    if (mask & 2u) m |= 0xFFu << 8;
    if (mask & 4u) m |= 0xFFu << bpos;
    if (mask & 8u) m |= 0xFFu << 24;
    return m;
}

ZR_HD float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return (ax * bx + ay * by) + az * bz;
}

// triangle.slang:34-38 psmain (per channel).
ZR_HD float shade_triangle_channel(float c, float t3) {
    const float arg = t3 + c * 6.28f;
    return c * (0.5f + 0.5f * zr_sinf(arg));
}

// blinn_phong.slang psmain: kd = colour, ks = 0.5, n = 32, ambient 0.05,
// L = normalize(0.3,0.5,0.8), V = (0,0,1), H = normalize(L+V).
ZR_HD void shade_blinn_phong(float nx, float ny, float nz, float kr, float kg, float kb, float out[4]) {
    const float Lx = 0x1.3651a0p-2f, Ly = 0x1.02995cp-1f, Lz = 0x1.9dc22cp-1f;
    const float Hx = 0x1.465e8ap-3f, Hy = 0x1.0ff974p-2f, Hz = 0x1.e6d20ap-1f;
    const float len2 = dot3(nx, ny, nz, nx, ny, nz);
    const float rl = len2 > 0.0f ? 1.0f / sqrtf(len2) : 0.0f;
    const float Nx = nx * rl, Ny = ny * rl, Nz = nz * rl;
    float ndl = dot3(Nx, Ny, Nz, Lx, Ly, Lz);
    float ndh = dot3(Nx, Ny, Nz, Hx, Hy, Hz);
    ndl = ndl > 0.0f ? ndl : 0.0f;
    ndh = ndh > 0.0f ? ndh : 0.0f;
    float sp = ndh * ndh;
    sp = sp * sp;
    sp = sp * sp;
    sp = sp * sp;
    sp = sp * sp;
    const float amb = 0.05f + ndl;
    out[0] = kr * amb + 0.5f * sp;
    out[1] = kg * amb + 0.5f * sp;
    out[2] = kb * amb + 0.5f * sp;
    out[3] = 1.0f;
}

}  // namespace zr
