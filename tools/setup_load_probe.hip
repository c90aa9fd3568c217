// setup_load_probe.hip -- how k_setup_bin's phase-1 loads could be issued
// (docs/EXPERIMENTS.md, round 5).  C2's geometry: 1M triangles, a 36-B vertex
// (position at offset 0), u32 indices 0..3N-1.  Each kernel reads every
// triangle's three positions once; the results are folded into one word per
// wave so nothing is dead.  Warm (the 120 MB stay in the Infinity Cache) and
// cold (eight copies cycled) timings, hipEvents over the launches.
//
//   gather   one lane per triangle: a 12-B index load, then three 12-B
//            position loads at stride 108 B (what phase 1 does today)
//   stream   the same bytes as a coalesced 16-B-per-lane stream (a floor)
//   span     one lane per triangle for the indices; the wave's vertex id range
//            [vmin, vmax] (a wave reduction) is loaded coalesced, 16 B per lane,
//            into a per-wave LDS slot, and each lane reads its positions there;
//            a wave whose range does not fit gathers as before
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

constexpr int kThreads = 1024;
constexpr int kStrideDw = 9;  // 36-B vertex

__global__ __launch_bounds__(kThreads) void k_gather(const float* vb, const uint32_t* ib, uint32_t n, uint32_t* out) {
    float acc = 0.f;
    for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < n; t += gridDim.x * kThreads) {
        const uint3 ix = *reinterpret_cast<const uint3*>(ib + 3ull * t);
        const float3 a = *reinterpret_cast<const float3*>(vb + (size_t)ix.x * kStrideDw);
        const float3 b = *reinterpret_cast<const float3*>(vb + (size_t)ix.y * kStrideDw);
        const float3 c = *reinterpret_cast<const float3*>(vb + (size_t)ix.z * kStrideDw);
        acc += a.x + a.y + a.z + b.x + b.y + b.z + c.x + c.y + c.z;
    }
    if (acc == 123.25f) out[blockIdx.x] = 1;
}

__global__ __launch_bounds__(kThreads) void k_stream(const float4* p, size_t n4, uint32_t* out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n4; i += (size_t)gridDim.x * kThreads) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 123.25f) out[blockIdx.x] = 1;
}

template <int SLOT_DW, int NT>
__global__ __launch_bounds__(NT) void k_span(const float* vb, const uint32_t* ib, uint32_t n, uint32_t* out) {
    __shared__ float s_slot[NT / 64][SLOT_DW];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    float* slot = s_slot[wave];
    float acc = 0.f;
    // a wave takes 64 consecutive triangles per round
    for (uint32_t base = (blockIdx.x * (NT / 64) + wave) * 64u; base < n; base += gridDim.x * NT) {
        const uint32_t t = base + lane;
        const bool ok = t < n;
        uint3 ix = make_uint3(0, 0, 0);
        if (ok) ix = *reinterpret_cast<const uint3*>(ib + 3ull * t);
        uint32_t lo = ok ? min(ix.x, min(ix.y, ix.z)) : 0xFFFFFFFFu, hi = ok ? max(ix.x, max(ix.y, ix.z)) : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        hi = __builtin_amdgcn_readfirstlane(hi);
        // the range's dwords, from a 16-B-aligned start
        const uint64_t d0 = (uint64_t)lo * kStrideDw, d1 = (uint64_t)hi * kStrideDw + 3u;  // [d0, d1)
        const uint64_t a0 = d0 & ~3ull;
        const uint32_t ndw = (uint32_t)(d1 - a0);
        float3 p[3];
        if (lo <= hi && ndw <= (uint32_t)SLOT_DW) {
            const float4* src = reinterpret_cast<const float4*>(vb + a0);
            for (uint32_t q = lane; q * 4u < ndw; q += 64u) reinterpret_cast<float4*>(slot)[q] = src[q];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t v[3] = {ix.x, ix.y, ix.z};
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t o = (uint32_t)((uint64_t)v[k] * kStrideDw - a0);
                p[k] = make_float3(slot[o], slot[o + 1], slot[o + 2]);
            }
            __builtin_amdgcn_wave_barrier();
        } else {
            p[0] = *reinterpret_cast<const float3*>(vb + (size_t)ix.x * kStrideDw);
            p[1] = *reinterpret_cast<const float3*>(vb + (size_t)ix.y * kStrideDw);
            p[2] = *reinterpret_cast<const float3*>(vb + (size_t)ix.z * kStrideDw);
        }
        if (ok) acc += p[0].x + p[0].y + p[0].z + p[1].x + p[1].y + p[1].z + p[2].x + p[2].y + p[2].z;
    }
    if (acc == 123.25f) out[blockIdx.x] = 1;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000u;
    const int copies = 8, reps = 20;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t vb_dw = (size_t)3 * n * kStrideDw + 4, ib_n = (size_t)3 * n;
    std::vector<float> hv(vb_dw);
    for (size_t i = 0; i < vb_dw; ++i) hv[i] = (float)(i % 97) * 0.01f;
    std::vector<uint32_t> hi(ib_n);
    for (size_t i = 0; i < ib_n; ++i) hi[i] = (uint32_t)i;
    float* vb[copies];
    uint32_t* ib[copies];
    for (int c = 0; c < copies; ++c) {
        CHECK(hipMalloc(&vb[c], vb_dw * 4));
        CHECK(hipMalloc(&ib[c], ib_n * 4));
        CHECK(hipMemcpy(vb[c], hv.data(), vb_dw * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(ib[c], hi.data(), ib_n * 4, hipMemcpyHostToDevice));
    }
    uint32_t* out;
    CHECK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double bytes = (double)vb_dw * 4 + (double)ib_n * 4;
    auto run = [&](const char* name, auto launch) {
        for (int cold = 0; cold < 2; ++cold) {
            for (int w = 0; w < 3; ++w) launch(0);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r) launch(cold ? r % copies : 0);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / reps;
            printf("%-10s %-4s %8.2f us  %7.1f GB/s (input bytes %.1f MB)\n", name, cold ? "cold" : "warm", us,
                   bytes / (us * 1e-6) / 1e9, bytes / 1e6);
        }
    };
    for (int wpc : {1, 2, 4}) {
        const int grid = cus * wpc;
        printf("-- grid %d x %d threads\n", grid, kThreads);
        run("gather", [&](int c) { hipLaunchKernelGGL(k_gather, dim3(grid), dim3(kThreads), 0, 0, vb[c], ib[c], n, out); });
        run("stream", [&](int c) {
            hipLaunchKernelGGL(k_stream, dim3(grid), dim3(kThreads), 0, 0, reinterpret_cast<const float4*>(vb[c]),
                               (vb_dw * 4) / 16, out);
        });
        // 8 waves x 7 KB of LDS slots per 512-thread workgroup
        run("span", [&](int c) {
            hipLaunchKernelGGL((k_span<1744, 512>), dim3(2 * grid), dim3(512), 0, 0, vb[c], ib[c], n, out);
        });
    }
    printf("probe ok\n");
    return 0;
}
