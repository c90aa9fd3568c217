// pmc_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the
// access shapes of the draw path (MI355X_MICROARCH.md §HBM: only 16-B/lane streaming
// reads are calibrated there).  Each kernel moves a known number of bytes through a
// 1 GiB buffer (4x the 256 MiB Infinity Cache, so re-reads cannot hide):
//   stream16  coalesced 16 B/lane reads            (the guide's calibrated case)
//   stream4   coalesced 4 B/lane reads             (bin lists, depth loads)
//   gather64  64 B/lane (4 x 16 B) at bijectively permuted record slots (TriRecord loads)
//   gather12  12 B/lane at permuted 12-B slots     (float3 vertex attribute loads)
//   store4    coalesced 4 B/lane stores            (colour / depth texels)
//   store64   64 B/lane stores, record layout      (TriRecord writes)
// Build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/build/pmc_calib
// Run:   rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- tools/build/pmc_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

static constexpr size_t kBytes = size_t(1) << 30;

__global__ void stream16(const int4* p, size_t n, unsigned* sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x7fffffff) atomicAdd(sink, 1u);
}

__global__ void stream4(const int* p, size_t n, unsigned* sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x7fffffff) atomicAdd(sink, 1u);
}

// n is a power of two: i * odd mod n is a bijection, every slot read exactly once.
__global__ void gather64(const int4* p, size_t n, unsigned* sink) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const size_t s = (i * 0x9E3779B1ull) & (n - 1);
    const int4* r = p + s * 4;
    const int4 a = r[0], b = r[1], c = r[2], d = r[3];
    const int acc = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ d.x;
    if (acc == 0x7fffffff) atomicAdd(sink, 1u);
}

__global__ void gather12(const float* p, size_t n, unsigned* sink) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const size_t s = (i * 0x9E3779B1ull) & (n - 1);
    const float* r = p + s * 3;
    const float acc = r[0] + r[1] + r[2];
    if (acc == 12345.0f) atomicAdd(sink, 1u);
}

__global__ void store4(int* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (int)i;
}

__global__ void store64(int4* p, size_t n) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    int4* r = p + i * 4;
    const int v = (int)i;
    r[0] = make_int4(v, v, v, v); r[1] = r[0]; r[2] = r[0]; r[3] = r[0];
}

int main() {
    char* buf = nullptr;
    unsigned* sink = nullptr;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(buf, 1, kBytes));
    CHECK(hipMemset(sink, 0, 4));
    CHECK(hipDeviceSynchronize());
    const int grid = 256 * 8 * 4;
    const size_t n16 = kBytes / 16, n4 = kBytes / 4, n64 = kBytes / 64;
    size_t n12 = 1;
    while (n12 * 2 * 12 <= kBytes) n12 *= 2;  // power of two slots of 12 B
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(stream16, dim3(grid), dim3(256), 0, 0, (const int4*)buf, n16, sink);
        hipLaunchKernelGGL(stream4, dim3(grid), dim3(256), 0, 0, (const int*)buf, n4, sink);
        hipLaunchKernelGGL(gather64, dim3((unsigned)(n64 / 256)), dim3(256), 0, 0, (const int4*)buf, n64, sink);
        hipLaunchKernelGGL(gather12, dim3((unsigned)(n12 / 256)), dim3(256), 0, 0, (const float*)buf, n12, sink);
        hipLaunchKernelGGL(store4, dim3(grid), dim3(256), 0, 0, (int*)buf, n4);
        hipLaunchKernelGGL(store64, dim3((unsigned)(n64 / 256)), dim3(256), 0, 0, (int4*)buf, n64);
    }
    CHECK(hipDeviceSynchronize());
    printf("{\"stream16\": %zu, \"stream4\": %zu, \"gather64\": %zu, \"gather12\": %zu, \"store4\": %zu, "
           "\"store64\": %zu}\n", kBytes, kBytes, kBytes, n12 * 12, kBytes, kBytes);
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
