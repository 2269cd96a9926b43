// A/B of streaming-read kernel shapes for dm_read_probe_async (the measured HBM read peak the
// bench reports).  Each variant XORs every 8-byte word of an 8 GiB buffer; prints GB/s and
// checks all variants agree.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/read_peak_ab tools/read_peak_ab.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u4 gu4;

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                \
            return 1;                                                         \
        }                                                                     \
    } while (0)

__device__ void finish(u4 a, uint64_t* out) {
    uint64_t v = (((uint64_t)a.y << 32) | a.x) ^ (((uint64_t)a.w << 32) | a.z);
    for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
    __shared__ uint64_t part[16];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (unsigned w = 0; w < blockDim.x / 64; w++) t ^= part[w];
        atomicXor(reinterpret_cast<unsigned long long*>(out), (unsigned long long)t);
    }
}

// grid-stride, U independent loads in flight per lane
template <int U>
__global__ __launch_bounds__(256) void stride_k(const uint8_t* p, uint64_t n16, uint64_t* out) {
    gu4* g = (gu4*)p;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    u4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = u4{0, 0, 0, 0};
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u4 x[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = g[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] ^= x[u];
    }
    for (; i < n16; i += stride) acc[0] ^= g[i];
#pragma unroll
    for (int u = 1; u < U; u++) acc[0] ^= acc[u];
    finish(acc[0], out);
}

// contiguous slab per workgroup, U loads in flight per lane (block-contiguous 4 KiB per load round)
template <int U>
__global__ __launch_bounds__(256) void slab_k(const uint8_t* p, uint64_t n16, uint64_t* out) {
    gu4* g = (gu4*)p;
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < n16 ? lo + per : n16;
    u4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = u4{0, 0, 0, 0};
    uint64_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 256 < hi; i += U * 256) {
        u4 x[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = g[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] ^= x[u];
    }
    for (; i < hi; i += 256) acc[0] ^= g[i];
#pragma unroll
    for (int u = 1; u < U; u++) acc[0] ^= acc[u];
    finish(acc[0], out);
}

// slab8 with nontemporal loads
template <int U>
__global__ __launch_bounds__(256) void slab_nt_k(const uint8_t* p, uint64_t n16, uint64_t* out) {
    const u4* g = (const u4*)p;
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < n16 ? lo + per : n16;
    u4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = u4{0, 0, 0, 0};
    uint64_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 256 < hi; i += U * 256) {
        u4 x[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = __builtin_nontemporal_load(g + i + u * 256);
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] ^= x[u];
    }
    for (; i < hi; i += 256) acc[0] ^= g[i];
#pragma unroll
    for (int u = 1; u < U; u++) acc[0] ^= acc[u];
    finish(acc[0], out);
}

typedef void (*Kern)(const uint8_t*, uint64_t, uint64_t*);

int main() {
    const uint64_t nbytes = 8ull << 30, n16 = nbytes / 16;
    uint8_t* buf;
    uint64_t* out;
    CHECK(hipMalloc(&buf, nbytes));
    CHECK(hipMalloc(&out, 8));
    CHECK(hipMemset(buf, 0x5a, nbytes));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct V {
        const char* name;
        Kern k;
        int per_cu;
    };
    std::vector<V> vs = {
        {"stride4 x8/CU (current)", stride_k<4>, 8},  {"stride4 x16/CU", stride_k<4>, 16},
        {"stride8 x8/CU", stride_k<8>, 8},            {"stride8 x16/CU", stride_k<8>, 16},
        {"stride2 x32/CU", stride_k<2>, 32},          {"slab4 x8/CU", slab_k<4>, 8},
        {"slab8 x8/CU", slab_k<8>, 8},                {"slab8 x16/CU", slab_k<8>, 16},
        {"slab4 x32/CU", slab_k<4>, 32},      {"slab16 x8/CU", slab_k<16>, 8},
        {"slab8 x32/CU", slab_k<8>, 32},      {"slab8nt x16/CU", slab_nt_k<8>, 16},
        {"slab4nt x32/CU", slab_nt_k<4>, 32}, {"slab16nt x8/CU", slab_nt_k<16>, 8},
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; rep++)
        for (auto& v : vs) {
            const unsigned grid = (unsigned)(v.per_cu * cus);
            CHECK(hipMemset(out, 0, 8));
            hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, buf, n16, out);
            CHECK(hipDeviceSynchronize());
            uint64_t x = 0;
            CHECK(hipMemcpy(&x, out, 8, hipMemcpyDeviceToHost));
            CHECK(hipEventRecord(e0, 0));
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, buf, n16, out);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 5;
            std::printf("rep %d  %-26s %8.1f GB/s  (%.3f ms)  xor %016llx\n", rep, v.name, nbytes / (ms * 1e-3) / 1e9, ms,
                        (unsigned long long)x);
        }
    return 0;
}
