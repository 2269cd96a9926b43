// Does hipFree / hipMalloc / hipHostFree wait for unrelated work on the device?  One stream runs a
// ~300 ms spin kernel; meanwhile the host times allocator calls (and hipFreeAsync on another
// stream).  If hipFree blocks ~300 ms, every buffer release in a stream's close serialises behind
// other callers' kernels on that GPU (merkle_stream.inl / process_stream.inl free at close).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/free_sync_probe tools/free_sync_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void spin(unsigned long long ticks, int* out) {
    const unsigned long long t0 = wall_clock64();   // constant-rate counter (100 MHz)
    unsigned long long t = t0;
    while (t - t0 < ticks) t = wall_clock64();
    if (threadIdx.x == 0) out[0] = (int)(t - t0);
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    int* out = nullptr;
    CK(hipMalloc(&out, 64));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    const unsigned long long ticks = 30000000ull;   // 300 ms at 100 MHz
    auto run = [&](const char* what, auto fn) -> int {
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, ticks, out);
        CK(hipGetLastError());
        auto t0 = std::chrono::steady_clock::now();
        while (ms_since(t0) < 20) {}   // the spin is surely running
        auto t1 = std::chrono::steady_clock::now();
        const int rc = fn();
        const double call = ms_since(t1);
        CK(hipStreamSynchronize(a));
        std::printf("%-44s %8.2f ms   (spin kernel total %.0f ms)\n", what, call, ms_since(t0));
        return rc;
    };
    void* p = nullptr;
    CK(hipMalloc(&p, 64 << 20));
    if (run("hipFree(64 MiB) while another stream runs", [&] { return (int)hipFree(p); })) return 1;
    if (run("hipMalloc(64 MiB) while another stream runs", [&] { return (int)hipMalloc(&p, 64 << 20); })) return 1;
    if (run("hipFreeAsync(64 MiB, other stream) + sync it", [&] {
            hipError_t e = hipFreeAsync(p, b);
            if (e == hipSuccess) e = hipStreamSynchronize(b);
            return (int)e;
        }))
        return 1;
    if (run("hipMallocAsync(64 MiB, other stream) + sync", [&] {
            hipError_t e = hipMallocAsync(&p, 64 << 20, b);
            if (e == hipSuccess) e = hipStreamSynchronize(b);
            return (int)e;
        }))
        return 1;
    CK(hipFreeAsync(p, b));
    CK(hipStreamSynchronize(b));
    void* h = nullptr;
    CK(hipHostMalloc(&h, 64 << 20, hipHostMallocDefault));
    if (run("hipHostFree(64 MiB pinned) while busy", [&] { return (int)hipHostFree(h); })) return 1;
    if (run("hipHostMalloc(64 MiB) while busy", [&] { return (int)hipHostMalloc(&h, 64 << 20, hipHostMallocDefault); }))
        return 1;
    CK(hipHostFree(h));
    hipEvent_t ev;
    if (run("hipEventCreate + Destroy while busy", [&] {
            hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventDestroy(ev);
            return (int)e;
        }))
        return 1;
    hipStream_t s2;
    if (run("hipStreamCreate + Destroy while busy", [&] {
            hipError_t e = hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipStreamDestroy(s2);
            return (int)e;
        }))
        return 1;
    std::printf("done\n");
    return 0;
}
