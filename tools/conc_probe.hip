// How many long kernels from different streams of one process run at once?  N streams (created
// back to back, normal priority; or alternating normal / high priority with "mixed") each get one
// 100 ms single-workgroup spin kernel, all launched together; the wall time is ~100 ms when all N
// run side by side and ~k x 100 ms when they serialise k-deep.  Prints one line per N.
// usage: conc_probe [mixed]      Build: hipcc --offload-arch=gfx950 -O2 -o tools/conc_probe tools/conc_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void spin(unsigned long long ticks, int* out) {
    const unsigned long long t0 = wall_clock64();   // constant-rate counter (100 MHz)
    unsigned long long t = t0;
    while (t - t0 < ticks) t = wall_clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = (int)(t - t0);
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const bool mixed = argc > 1 && std::strcmp(argv[1], "mixed") == 0;
    int* out = nullptr;
    CK(hipMalloc(&out, 4096));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int n = 1; n <= 8; n++) {
        std::vector<hipStream_t> ss(n);
        for (int i = 0; i < n; i++) {
            if (mixed && i % 2) CK(hipStreamCreateWithPriority(&ss[i], hipStreamNonBlocking, hi));
            else CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
        }
        for (int i = 0; i < n; i++) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, ss[i], 100000ull, out);   // warm
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; i++) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, ss[i], 10000000ull, out + i);
        CK(hipDeviceSynchronize());
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::printf("%s streams=%d wall_ms=%.1f serial_depth=%.2f\n", mixed ? "mixed" : "normal", n, ms, ms / 100.0);
        for (auto s : ss) CK(hipStreamDestroy(s));
    }
    std::printf("done\n");
    return 0;
}
