// How many long kernels from different streams of one process run at once?  N streams (created
// back to back, normal priority; or alternating normal / high priority with "mixed") each get one
// 100 ms single-workgroup spin kernel, all launched together; the wall time is ~100 ms when all N
// run side by side and ~k x 100 ms when they serialise k-deep.  Prints one line per N.
// usage: conc_probe [normal|mixed|lds|lanes|cumask]      Build: hipcc --offload-arch=gfx950 -O2 -o tools/conc_probe tools/conc_probe.hip
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

// K1Q-shaped: 32 workgroups of 128 threads, each holding 64 KiB of dynamic LDS (<= 2 per CU)
__global__ void spin_lds(unsigned long long ticks, int* out) {
    extern __shared__ int lds[];
    const unsigned long long t0 = wall_clock64();
    unsigned long long t = t0;
    lds[threadIdx.x] = (int)threadIdx.x;
    while (t - t0 < ticks) t = wall_clock64();
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (int)(t - t0) + lds[5];
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
    // modes: normal | mixed (alternate normal / high) | lds (K1Q-shaped kernels) |
    //        lanes (K1Q-shaped kernels; every compute stream followed by an idle lowest-priority stream)
    const char* mode = argc > 1 ? argv[1] : "normal";
    const bool mixed = std::strcmp(mode, "mixed") == 0;
    const bool lds = std::strcmp(mode, "lds") == 0 || std::strcmp(mode, "lanes") == 0 || std::strcmp(mode, "cumask") == 0;
    const bool lanes = std::strcmp(mode, "lanes") == 0;
    // cumask: K1Q-shaped kernels on streams made by hipExtStreamCreateWithCUMask (every CU enabled),
    // after 8 ordinary streams were created first (the queue pool already full)
    const bool cumask = std::strcmp(mode, "cumask") == 0;
    std::vector<hipStream_t> filler;
    if (cumask)
        for (int i = 0; i < 8; i++) {
            hipStream_t x;
            CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
            filler.push_back(x);
        }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> full((cus + 31) / 32, 0xffffffffu);
    int* out = nullptr;
    CK(hipMalloc(&out, 4096));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int n = 1; n <= 8; n++) {
        std::vector<hipStream_t> ss(n), idle;
        for (int i = 0; i < n; i++) {
            if (mixed && i % 2) CK(hipStreamCreateWithPriority(&ss[i], hipStreamNonBlocking, hi));
            else if (cumask) CK(hipExtStreamCreateWithCUMask(&ss[i], (uint32_t)full.size(), full.data()));
            else CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
            if (lanes) {
                hipStream_t x;
                CK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, lo));
                idle.push_back(x);
            }
        }
        auto launch = [&](int i, unsigned long long ticks) {
            if (lds) hipLaunchKernelGGL(spin_lds, dim3(32), dim3(128), 64 << 10, ss[i], ticks, out + 32 * i);
            else hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, ss[i], ticks, out + i);
        };
        for (int i = 0; i < n; i++) launch(i, 100000ull);   // warm
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; i++) launch(i, 10000000ull);
        CK(hipDeviceSynchronize());
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::printf("%s streams=%d wall_ms=%.1f serial_depth=%.2f\n", mode, n, ms, ms / 100.0);
        for (auto s : ss) CK(hipStreamDestroy(s));
        for (auto s : idle) CK(hipStreamDestroy(s));
    }
    for (auto s : filler) CK(hipStreamDestroy(s));
    std::printf("done\n");
    return 0;
}
