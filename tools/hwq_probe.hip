// Which HIP streams share a hardware queue?  With GPU_MAX_HW_QUEUES = 4 (the box's default) a
// process's streams are multiplexed onto a few HSA queues; two streams on one queue execute in
// one FIFO, so a short kernel on stream B waits for a long kernel already queued on stream A.
// The library relies on short work (RS, copies, tree levels) not waiting behind 0.5 s leaf
// chains launched on other streams (fullproc_capi.inl striped pass, the batcher's slots).
//
// For every ordered pair (A, B): a 30 ms spin kernel on A, then (10 ms later) a 1-thread kernel
// on B; B "waits" if its kernel ends after the spin.  Streams: normal, high and low priority, in
// creation order, then the same after destroying some (what a process with earlier contexts sees).
// usage: hwq_probe [high-priority streams (3)] [normal streams (8)]
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/hwq_probe tools/hwq_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <vector>

__global__ void spin(unsigned long long ticks, int* out) {
    const unsigned long long t0 = wall_clock64();   // constant-rate counter (100 MHz)
    unsigned long long t = t0;
    while (t - t0 < ticks) t = wall_clock64();
    if (threadIdx.x == 0) out[0] = (int)(t - t0);
}

__global__ void tiny(int* out) {
    if (threadIdx.x == 0) out[1] += 1;
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

struct Named {
    hipStream_t s;
    std::string name;
};

// 1 if a tiny kernel on b waits for a spin on a; -1 on error
static int waits(hipStream_t a, hipStream_t b, int* out, void* host, void* dev) {
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, 3000000ull, out);   // 30 ms
    if (hipGetLastError() != hipSuccess) return -1;
    auto t0 = std::chrono::steady_clock::now();
    while (ms_since(t0) < 10) {}
    if (host) {
        if (hipMemcpyAsync(dev, host, 4096, hipMemcpyHostToDevice, b) != hipSuccess) return -1;
    } else {
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, b, out);
    }
    while (hipStreamQuery(b) == hipErrorNotReady) {}
    const double tb = ms_since(t0);
    if (hipStreamSynchronize(a) != hipSuccess) return -1;
    return tb > 25.0 ? 1 : 0;
}

static int matrix(const std::vector<Named>& ss, int* out, void* host, void* dev, const char* what) {
    std::printf("\n%s: row = stream with the 30 ms spin, column = stream whose work waits (X)\n%10s", what, "");
    for (auto& c : ss) std::printf(" %4s", c.name.c_str());
    std::printf("\n");
    for (auto& r : ss) {
        std::printf("%10s", r.name.c_str());
        for (auto& c : ss) {
            if (r.s == c.s) {
                std::printf(" %4s", "-");
                continue;
            }
            const int w = waits(r.s, c.s, out, host, dev);
            if (w < 0) return 1;
            std::printf(" %4s", w ? "X" : ".");
        }
        std::printf("\n");
    }
    return 0;
}

int main(int argc, char** argv) {
    const int nhigh = argc > 1 ? std::atoi(argv[1]) : 3;   // high-priority streams to create
    const int nnorm = argc > 2 ? std::atoi(argv[2]) : 8;
    int* out = nullptr;
    void* dev = nullptr;
    void* host = nullptr;
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&dev, 4096));
    CK(hipHostMalloc(&host, 4096, hipHostMallocDefault));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    std::printf("priority range: least %d greatest %d; GPU_MAX_HW_QUEUES=%s\n", lo, hi,
                std::getenv("GPU_MAX_HW_QUEUES") ? std::getenv("GPU_MAX_HW_QUEUES") : "(unset)");
    std::vector<Named> ss;
    for (int i = 0; i < nnorm; i++) {
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        ss.push_back({s, "n" + std::to_string(i)});
    }
    for (int i = 0; i < nhigh; i++) {
        hipStream_t s;
        CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
        ss.push_back({s, "h" + std::to_string(i)});
    }
    for (int i = 0; i < 2; i++) {
        hipStream_t s;
        CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, lo));
        ss.push_back({s, "l" + std::to_string(i)});
    }
    if (matrix(ss, out, nullptr, nullptr, "kernels")) return 1;
    if (matrix(ss, out, host, dev, "4 KiB H2D copy on the column stream")) return 1;
    // destroy n0, n2, n5 and create three more: which queues do the new streams get?
    for (int i : {5, 2, 0}) {
        CK(hipStreamDestroy(ss[i].s));
        ss.erase(ss.begin() + i);
    }
    for (int i = 0; i < 3; i++) {
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        ss.push_back({s, "m" + std::to_string(i)});
    }
    if (matrix(ss, out, nullptr, nullptr, "kernels, after destroying n0 n2 n5 and creating m0 m1 m2")) return 1;
    for (auto& n : ss) CK(hipStreamDestroy(n.s));
    std::printf("done\n");
    return 0;
}
