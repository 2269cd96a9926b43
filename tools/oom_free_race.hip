// Does a hipMalloc that runs out of device memory crash the HSA runtime -- by itself, or only while
// another thread's hipFree of a large block is still pending behind a running kernel?
//
// Round 4 saw four segfaults in libhsa-runtime64 (pthread_mutex_lock) under hipMalloc, called from
// DevBuf::ensure while the context reaper's hipFree of the lane's old 4 GiB block was waiting for a
// 0.5 s chain on another stream, with free HBM below the request (tests/test_runtime_gpu.py,
// test_lane_growth_near_full_hbm_waits_for_deferred_frees).  This isolates the two conditions:
//
//   phase 1 "oom":     no pending free.  Free HBM ~5 GiB, hipMalloc(6 GiB) x kReps.
//   phase 2 "race":    thread A queues a ~400 ms spin kernel, then hipFree(4 GiB) (blocks until the
//                      kernel ends); thread B, once A is inside hipFree, calls hipMalloc(6 GiB) with
//                      ~5 GiB free.  x kReps.
//   phase 3 "locked":  phase 2 with one mutex held around A's hipFree and B's (pre-checked) hipMalloc
//                      -- the discipline merkle_capi.hip's DevAlloc enforces.  x kReps.
//
// Every phase prints its verdict line before the next starts, so a crash names its phase.
// Built two ways (tools/oom_free_race.sh): a plain executable, and a shared object whose
// oom_free_race(phase_mask) is called from a process that has initialised torch (the round-4
// crash went through libroctracer64, which torch's HIP loads).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace {

__global__ void spin(unsigned long long ticks, int* out) {
    const unsigned long long t0 = wall_clock64();   // constant-rate counter (100 MHz)
    unsigned long long t = t0;
    while (t - t0 < ticks) t = wall_clock64();
    if (threadIdx.x == 0) out[0] = (int)(t - t0);
}

constexpr size_t GiB = 1ull << 30;
constexpr int kReps = 5;
constexpr unsigned long long kSpinTicks = 40000000ull;   // 400 ms at 100 MHz

size_t free_now() {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) (void)hipGetLastError();
    return fr;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Hog device memory until about `leave` bytes remain free; returns the blocks.
std::vector<void*> hog_until(size_t leave) {
    std::vector<void*> v;
    for (int i = 0; i < 512; i++) {
        const size_t fr = free_now();
        if (fr <= leave + (64ull << 20)) break;
        size_t take = fr - leave;
        if (take > 8 * GiB) take = 8 * GiB;
        void* p = nullptr;
        if (hipMalloc(&p, take) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        v.push_back(p);
    }
    return v;
}

void release(std::vector<void*>& v) {
    for (void* p : v) (void)hipFree(p);
    v.clear();
}

int phase_oom() {
    const auto tp = std::chrono::steady_clock::now();
    std::vector<void*> hog = hog_until(5 * GiB);
    std::printf("  oom: hog taken in %.0f ms\n", ms_since(tp));
    std::fflush(stdout);
    int ooms = 0, oks = 0;
    for (int r = 0; r < kReps; r++) {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, 6 * GiB);
        if (e == hipSuccess) {
            oks++;
            (void)hipFree(p);
        } else {
            ooms++;
            (void)hipGetLastError();
        }
    }
    std::printf("phase oom: free before %.2f GiB, hipMalloc(6 GiB) x%d -> %d out-of-memory, %d ok, no crash\n",
                (double)free_now() / GiB, kReps, ooms, oks);
    std::fflush(stdout);
    release(hog);
    return 0;
}

int phase_race(bool locked) {
    int* out = nullptr;
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    std::mutex mu;
    int ooms = 0, oks = 0, skipped = 0;
    double worst_wait = 0;
    // the hog is taken once per phase (clearing ~280 GiB of fresh VRAM per repetition is slow)
    std::vector<void*> hog = hog_until(9 * GiB);
    const auto tp = std::chrono::steady_clock::now();
    for (int r = 0; r < kReps; r++) {
        void* old = nullptr;
        if (hipMalloc(&old, 4 * GiB) != hipSuccess) return 1;   // leaves ~5 GiB free
        std::atomic<int> in_free{0};
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, kSpinTicks, out);
        if (hipGetLastError() != hipSuccess) return 1;
        std::thread a([&] {
            (void)hipSetDevice(0);
            if (locked) {
                std::lock_guard<std::mutex> lk(mu);
                in_free = 1;
                (void)hipFree(old);   // waits for the spin kernel
            } else {
                in_free = 1;
                (void)hipFree(old);
            }
        });
        while (!in_free.load()) std::this_thread::yield();
        std::this_thread::sleep_for(std::chrono::milliseconds(30));   // A is inside hipFree
        auto t0 = std::chrono::steady_clock::now();
        void* p = nullptr;
        hipError_t e;
        if (locked) {
            std::lock_guard<std::mutex> lk(mu);
            worst_wait = std::max(worst_wait, ms_since(t0));
            if (free_now() < 6 * GiB + (256ull << 20)) {
                e = hipErrorOutOfMemory;   // never ask for what is not free
                skipped++;
            } else {
                e = hipMalloc(&p, 6 * GiB);
            }
        } else {
            e = hipMalloc(&p, 6 * GiB);
        }
        if (e == hipSuccess) {
            oks++;
        } else {
            ooms++;
            (void)hipGetLastError();
        }
        a.join();
        if (p) (void)hipFree(p);
        (void)hipStreamSynchronize(s);
        std::printf("  %s rep %d: %s, %.0f ms into the phase\n", locked ? "locked" : "race", r,
                    e == hipSuccess ? "allocated" : "out of memory", ms_since(tp));
        std::fflush(stdout);
    }
    release(hog);
    std::printf("phase %s: hipMalloc(6 GiB) during a pending hipFree(4 GiB) x%d -> %d ok, %d out-of-memory "
                "(%d declined by the free-memory check), worst lock wait %.0f ms, %.0f ms, no crash\n",
                locked ? "locked" : "race", kReps, oks, ooms, skipped, worst_wait, ms_since(tp));
    std::fflush(stdout);
    (void)hipStreamDestroy(s);
    (void)hipFree(out);
    return 0;
}

}  // namespace

extern "C" int oom_free_race(int mask) {
    if (hipSetDevice(0) != hipSuccess) return 1;
    std::printf("device 0: %.2f GiB free at start\n", (double)free_now() / GiB);
    std::fflush(stdout);
    if ((mask & 1) && phase_oom()) return 1;
    if ((mask & 2) && phase_race(false)) return 1;
    if ((mask & 4) && phase_race(true)) return 1;
    return 0;
}

#ifdef OOM_RACE_MAIN
int main(int argc, char** argv) { return oom_free_race(argc > 1 ? std::atoi(argv[1]) : 7); }
#endif
