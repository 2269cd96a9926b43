// batcher_conc.cpp -- c uploads arriving at once: the GPU coalescing executor (dm_batcher) against
// the CPU restatement on T threads, driven from native threads (a gin server's goroutines call the
// library through cgo at ~1 us a call; a Python driver adds its own per-request cost on top).
// Measurement tool for INTEGRATION.md's handler guidance; the oracle is only the CPU side and the
// checker.  Every result is compared with the oracle's.
//
// build: hipcc -O2 -std=c++20 -I include tools/batcher_conc.cpp -o tools/batcher_conc
//          -L deoss_amd -ldeoss_merkle -L oracle -loracle_merkle -Wl,-rpath,'$ORIGIN/../deoss_amd:$ORIGIN/../oracle' -lpthread
// usage: tools/batcher_conc <root|process> <request bytes> <cpu threads> <pinned 0|1> <c1> [c2 ...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <barrier>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "deoss_merkle.h"

extern "C" {
void or_fill_splitmix(void* dst, uint64_t off, uint64_t nbytes, uint64_t seed);
int or_root_buffer(const void* buf, uint64_t len, uint64_t chunk, uint8_t* leaf_out, uint8_t root[32], int nthreads);
int64_t or_full_processing(const void* buf, uint64_t len, uint64_t segment, int data, int parity, uint8_t* seg_hashes,
                           uint8_t* frag_hashes, uint8_t fid[32], uint8_t* frags, int nthreads);
}

namespace {

constexpr uint64_t kUnit = 32ull << 20;   // chunk (root) / segment (process)
constexpr int kPool = 64;                  // distinct request bodies, reused round-robin

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s <root|process> <bytes> <cpu threads> <pinned 0|1> <c1> [c2 ...]\n", argv[0]);
        return 2;
    }
    const bool proc = std::string(argv[1]) == "process";
    const uint64_t nbytes = std::strtoull(argv[2], nullptr, 10);
    const int T = std::atoi(argv[3]);
    const bool pinned = std::atoi(argv[4]) != 0;
    std::vector<int> cs;
    for (int i = 5; i < argc; i++) cs.push_back(std::atoi(argv[i]));
    const uint64_t pitch = (nbytes + 4095) / 4096 * 4096;
    uint8_t* pool = nullptr;
    if (pinned) {
        if (dm_host_alloc(pitch * kPool, reinterpret_cast<void**>(&pool)) != DM_OK) return 3;
    } else {
        pool = static_cast<uint8_t*>(std::aligned_alloc(4096, pitch * kPool));
    }
    for (int j = 0; j < kPool; j++) or_fill_splitmix(pool + j * pitch, 0, (nbytes + 7) / 8 * 8, 0xDE0558800ull + j);
    std::vector<std::array<uint8_t, 32>> want(kPool);
    for (int j = 0; j < kPool; j++) {
        if (proc) {
            const uint64_t nseg = (nbytes + kUnit - 1) / kUnit;
            std::vector<uint8_t> sh(32 * nseg), fh(32 * nseg * 12);
            or_full_processing(pool + j * pitch, nbytes, kUnit, 4, 8, sh.data(), fh.data(), want[j].data(), nullptr, 1);
        } else {
            or_root_buffer(pool + j * pitch, nbytes, kUnit, nullptr, want[j].data(), 1);
        }
    }
    dm_batcher* b = nullptr;
    int rc = dm_batcher_create(nullptr, 0, proc ? DM_BATCH_PROCESS : DM_BATCH_ROOT, kUnit, 4, 8, 0, 0, 0, 2000, &b);
    if (rc != DM_OK) {
        std::fprintf(stderr, "dm_batcher_create: %s\n", dm_batcher_last_error());
        return 4;
    }
    auto gpu_wave = [&](int c, bool* ok) {
        std::vector<std::array<uint8_t, 32>> got(c);
        std::barrier go(c + 1);
        std::vector<std::thread> th;
        std::atomic<int> bad{0};
        for (int t = 0; t < c; t++)
            th.emplace_back([&, t] {
                go.arrive_and_wait();
                const uint8_t* src = pool + (t % kPool) * pitch;
                const int r = proc ? dm_batcher_process(b, src, nbytes, nullptr, nullptr, nullptr, got[t].data())
                                   : dm_batcher_root(b, src, nbytes, nullptr, got[t].data());
                if (r != DM_OK || got[t] != want[t % kPool]) bad++;
            });
        go.arrive_and_wait();
        const double t0 = now_ms();
        for (auto& x : th) x.join();
        const double ms = now_ms() - t0;
        *ok = bad == 0;
        return ms;
    };
    auto cpu_wave = [&](int c, bool* ok) {
        std::atomic<int> next{0}, bad{0};
        std::vector<std::thread> th;
        const double t0 = now_ms();
        for (int t = 0; t < T; t++)
            th.emplace_back([&] {
                std::vector<uint8_t> sh(32 * ((nbytes + kUnit - 1) / kUnit)), fh(sh.size() * 12);
                for (int j; (j = next++) < c;) {
                    std::array<uint8_t, 32> r{};
                    const uint8_t* src = pool + (j % kPool) * pitch;
                    if (proc) or_full_processing(src, nbytes, kUnit, 4, 8, sh.data(), fh.data(), r.data(), nullptr, 1);
                    else or_root_buffer(src, nbytes, kUnit, nullptr, r.data(), 1);
                    if (r != want[j % kPool]) bad++;
                }
            });
        for (auto& x : th) x.join();
        *ok = bad == 0;
        return now_ms() - t0;
    };
    bool ok = true, g_ok = true, c_ok = true;
    int maxc = 0;
    for (int c : cs) maxc = std::max(maxc, c);
    gpu_wave(maxc, &g_ok);   // warm every slot's buffers at the largest wave
    std::printf("{\"mode\": \"%s\", \"request_bytes\": %llu, \"bodies\": \"%s\", \"cpu_threads\": %d, \"rows\": [",
                proc ? "process" : "root", (unsigned long long)nbytes, pinned ? "pinned" : "pageable", T);
    int first = -1;
    for (size_t i = 0; i < cs.size(); i++) {
        const double g = gpu_wave(cs[i], &g_ok);
        const double c = cpu_wave(cs[i], &c_ok);
        ok = ok && g_ok && c_ok;
        if (first < 0 && g < c) first = cs[i];
        std::printf("%s{\"concurrent\": %d, \"gpu_ms\": %.2f, \"cpu_ms\": %.2f}", i ? ", " : "", cs[i], g, c);
    }
    uint64_t nreq = 0, nbat = 0, maxb = 0;
    dm_batcher_stats(b, &nreq, &nbat, &maxb);
    std::printf("], \"gpu_faster_from\": %d, \"batches\": %llu, \"largest_batch\": %llu, \"bit_exact\": %s}\n", first,
                (unsigned long long)nbat, (unsigned long long)maxb, ok ? "true" : "false");
    dm_batcher_destroy(b);
    if (pinned) dm_host_free(pool);
    else std::free(pool);
    return ok ? 0 : 1;
}
