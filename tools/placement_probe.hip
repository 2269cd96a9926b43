// placement_probe.hip -- where the dispatcher puts the waves of K1Q-shaped workgroups on gfx950.
//
// Question: in the compact K1Q launch (128-thread workgroups = producer wave 0 + consumer wave 1,
// 33 KiB of LDS, four workgroups per CU; 8,192 leaves = 1,024 workgroups) does every SIMD get one
// consumer, or do consumers pair up on some SIMDs while producers pair up on others?  Each wave
// reads HW_ID (SIMD, CU, SH, SE) and XCC_ID, spins long enough for the whole grid to be resident,
// and stores what it saw (vector stores).  Prints JSON: the per-SIMD count of wave-1s (consumers)
// over every (XCC, SE, SH, CU, SIMD) that held a wave.  Also the wide shape (64 KiB, <= 2 per CU).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/placement_probe tools/placement_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int LDS_UINT4>
__global__ __launch_bounds__(128) void probe(uint32_t* out, int spin) {
    __shared__ uint4 lds[LDS_UINT4];
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint32_t wave = threadIdx.x >> 6;
    // keep the wave resident (and the LDS allocation live) for a while
    uint32_t acc = threadIdx.x;
    const uint64_t t0 = __builtin_readcyclecounter();
    while ((int64_t)(__builtin_readcyclecounter() - t0) < (int64_t)spin) {
        lds[threadIdx.x % LDS_UINT4] = make_uint4(acc, acc, acc, acc);
        acc = acc * 1664525u + lds[(threadIdx.x + 1) % LDS_UINT4].x;
    }
    if ((threadIdx.x & 63) == 0) {
        uint32_t* o = out + 4 * (blockIdx.x * 2 + wave);
        o[0] = hw;
        o[1] = xcc;
        o[2] = wave;
        o[3] = acc == 0x12345678u ? 1u : 0u;
    }
}

template <int LDS_UINT4>
int run(const char* name, int wgs, int spin, bool last) {
    uint32_t* d = nullptr;
    CHK(hipMalloc(&d, (size_t)wgs * 2 * 16));
    CHK(hipMemset(d, 0xff, (size_t)wgs * 2 * 16));
    probe<LDS_UINT4><<<wgs, 128>>>(d, spin);
    CHK(hipDeviceSynchronize());
    std::vector<uint32_t> h((size_t)wgs * 8);
    CHK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    CHK(hipFree(d));
    // key: (xcc, se, sh, cu, simd) -> (consumers, producers)
    std::map<std::tuple<int, int, int, int, int>, std::pair<int, int>> m;
    std::map<std::tuple<int, int, int, int>, int> wg_per_cu;
    int same_simd = 0;
    for (int b = 0; b < wgs; b++) {
        int simd_of[2] = {-1, -1};
        std::tuple<int, int, int, int> cu_of;
        for (int w = 0; w < 2; w++) {
            const uint32_t* o = &h[(size_t)(b * 2 + w) * 4];
            const uint32_t hw = o[0], xcc = o[1] & 0xf;
            const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            auto& e = m[{(int)xcc, se, sh, cu, simd}];
            if (w == 1) e.first++;
            else e.second++;
            simd_of[w] = simd;
            cu_of = {(int)xcc, se, sh, cu};
        }
        wg_per_cu[cu_of]++;
        if (simd_of[0] == simd_of[1]) same_simd++;
    }
    std::map<std::pair<int, int>, int> hist;   // (consumers, producers) on one SIMD -> SIMDs
    for (auto& kv : m) hist[kv.second]++;
    std::map<int, int> cu_hist;
    for (auto& kv : wg_per_cu) cu_hist[kv.second]++;
    printf("  \"%s\": {\"workgroups\": %d, \"simds_used\": %zu, \"cus_used\": %zu, \"wg_both_waves_same_simd\": %d, "
           "\"simds_by_consumers_producers\": {",
           name, wgs, m.size(), wg_per_cu.size(), same_simd);
    bool first = true;
    for (auto& kv : hist) {
        printf("%s\"%dC+%dP\": %d", first ? "" : ", ", kv.first.first, kv.first.second, kv.second);
        first = false;
    }
    printf("}, \"cus_by_workgroups\": {");
    first = true;
    for (auto& kv : cu_hist) {
        printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
        first = false;
    }
    printf("}}%s\n", last ? "" : ",");
    return 0;
}

int main() {
    const int spin = 20000000;   // ~8 ms at 2.4 GHz: every workgroup of the grid is resident at once
    printf("{\n");
    // compact K1Q: 33 KiB of LDS (2,112 uint4 = 33 KiB), four per CU; 8,192 leaves = 1,024 WGs
    if (run<2112>("compact_1024wg", 1024, spin, false)) return 1;
    // wide K1Q: 64 KiB, <= 2 per CU; 256 leaves = 32 WGs, 4,096 leaves = 512 WGs
    if (run<4096>("wide_32wg", 32, spin, false)) return 1;
    if (run<4096>("wide_512wg", 512, spin, true)) return 1;
    printf("}\n");
    return 0;
}
