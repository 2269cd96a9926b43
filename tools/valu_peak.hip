// valu_peak.hip -- measure the integer VALU rates SHA-256 is built from, on gfx950.
//
// Every measured instruction is emitted by inline asm (the compiler cannot fold rotate chains).
// Prints JSON:
//  - chip-wide lane-ops/s for v_alignbit_b32, v_bitop3_b32, v_add3_u32, v_add_u32 (8 independent
//    chains per lane, 16 waves per CU);
//  - one wave alone: cycles per instruction for 8 independent chains and for 1 dependent chain
//    (the latency-bound regime of few large leaves), and 2 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_peak tools/valu_peak.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int OP>
__device__ __forceinline__ uint32_t op(uint32_t x, uint32_t y, uint32_t z) {
    uint32_t r;
    if constexpr (OP == 0) asm volatile("v_alignbit_b32 %0, %1, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    else if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    else if constexpr (OP == 2) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    else if constexpr (OP == 3) asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    else if constexpr (OP == 4) asm volatile("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    // DPP add: the nop covers the VALU-write -> DPP-read wait states of a dependent chain
    else asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf"
                      : "=v"(r) : "v"(x), "v"(y));
    return r;
}

template <int OP, int CHAINS>
__global__ __launch_bounds__(256) void ops_kernel(uint32_t* out, int iters, uint32_t seed) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = seed * (threadIdx.x + 17 * i + 1) ^ (blockIdx.x << i);
    const uint32_t k = seed | 5u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int c = 0; c < CHAINS; c++) v[c] = op<OP>(v[c], k, v[c]);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i];
    if (acc == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP, int CHAINS>
double run(int blocks, int threads, int iters, uint32_t* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((ops_kernel<OP, CHAINS>), dim3(blocks), dim3(threads), 0, 0, out, iters, 3u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((ops_kernel<OP, CHAINS>), dim3(blocks), dim3(threads), 0, 0, out, iters, 5u);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    const double ops = (double)blocks * threads * iters * 16.0 * CHAINS;
    return ops / (ms * 1e-3);   // lane-ops per second
}

int main() {
    uint32_t* out;
    CHK(hipMalloc(&out, 64ull << 20));
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int iters = 2048;
    const double clk = p.clockRate * 1e3;   // Hz (nominal max)
    double al = run<0, 8>(cus * 4, 256, iters, out);
    double al8 = run<0, 8>(cus * 2, 256, iters, out);
    double b3 = run<1, 8>(cus * 4, 256, iters, out);
    double ad3 = run<2, 8>(cus * 4, 256, iters, out);
    double ad = run<3, 8>(cus * 4, 256, iters, out);
    // single wave: lane-ops/s / 64 lanes = wave-instructions per second
    double w1_ind = run<0, 8>(1, 64, iters, out) / 64.0;
    double w1_dep = run<0, 1>(1, 64, iters, out) / 64.0;
    double w1_dep_add3 = run<2, 1>(1, 64, iters, out) / 64.0;
    // 8 waves in one workgroup = 2 waves per SIMD, independent chains
    double w8_ind = run<0, 8>(1, 512, iters, out) / 512.0;
    double xad = run<4, 8>(cus * 4, 256, iters, out);
    double w1_dep_add = run<3, 1>(1, 64, iters, out) / 64.0;
    double w1_dep_bitop3 = run<1, 1>(1, 64, iters, out) / 64.0;
    double w1_dep_xad = run<4, 1>(1, 64, iters, out) / 64.0;
    double w1_dep_dpp = run<5, 1>(1, 64, iters, out) / 64.0;
    double w1_ind_add = run<3, 8>(1, 64, iters, out) / 64.0;
    printf("{\"cus\": %d, \"clock_hz_nominal\": %.0f, \"alignbit_lane_ops_s_16w\": %.4e, \"alignbit_lane_ops_s_8w\": %.4e, "
           "\"bitop3_lane_ops_s\": %.4e, \"add3_lane_ops_s\": %.4e, \"add_lane_ops_s\": %.4e, "
           "\"one_wave_indep_cycles_per_inst\": %.3f, \"one_wave_dep_cycles_per_inst\": %.3f, "
           "\"one_wave_dep_add3_cycles_per_inst\": %.3f, \"two_waves_per_simd_cycles_per_inst_per_wave\": %.3f, "
           "\"xad_lane_ops_s\": %.4e, \"one_wave_dep_add_cycles_per_inst\": %.3f, "
           "\"one_wave_dep_bitop3_cycles_per_inst\": %.3f, \"one_wave_dep_xad_cycles_per_inst\": %.3f, "
           "\"one_wave_dep_nop_dpp_add_cycles_per_pair\": %.3f, \"one_wave_indep_add_cycles_per_inst\": %.3f}\n",
           cus, clk, al, al8, b3, ad3, ad, clk / w1_ind, clk / w1_dep, clk / w1_dep_add3, clk / w8_ind, xad,
           clk / w1_dep_add, clk / w1_dep_bitop3, clk / w1_dep_xad, clk / w1_dep_dpp, clk / w1_ind_add);
    CHK(hipFree(out));
    return 0;
}
