// valu_peak.hip -- measure the integer VALU rates SHA-256 is built from, on gfx950.
//
// Prints JSON: chip-wide lane-ops/s for v_alignbit_b32 / v_bitop3_b32 / v_add3_u32 (8 independent
// chains per lane, many waves), and one wave's issue rate for independent and dependent chains
// (the latency-bound regime of few large leaves).  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int OP, int CHAINS>
__global__ __launch_bounds__(256) void ops_kernel(uint32_t* out, int iters, uint32_t seed) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = seed * (threadIdx.x + 17 * i + 1) ^ (blockIdx.x << i);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int c = 0; c < CHAINS; c++) {
                uint32_t x = v[c], y = v[(c + 1) % 8] | 1u;
                if constexpr (OP == 0) v[c] = __builtin_amdgcn_alignbit(x, x, 7 + r);
                else if constexpr (OP == 1) v[c] = __builtin_amdgcn_bitop3_b32(x, y, v[(c + 2) % 8], 0x96);
                else v[c] = x + y + v[(c + 2) % 8] + 0x9e3779b9u * 0;   // add3
            }
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
    double ops = (double)blocks * threads * iters * 16.0 * CHAINS;
    return ops / (ms * 1e-3);   // lane-ops per second
}

int main() {
    uint32_t* out;
    CHK(hipMalloc(&out, 64ull << 20));
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int iters = 4096;
    // chip-wide: 8 waves per CU (2 per SIMD) and 16 per CU
    double al8 = run<0, 8>(cus * 2, 256, iters, out);
    double al16 = run<0, 8>(cus * 4, 256, iters, out);
    double b3 = run<1, 8>(cus * 4, 256, iters, out);
    double ad3 = run<2, 8>(cus * 4, 256, iters, out);
    // one wave alone: independent (8 chains) and dependent (1 chain) alignbit; ops per cycle at clockRate
    double one_ind = run<0, 8>(1, 64, iters, out) / 64.0;   // wave-instructions per second
    double one_dep = run<0, 1>(1, 64, iters, out) / 64.0;
    double clk = p.clockRate * 1e3;   // Hz
    printf("{\"cus\": %d, \"clock_hz\": %.0f, \"alignbit_lane_ops_s_8w\": %.4e, \"alignbit_lane_ops_s_16w\": %.4e, "
           "\"bitop3_lane_ops_s\": %.4e, \"add3_lane_ops_s\": %.4e, "
           "\"one_wave_indep_cycles_per_inst\": %.3f, \"one_wave_dep_cycles_per_inst\": %.3f}\n",
           cus, clk, al8, al16, b3, ad3, clk / one_ind, clk / one_dep);
    CHK(hipFree(out));
    return 0;
}
