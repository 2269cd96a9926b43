// round_bench.hip -- time the K1Q round instruction sequences on gfx950 (timing only, data is
// arbitrary).  A: the lock-step round (9 VALU: both triples on the same round, two DPP exchanges).
// B: the a-triple two rounds behind the e-triple, one symmetric row_ror:8 exchange per step
// (8 VALU, 4-deep chain).  Prints JSON: ns and nominal-clock cycles per round, one wave alone and
// one wave per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/round_bench tools/round_bench.hip
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

// A: lock-step round, as DM_QUAD_ROUND_ASM + DM_QUAD_NEXT_H (one asm block per 4 rounds, so the
// compiler inserts nothing between rounds)
#define STEP_A(X4, X5, X6, X7, VN)                                                             \
    "v_alignbit_b32 %[r], %[" X4 "], %[" X4 "], %[sh]\n\t"                                   \
    "v_bitop3_b32 %[f], %[" X4 "], %[" X5 "], %[msk] bitop3:0x1e\n\t"                       \
    "v_bitop3_b32 %[f], %[f], %[" X6 "], %[" X5 "] bitop3:0xca\n\t"                          \
    "v_xor_b32_dpp %[s], %[r], %[r] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_xor_b32_dpp %[s], %[r], %[s] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_add3_u32 %[" X7 "], %[s], %[f], %[h]\n\t"                                            \
    "v_xad_u32 %[h], %[" X6 "], %[neg], %[" VN "]\n\t"                                       \
    "v_add_u32_dpp %[h], %[" X6 "], %[h] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"           \
    "v_add_u32_dpp %[" X7 "], %[" X7 "], %[" X7 "] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"

// B: skewed step.  H (this step's add3 term) was made by the previous step; HN is the next one.
#define STEP_B(X4, X5, X6, X7, H, HN, VN)                                                      \
    "v_alignbit_b32 %[r], %[" X4 "], %[" X4 "], %[sh]\n\t"                                   \
    "v_bitop3_b32 %[f], %[" X4 "], %[" X5 "], %[msk] bitop3:0x1e\n\t"                       \
    "v_xad_u32 %[" HN "], %[" X6 "], %[neg], %[" VN "]\n\t"                                  \
    "v_xor_b32_dpp %[s], %[r], %[r] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_bitop3_b32 %[f], %[f], %[" X6 "], %[" X5 "] bitop3:0xca\n\t"                          \
    "v_xor_b32_dpp %[s], %[r], %[s] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_add_u32_dpp %[" HN "], %[" X4 "], %[" HN "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t" \
    "v_add3_u32 %[" X7 "], %[s], %[f], %[" H "]\n\t"

// C: B with the two H instructions in other slots
#define STEP_C(X4, X5, X6, X7, H, HN, VN)                                                      \
    "v_alignbit_b32 %[r], %[" X4 "], %[" X4 "], %[sh]\n\t"                                   \
    "v_bitop3_b32 %[f], %[" X4 "], %[" X5 "], %[msk] bitop3:0x1e\n\t"                       \
    "v_add_u32_dpp %[" HN "], %[" X5 "], %[" HN "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t" \
    "v_xor_b32_dpp %[s], %[r], %[r] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_bitop3_b32 %[f], %[f], %[" X6 "], %[" X5 "] bitop3:0xca\n\t"                          \
    "v_xor_b32_dpp %[s], %[r], %[s] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_xad_u32 %[" H "], %[" X5 "], %[neg], %[" VN "]\n\t"                                   \
    "v_add3_u32 %[" X7 "], %[s], %[f], %[" HN "]\n\t"

// D: every chain edge two slots apart: A, f1, xor1, f, xor2, xad(next), add3, add_dpp(next)
#define STEP_D(X4, X5, X6, X7, H, HN, VN)                                                      \
    "v_alignbit_b32 %[r], %[" X4 "], %[" X4 "], %[sh]\n\t"                                   \
    "v_bitop3_b32 %[f], %[" X4 "], %[" X5 "], %[msk] bitop3:0x1e\n\t"                       \
    "v_xor_b32_dpp %[s], %[r], %[r] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_bitop3_b32 %[f], %[f], %[" X6 "], %[" X5 "] bitop3:0xca\n\t"                          \
    "v_xor_b32_dpp %[s], %[r], %[s] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"     \
    "v_xad_u32 %[" HN "], %[" X6 "], %[neg], %[" VN "]\n\t"                                  \
    "v_add3_u32 %[" X7 "], %[s], %[f], %[" H "]\n\t"                                        \
    "v_add_u32_dpp %[" HN "], %[" X4 "], %[" HN "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"

#define OPS                                                                                    \
    : [a] "+v"(x4), [b] "+v"(x5), [c] "+v"(x6), [d] "+v"(x7), [h] "+v"(h), [g] "+v"(hb),      \
      [r] "=&v"(r_), [f] "=&v"(f_), [s] "=&v"(s_)                                              \
    : [sh] "v"(sh), [msk] "v"(msk), [neg] "v"(neg), [v0] "v"(v0), [v1] "v"(v1), [v2] "v"(v2),  \
      [v3] "v"(v3)

template <int MODE>
__global__ __launch_bounds__(64) void round_kernel(uint32_t* out, int iters, uint32_t seed) {
    const uint32_t lane = threadIdx.x;
    uint32_t x4 = seed * (lane + 1), x5 = x4 ^ 0x9e3779b9u, x6 = x4 + 7, x7 = x5 * 3;
    uint32_t h = lane, hb = lane * 5;
    uint32_t r_, f_, s_;
    const uint32_t sh = 6 + (lane & 3), msk = (lane & 4) ? 0u : ~0u, neg = (lane & 4) ? ~0u : 0u;
    uint32_t v0 = seed + lane, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7;
    for (int it = 0; it < iters; it++) {
        if constexpr (MODE == 0) {
            asm volatile(STEP_A("a", "b", "c", "d", "v0") STEP_A("d", "a", "b", "c", "v1")
                         STEP_A("c", "d", "a", "b", "v2") STEP_A("b", "c", "d", "a", "v3") OPS);
        } else if constexpr (MODE == 1) {
            asm volatile(STEP_B("a", "b", "c", "d", "h", "g", "v0") STEP_B("d", "a", "b", "c", "g", "h", "v1")
                         STEP_B("c", "d", "a", "b", "h", "g", "v2") STEP_B("b", "c", "d", "a", "g", "h", "v3") OPS);
        } else if constexpr (MODE == 3) {
            asm volatile(STEP_D("a", "b", "c", "d", "h", "g", "v0") STEP_D("d", "a", "b", "c", "g", "h", "v1")
                         STEP_D("c", "d", "a", "b", "h", "g", "v2") STEP_D("b", "c", "d", "a", "g", "h", "v3") OPS);
        } else {
            asm volatile(STEP_C("a", "b", "c", "d", "h", "g", "v0") STEP_C("d", "a", "b", "c", "g", "h", "v1")
                         STEP_C("c", "d", "a", "b", "h", "g", "v2") STEP_C("b", "c", "d", "a", "g", "h", "v3") OPS);
        }
    }
    const uint32_t acc = x4 ^ x5 ^ x6 ^ x7 ^ h ^ hb;
    if (acc == 0x12345678u) out[blockIdx.x * 64 + lane] = acc;
}

template <int MODE>
double ns_per_round(int blocks, int iters, uint32_t* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((round_kernel<MODE>), dim3(blocks), dim3(64), 0, 0, out, iters, 3u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((round_kernel<MODE>), dim3(blocks), dim3(64), 0, 0, out, iters, 5u);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms * 1e6 / (4.0 * iters);
}

int main() {
    uint32_t* out;
    CHK(hipMalloc(&out, 1 << 20));
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double ghz = p.clockRate * 1e-6;
    const int iters = 1 << 17;
    double a1 = ns_per_round<0>(1, iters, out), b1 = ns_per_round<1>(1, iters, out);
    double a32 = ns_per_round<0>(32, iters, out), b32 = ns_per_round<1>(32, iters, out);
    double aS = ns_per_round<0>(cus * 4, iters, out), bS = ns_per_round<1>(cus * 4, iters, out);
    double c1 = ns_per_round<2>(1, iters, out), c32 = ns_per_round<2>(32, iters, out);
    double d1 = ns_per_round<3>(1, iters, out), d32 = ns_per_round<3>(32, iters, out);
    printf("{\"clock_ghz_nominal\": %.3f, \"lockstep_9\": {\"ns_1wave\": %.3f, \"cyc_1wave\": %.2f, \"ns_32waves\": %.3f, "
           "\"ns_1_per_simd\": %.3f}, \"skew2_8\": {\"ns_1wave\": %.3f, \"cyc_1wave\": %.2f, \"ns_32waves\": %.3f, "
           "\"ns_1_per_simd\": %.3f}, \"skew2_8_reordered\": {\"ns_1wave\": %.3f, \"cyc_1wave\": %.2f, \"ns_32waves\": %.3f}, \"skew2_8_spaced\": {\"ns_1wave\": %.3f, \"cyc_1wave\": %.2f, \"ns_32waves\": %.3f}}\n",
           ghz, a1, a1 * ghz, a32, aS, b1, b1 * ghz, b32, bS, c1, c1 * ghz, c32, d1, d1 * ghz, d32);
    CHK(hipFree(out));
    return 0;
}
