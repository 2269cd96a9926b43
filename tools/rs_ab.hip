// rs_ab.hip -- what bounds rs_code_kernel?  Standalone A/B on one MI355X:
//   copy      : 1 read : 1 write streaming copy (the guide's 6.3 TB/s reference pattern)
//   stream12  : the RS access pattern with no arithmetic -- 4 x 16-B reads, 8 x 16-B writes per
//               lane per 16 positions (each output = xor of the inputs), same grid and strides
//   rs        : rs_code_kernel<4> as shipped (256-entry x 8-B LDS table per input, one lookup per
//               input byte, bank conflicts from random indices)
//   rs_nib    : nibble tables, 32 bank-pair replicas (conflict-free ds_read_b64, 2 lookups/byte)
// Data: 256 segments x 32 MiB (8 GiB in, 16 GiB out), GF(2^8) tables from random coefficients.
// rs_nib is checked byte for byte against the shipped kernel.  Build: hipcc --offload-arch=gfx950 -O3 tools/rs_ab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../deoss_amd/csrc/rs_kernels.hpp"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1d : 0));
        b >>= 1;
    }
    return r;
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const dm::rs_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const dm::rs_u32x4*>(in + i));
        __builtin_nontemporal_store(v, reinterpret_cast<dm::rs_u32x4*>(out + i));
    }
}

// Plain (temporal) copy, one uint4 per thread, no grid-stride loop.
__global__ __launch_bounds__(256) void copy_flat_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// RS access pattern, plain stores, U units per lane per iteration (more bytes in flight).
template <int U, bool NT>
__global__ __launch_bounds__(256) void stream12u_kernel(dm::RsArgs a) {
    const uint64_t ustride = (uint64_t)gridDim.x * 256;
    for (uint64_t seg = blockIdx.y; seg < a.nseg; seg += gridDim.y) {
        const uint64_t ib = seg * a.in_seg_stride, ob = seg * a.out_seg_stride;
        for (uint64_t u0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; u0 < a.units_per_seg; u0 += U * ustride) {
            uint4 x[U][4];
#pragma unroll
            for (int v = 0; v < U; v++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    x[v][j] = u0 + v * ustride < a.units_per_seg ? dm::rs_load(a.in[j] + ib + (u0 + v * ustride) * 16)
                                                                  : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int v = 0; v < U; v++) {
                const uint64_t u = u0 + v * ustride;
                if (u >= a.units_per_seg) break;
                uint4 s = x[v][0];
                s.x ^= x[v][1].x ^ x[v][2].x ^ x[v][3].x;
                s.y ^= x[v][1].y ^ x[v][2].y ^ x[v][3].y;
                s.z ^= x[v][1].z ^ x[v][2].z ^ x[v][3].z;
                s.w ^= x[v][1].w ^ x[v][2].w ^ x[v][3].w;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    uint8_t* dst = a.out[i] + ob + u * 16;
                    const uint4 o = make_uint4(s.x + i, s.y, s.z, s.w);
                    if (NT) dm::rs_store(dst, o);
                    else *reinterpret_cast<uint4*>(dst) = o;
                }
            }
        }
    }
}

// RS access pattern without the table lookups.
__global__ __launch_bounds__(256) void stream12_kernel(dm::RsArgs a) {
    const uint64_t ustride = (uint64_t)gridDim.x * 256;
    for (uint64_t seg = blockIdx.y; seg < a.nseg; seg += gridDim.y) {
        const uint64_t ib = seg * a.in_seg_stride, ob = seg * a.out_seg_stride;
        for (uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x; u < a.units_per_seg; u += ustride) {
            uint4 x[4];
#pragma unroll
            for (int j = 0; j < 4; j++) x[j] = dm::rs_load(a.in[j] + ib + u * 16);
            uint4 s = x[0];
            s.x ^= x[1].x ^ x[2].x ^ x[3].x;
            s.y ^= x[1].y ^ x[2].y ^ x[3].y;
            s.z ^= x[1].z ^ x[2].z ^ x[3].z;
            s.w ^= x[1].w ^ x[2].w ^ x[3].w;
#pragma unroll
            for (int i = 0; i < 8; i++) dm::rs_store(a.out[i] + ob + u * 16, make_uint4(s.x + i, s.y, s.z, s.w));
        }
    }
}

// Conflict-free alternative measured against the shipped kernel: nibble tables (T[x] =
// T[x & 15] ^ T[x & 0xf0], GF(2^8) products are xor-linear), 32 bank-pair replicas interleaved so
// lane l reads only banks 2(l%32), 2(l%32)+1.  Bit-identical output; 0 bank conflicts, 2.4x the
// VALU, and 2.7 % slower (profiles/r02/LOGS.md#r02d_rs_ab_repeats.log): not shipped.
constexpr int kNib = 32;
template <int NIN>
__global__ __launch_bounds__(256) void rs_nib_kernel(dm::RsArgs a) {
    __shared__ uint2 tab[NIN * kNib * 32];
    for (uint32_t t = threadIdx.x; t < NIN * kNib * 32; t += 256) tab[t] = a.table[t / 32];
    __syncthreads();
    const uint32_t rep = threadIdx.x & 31;
    const uint64_t ustride = (uint64_t)gridDim.x * 256;
    for (uint64_t seg = blockIdx.y; seg < a.nseg; seg += gridDim.y) {
        const uint64_t ib = seg * a.in_seg_stride, ob = seg * a.out_seg_stride;
        uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
        uint4 nx[NIN];
        if (u < a.units_per_seg) {
#pragma unroll
            for (int j = 0; j < NIN; j++) nx[j] = dm::rs_load(a.in[j] + ib + u * 16);
        }
        for (; u < a.units_per_seg; u += ustride) {
            const uint64_t off = u * 16;
            uint4 x[NIN];
#pragma unroll
            for (int j = 0; j < NIN; j++) x[j] = nx[j];
            if (u + ustride < a.units_per_seg) {
#pragma unroll
                for (int j = 0; j < NIN; j++) nx[j] = dm::rs_load(a.in[j] + ib + off + ustride * 16);
            }
            uint2 acc[16];
#pragma unroll
            for (int p = 0; p < 16; p++) acc[p] = make_uint2(0, 0);
#pragma unroll
            for (int j = 0; j < NIN; j++) {
                const uint32_t w[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
                const uint2* tj = tab + j * kNib * 32 + rep;
#pragma unroll
                for (int q = 0; q < 4; q++) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t lo = (w[q] >> (8 * k)) & 15u, hi = (w[q] >> (8 * k + 4)) & 15u;
                        const uint2 e0 = tj[lo * 32], e1 = tj[(16 + hi) * 32];
                        acc[4 * q + k].x ^= e0.x ^ e1.x;
                        acc[4 * q + k].y ^= e0.y ^ e1.y;
                    }
                }
            }
            uint32_t lo[4][4], hi[4][4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                dm::transpose4(acc[4 * q].x, acc[4 * q + 1].x, acc[4 * q + 2].x, acc[4 * q + 3].x, lo[q]);
                dm::transpose4(acc[4 * q].y, acc[4 * q + 1].y, acc[4 * q + 2].y, acc[4 * q + 3].y, hi[q]);
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i < (int)a.nout) dm::rs_store(a.out[i] + ob + off, make_uint4(lo[0][i], lo[1][i], lo[2][i], lo[3][i]));
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i + 4 < (int)a.nout)
                    dm::rs_store(a.out[i + 4] + ob + off, make_uint4(hi[0][i], hi[1][i], hi[2][i], hi[3][i]));
        }
    }
}


int main() {
    const int K = 4, M = 8;
    const uint64_t seg = 32ull << 20, shard = seg / K, nseg = 256;
    const uint64_t in_bytes = nseg * seg, out_bytes = nseg * M * shard;
    uint8_t *din, *dout, *dout2;
    CK(hipMalloc(&din, in_bytes));
    CK(hipMalloc(&dout, out_bytes));
    CK(hipMalloc(&dout2, out_bytes));
    {   // input bytes: any pattern with all byte values
        std::vector<uint8_t> h(64 << 20);
        uint64_t z = 0x9e3779b97f4a7c15ull;
        for (auto& b : h) {
            z ^= z << 13; z ^= z >> 7; z ^= z << 17;
            b = (uint8_t)z;
        }
        for (uint64_t o = 0; o < in_bytes; o += h.size()) CK(hipMemcpy(din + o, h.data(), h.size(), hipMemcpyHostToDevice));
    }
    uint8_t coef[M][K];
    for (int i = 0; i < M; i++)
        for (int j = 0; j < K; j++) coef[i][j] = (uint8_t)(17 * i + 31 * j + 3);
    std::vector<uint64_t> tab(K * 256), nib(K * kNib);
    for (int j = 0; j < K; j++)
        for (int x = 0; x < 256; x++) {
            uint64_t e = 0;
            for (int i = 0; i < M; i++) e |= (uint64_t)gmul(coef[i][j], (uint8_t)x) << (8 * i);
            tab[j * 256 + x] = e;
        }
    for (int j = 0; j < K; j++)
        for (int e = 0; e < 16; e++) {
            nib[j * kNib + e] = tab[j * 256 + e];
            nib[j * kNib + 16 + e] = tab[j * 256 + (e << 4)];
        }
    uint2 *dtab, *dnib;
    CK(hipMalloc(&dtab, tab.size() * 8));
    CK(hipMalloc(&dnib, nib.size() * 8));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dnib, nib.data(), nib.size() * 8, hipMemcpyHostToDevice));
    auto args = [&](uint8_t* out, const uint2* table) {
        dm::RsArgs a{};
        for (int j = 0; j < K; j++) a.in[j] = din + j * shard;
        for (int i = 0; i < M; i++) a.out[i] = out + i * shard;
        a.in_seg_stride = seg;
        a.out_seg_stride = M * shard;
        a.units_per_seg = shard / 16;
        a.nseg = nseg;
        a.table = table;
        a.nout = M;
        return a;
    };
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t gy = 256, gx = (uint32_t)((8ull * cus + gy - 1) / gy);   // launch_rs's shape
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"TBps\": %.4f}\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    const double rs_bytes = (double)in_bytes + (double)out_bytes;
    timeit("copy (1R:1W, 16 GiB moved)", 2.0 * (double)in_bytes, [&] {
        hipLaunchKernelGGL(copy_kernel, dim3(8 * cus), dim3(256), 0, 0, (const uint4*)din, (uint4*)dout, in_bytes / 16);
    });
    timeit("copy_flat (1R:1W, plain, 1 uint4/thread)", 2.0 * (double)in_bytes, [&] {
        hipLaunchKernelGGL(copy_flat_kernel, dim3((uint32_t)(in_bytes / 16 / 256)), dim3(256), 0, 0, (const uint4*)din,
                           (uint4*)dout, in_bytes / 16);
    });
    timeit("copy (1R:1W, 16 GiB moved) again", 2.0 * (double)in_bytes, [&] {
        hipLaunchKernelGGL(copy_kernel, dim3(8 * cus), dim3(256), 0, 0, (const uint4*)din, (uint4*)dout, in_bytes / 16);
    });
    timeit("stream12u<1, plain stores>", rs_bytes, [&] {
        hipLaunchKernelGGL((stream12u_kernel<1, false>), dim3(gx, gy), dim3(256), 0, 0, args(dout, dtab));
    });
    timeit("stream12u<2, nt stores>", rs_bytes, [&] {
        hipLaunchKernelGGL((stream12u_kernel<2, true>), dim3(gx, gy), dim3(256), 0, 0, args(dout, dtab));
    });
    timeit("stream12u<2, plain stores>", rs_bytes, [&] {
        hipLaunchKernelGGL((stream12u_kernel<2, false>), dim3(gx, gy), dim3(256), 0, 0, args(dout, dtab));
    });
    timeit("stream12u<1, nt>, 2x grid", rs_bytes, [&] {
        hipLaunchKernelGGL((stream12u_kernel<1, true>), dim3(2 * gx, gy), dim3(256), 0, 0, args(dout, dtab));
    });
    timeit("stream12u<1, nt>, 4x grid", rs_bytes, [&] {
        hipLaunchKernelGGL((stream12u_kernel<1, true>), dim3(4 * gx, gy), dim3(256), 0, 0, args(dout, dtab));
    });
    timeit("stream12 (RS pattern, no tables)", rs_bytes, [&] {
        hipLaunchKernelGGL(stream12_kernel, dim3(gx, gy), dim3(256), 0, 0, args(dout, dtab));
    });
    timeit("rs_code_kernel<4> (shipped: 256-entry tables)", rs_bytes, [&] {
        hipLaunchKernelGGL(dm::rs_code_kernel<4>, dim3(gx, gy), dim3(256), 0, 0, args(dout, dtab));
    });
    timeit("rs_nib_kernel<4> (replicated nibble tables, conflict-free)", rs_bytes, [&] {
        hipLaunchKernelGGL(rs_nib_kernel<4>, dim3(gx, gy), dim3(256), 0, 0, args(dout2, dnib));
    });
    // interleaved repeats of the three same-pattern kernels (run-to-run spread is a few %)
    for (int round = 0; round < 5; round++) {
        timeit("rep stream12", rs_bytes, [&] {
            hipLaunchKernelGGL(stream12_kernel, dim3(gx, gy), dim3(256), 0, 0, args(dout, dtab));
        });
        timeit("rep rs_code (shipped)", rs_bytes, [&] {
            hipLaunchKernelGGL(dm::rs_code_kernel<4>, dim3(gx, gy), dim3(256), 0, 0, args(dout, dtab));
        });
        timeit("rep rs_nib", rs_bytes, [&] {
            hipLaunchKernelGGL(rs_nib_kernel<4>, dim3(gx, gy), dim3(256), 0, 0, args(dout2, dnib));
        });
    }
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> a(64 << 20), b(64 << 20);
    bool same = true;
    for (uint64_t o = 0; o < out_bytes && same; o += 1ull << 30) {   // spot-check 64 MiB per GiB
        CK(hipMemcpy(a.data(), dout + o, a.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), dout2 + o, b.size(), hipMemcpyDeviceToHost));
        same = std::memcmp(a.data(), b.data(), a.size()) == 0;
    }
    std::printf("{\"nib_equals_shipped\": %s}\n", same ? "true" : "false");
    return same ? 0 : 2;
}
