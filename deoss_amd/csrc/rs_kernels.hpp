// rs_kernels.hpp -- gfx950 Reed-Solomon fragment coding (GF(2^8)), the stage after hashing on the
// DeOSS upload path.  Included by merkle_capi.hip only.
//
// Reference: cess-go-sdk erasure-codes each 32 MiB segment into chain.DataShards = 4 data and
// chain.ParShards = 8 parity fragments (node/tracker.go:250,369, node/fileHandler.go:250) with
// klauspost/reedsolomon v1.12.4 (go.mod:65): parity[i] = sum_j M[i][j] * data[j] over GF(2^8)
// (polynomial 0x11d), M = Vandermonde x inverse(top square).  The same kernel applies any
// (nout x nin) GF matrix, so Reconstruct uses it with a decode matrix built on the host.
//
// HBM-bound byte work, not a GEMM: every input byte x of shard j is looked up ONCE in an LDS
// table T_j[x] whose 8 bytes are (M[0][j]*x, ..., M[7][j]*x) -- the contributions of that byte to
// all (up to 8) outputs at the same position -- and the lookups of the nin inputs are xor-ed.
// A lane owns 16 consecutive positions (one uint4 per shard), so per 16 positions it issues nin
// 16-B loads, 16*nin ds_read_b64, and nout 16-B stores; the position-major accumulators are
// turned into shard-major output words by 4x4 byte transposes (v_perm_b32).
// What bounds it (tools/rs_ab.hip, profiles/r02/LOGS.md#r02d_rs_ab_repeats.log, interleaved repeats on one
// box): this kernel 5.09 ms per 8 GiB of segments, the same access pattern with no table at all
// 5.13 ms, a conflict-free variant (replicated nibble tables, 0 bank conflicts) 5.23 ms.  The
// random-index bank conflicts (68 % of LDS cycles) are hidden under the 1-read : 2-write HBM
// stream, which itself runs at 5.0 TB/s against 6.2-6.3 TB/s for a 1:1 copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dm {

constexpr int kRsMaxIn = 8;
constexpr int kRsMaxOut = 8;
constexpr int kRsThreads = 256;

struct RsArgs {
    const uint8_t* in[kRsMaxIn];   // input shard j of segment 0
    uint8_t* out[kRsMaxOut];       // output shard i of segment 0
    uint64_t in_seg_stride;        // bytes from segment s to s+1 (inputs)
    uint64_t out_seg_stride;       // bytes from segment s to s+1 (outputs)
    uint64_t units_per_seg;        // shard bytes / 16
    uint64_t nseg;
    const uint2* table;            // [nin][256] x 8 B: byte i of entry x = M[i][j] * x
    uint32_t nout;
};

// 4x4 byte transpose: out_r byte c = in_c byte r (in_c = a, b, c, d).
__device__ __forceinline__ void transpose4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t (&o)[4]) {
    const uint32_t ab_lo = __builtin_amdgcn_perm(b, a, 0x05010400u);   // a0 b0 a1 b1
    const uint32_t ab_hi = __builtin_amdgcn_perm(b, a, 0x07030602u);   // a2 b2 a3 b3
    const uint32_t cd_lo = __builtin_amdgcn_perm(d, c, 0x05010400u);
    const uint32_t cd_hi = __builtin_amdgcn_perm(d, c, 0x07030602u);
    o[0] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);            // a0 b0 c0 d0
    o[1] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);            // a1 b1 c1 d1
    o[2] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
    o[3] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
}

#ifndef DM_RS_NT_STORE
#define DM_RS_NT_STORE 1
#endif
#ifndef DM_RS_NT_LOAD
#define DM_RS_NT_LOAD 0
#endif
#ifndef DM_RS_WAVES
#define DM_RS_WAVES 0
#endif

typedef unsigned int rs_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 rs_load(const uint8_t* p) {
#if DM_RS_NT_LOAD
    const rs_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const rs_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *reinterpret_cast<const uint4*>(p);
#endif
}

__device__ __forceinline__ void rs_store(uint8_t* p, uint4 v) {
#if DM_RS_NT_STORE
    const rs_u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<rs_u32x4*>(p));
#else
    *reinterpret_cast<uint4*>(p) = v;
#endif
}

// Grid: x strides over a segment's 16-byte units, y over segments (no 64-bit division).
template <int NIN>
__global__ __launch_bounds__(kRsThreads)
#if DM_RS_WAVES
__attribute__((amdgpu_waves_per_eu(DM_RS_WAVES)))
#endif
void rs_code_kernel(RsArgs a) {
    __shared__ uint2 tab[NIN * 256];
    for (uint32_t t = threadIdx.x; t < NIN * 256; t += kRsThreads) tab[t] = a.table[t];
    __syncthreads();
    const uint64_t ustride = (uint64_t)gridDim.x * kRsThreads;
    for (uint64_t seg = blockIdx.y; seg < a.nseg; seg += gridDim.y) {
        const uint64_t ib = seg * a.in_seg_stride;
        const uint64_t ob = seg * a.out_seg_stride;
        uint64_t u = (uint64_t)blockIdx.x * kRsThreads + threadIdx.x;
        // register double buffer: the next unit's loads are in flight while this one is coded
        uint4 nx[NIN];
        if (u < a.units_per_seg) {
#pragma unroll
            for (int j = 0; j < NIN; j++) nx[j] = rs_load(a.in[j] + ib + u * 16);
        }
        for (; u < a.units_per_seg; u += ustride) {
            const uint64_t off = u * 16;
            uint4 x[NIN];
#pragma unroll
            for (int j = 0; j < NIN; j++) x[j] = nx[j];
            if (u + ustride < a.units_per_seg) {
#pragma unroll
                for (int j = 0; j < NIN; j++) nx[j] = rs_load(a.in[j] + ib + off + ustride * 16);
            }
            uint2 acc[16];
#pragma unroll
            for (int p = 0; p < 16; p++) acc[p] = make_uint2(0, 0);
#pragma unroll
            for (int j = 0; j < NIN; j++) {
                const uint32_t w[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
                const uint2* tj = tab + j * 256;
#pragma unroll
                for (int q = 0; q < 4; q++) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint2 e = tj[(w[q] >> (8 * k)) & 0xffu];
                        acc[4 * q + k].x ^= e.x;
                        acc[4 * q + k].y ^= e.y;
                    }
                }
            }
            // output shard i, word q = byte i of acc[4q .. 4q+3]
            uint32_t lo[4][4], hi[4][4];   // [q][row]
#pragma unroll
            for (int q = 0; q < 4; q++) {
                transpose4(acc[4 * q].x, acc[4 * q + 1].x, acc[4 * q + 2].x, acc[4 * q + 3].x, lo[q]);
                transpose4(acc[4 * q].y, acc[4 * q + 1].y, acc[4 * q + 2].y, acc[4 * q + 3].y, hi[q]);
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i < (int)a.nout)
                    rs_store(a.out[i] + ob + off, make_uint4(lo[0][i], lo[1][i], lo[2][i], lo[3][i]));
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (i + 4 < (int)a.nout)
                    rs_store(a.out[i + 4] + ob + off, make_uint4(hi[0][i], hi[1][i], hi[2][i], hi[3][i]));
        }
    }
}

}  // namespace dm
