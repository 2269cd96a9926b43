// merkle_kernels.hpp -- gfx950 kernels of the DeOSS Merkle path (K1 leaf, K2 tree reduce,
// K3 batched per-object trees, synthetic generator).  Included by merkle_capi.hip only.
//
// Reference algorithm: common/hashtree/hashtree.go:23-30 (leaf = SHA-256 of the chunk),
// common/hashtree/types.go:19-39 (one leaf per chunk), cbergoon/merkletree v0.2.0 (go.mod:10)
// buildWithContent/buildIntermediate: level rule out[j] = H(in[2j] || in[min(2j+1, n-1)]),
// repeated until one node remains, at least one level.
//
// Device memory formats: chunk bytes as given; every digest / tree node is the canonical
// 32-byte big-endian SHA-256 output (what Go's h.Sum(nil) returns).  Inside a kernel nodes
// live as 8 state words (byte swapped once at load / store).
#pragma once
#include "sha256_gfx950.hpp"

namespace dm {

constexpr int kBlock = 256;         // threads per workgroup for K1/K2/K3
constexpr int kLeafFuseMax = 8;     // K1 reduces its 256 leaves by up to 8 levels in LDS
constexpr int kReduceTile = 512;    // K2 inputs per workgroup (9 levels max)

struct LeafArgs {
    const uint8_t* base;        // uniform mode: leaf i starts at base + i * pitch
    uint64_t pitch;
    uint64_t leaf_len;          // uniform mode: length of leaves 0 .. n-2
    uint64_t last_len;          // uniform mode: length of leaf n-1
    const uint64_t* addrs;      // table mode: device address of leaf i
    const uint64_t* lens;       // table mode: length of leaf i
    uint64_t nleaves;
    // stripe (resumable) mode: this launch absorbs bytes [byte_off, byte_end) of every leaf;
    // leaf data pointers then point at byte byte_off of the leaf.  Single shot: 0 / ~0.
    uint64_t byte_off;
    uint64_t byte_end;
    uint32_t* state;            // 8 words per leaf, in/out between stripes (nullptr: single shot)
    uint8_t* digests;           // 32 B per leaf (nullptr: not stored)
    uint8_t* level_out;         // fused mode: nodes after fuse_levels levels
    uint32_t fuse_levels;       // 0 .. kLeafFuseMax
};

__device__ __forceinline__ void load_digest(const uint8_t* p, uint32_t (&v)[8]) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 x = q[0], y = q[1];
    v[0] = bswap32(x.x); v[1] = bswap32(x.y); v[2] = bswap32(x.z); v[3] = bswap32(x.w);
    v[4] = bswap32(y.x); v[5] = bswap32(y.y); v[6] = bswap32(y.z); v[7] = bswap32(y.w);
}

__device__ __forceinline__ void store_digest(uint8_t* p, const uint32_t (&v)[8]) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(bswap32(v[0]), bswap32(v[1]), bswap32(v[2]), bswap32(v[3]));
    q[1] = make_uint4(bswap32(v[4]), bswap32(v[5]), bswap32(v[6]), bswap32(v[7]));
}

// Load one 64-byte block (16 B aligned) as 4 vector loads.

// Leaf bytes always live in global memory.  Table-mode leaf pointers come from memory, so the
// compiler cannot infer their address space: without the cast it emits FLAT loads (split into
// dwordx3/x4/x1 pieces, counted against lgkmcnt with the LDS traffic), which cost K1Q's producer
// 9 % in table mode (batches of 4,096 leaves: 46.0 vs 42.1 ms).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4_t global_u32x4;

typedef __attribute__((address_space(1))) const uint8_t global_u8;
typedef __attribute__((address_space(1))) const uint32_t global_u32;

// Blocks are held as the loaded vector type: converting to uint4 costs 16 extra v_mov_b32 per
// block in K1's register double buffer (1,434 vs 1,418 VALU per block).
struct Blk { u32x4_t q0, q1, q2, q3; };
__device__ __forceinline__ const global_u8* gbytes(const uint8_t* p) { return (const global_u8*)p; }

template <bool ALIGNED>
__device__ __forceinline__ Blk load_block(const uint8_t* p) {
    Blk b;
    if constexpr (ALIGNED) {
        const global_u32x4* q = (const global_u32x4*)(p);
        b.q0 = q[0]; b.q1 = q[1]; b.q2 = q[2]; b.q3 = q[3];
    } else {
        uint8_t t[64];
        const global_u8* g = gbytes(p);
#pragma unroll
        for (int k = 0; k < 64; k++) t[k] = g[k];
        __builtin_memcpy(&b, t, 64);
    }
    return b;
}

__device__ __forceinline__ void block_words(const Blk& b, uint32_t (&w)[16]) {
    w[0] = bswap32(b.q0.x);  w[1] = bswap32(b.q0.y);  w[2] = bswap32(b.q0.z);  w[3] = bswap32(b.q0.w);
    w[4] = bswap32(b.q1.x);  w[5] = bswap32(b.q1.y);  w[6] = bswap32(b.q1.z);  w[7] = bswap32(b.q1.w);
    w[8] = bswap32(b.q2.x);  w[9] = bswap32(b.q2.y);  w[10] = bswap32(b.q2.z); w[11] = bswap32(b.q2.w);
    w[12] = bswap32(b.q3.x); w[13] = bswap32(b.q3.y); w[14] = bswap32(b.q3.z); w[15] = bswap32(b.q3.w);
}

// Absorb nb full blocks starting at p, the next block's loads in flight during each
// compression (register double buffer).  A paired 128-byte variant was measured to make hipcc
// sink the prefetch next to its use (DESIGN.md "K1"), so blocks stay 64 bytes per iteration.
#ifndef DM_K1_LINES
#define DM_K1_LINES 1
#endif
template <bool ALIGNED>
__device__ __forceinline__ void absorb_blocks(uint32_t (&st)[8], const uint8_t* p, uint64_t nb) {
    if (nb == 0) return;
    if constexpr (ALIGNED && DM_K1_LINES) {
        // Whole 128-byte lines: each iteration absorbs two blocks and issues all eight 16-B loads
        // of the NEXT line at once, so every L2 line a lane touches is consumed in one go.  With
        // one block (half a line) per iteration the second half was requested ~1,400 instructions
        // later, after ~24 waves per CU had pulled their own lines through the 4 MiB XCD L2, and
        // 36 % of the lines were fetched twice at 64 KiB chunks (profiles/k1_traffic.json).
        // Loads past the leaf's last block re-read that block (already in cache): no branches
        // around the loads, so they issue as one burst.
        const uint64_t last = nb - 1;
        Blk c0 = load_block<true>(p), c1 = load_block<true>(p + 64 * (last < 1 ? last : 1));
        for (uint64_t b = 0; b < nb; b += 2) {
            const uint64_t b2 = b + 2 < last ? b + 2 : last, b3 = b + 3 < last ? b + 3 : last;
            const Blk n0 = load_block<true>(p + 64 * b2), n1 = load_block<true>(p + 64 * b3);
            __builtin_amdgcn_sched_barrier(0);   // the next line's loads stay ahead of the rounds
            uint32_t w[16];
            block_words(c0, w);
            compress(st, w);
            if (b + 1 < nb) {
                block_words(c1, w);
                compress(st, w);
            }
            c0 = n0;
            c1 = n1;
        }
        return;
    }
    Blk cur = load_block<ALIGNED>(p);
    for (uint64_t b = 0; b < nb; b++) {
        uint32_t w[16];
        block_words(cur, w);
        if (b + 1 < nb) cur = load_block<ALIGNED>(p + 64 * (b + 1));
        compress(st, w);
    }
}

// FIPS 180-4 padding of the final r (< 64) bytes at p, total message length len bytes.
template <bool ALIGNED>
__device__ __forceinline__ void absorb_tail(uint32_t (&st)[8], const uint8_t* p, uint32_t r, uint64_t len) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint32_t v = 0;
        if ((uint32_t)(4 * k + 4) <= r) {
            if constexpr (ALIGNED) {
                v = bswap32(*(const global_u32*)(p + 4 * k));
            } else {
                const global_u8* g = gbytes(p);
                v = ((uint32_t)g[4 * k] << 24) | ((uint32_t)g[4 * k + 1] << 16) |
                    ((uint32_t)g[4 * k + 2] << 8) | (uint32_t)g[4 * k + 3];
            }
        } else if ((uint32_t)(4 * k) <= r) {
            // word holding the 0x80 terminator (and 0..3 message bytes)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t idx = 4 * k + j;
                uint32_t byte = idx < r ? (uint32_t)gbytes(p)[idx] : (idx == r ? 0x80u : 0u);
                v |= byte << (24 - 8 * j);
            }
        }
        w[k] = v;
    }
    const uint64_t bits = len * 8;
    if (r <= 55) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        compress(st, w);
    } else {
        compress(st, w);
#pragma unroll
        for (int k = 0; k < 14; k++) w[k] = 0;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        compress(st, w);
    }
}

// Reduce `cnt` nodes held in LDS (state words, buffer a) for `levels` levels with the
// merkletree rule; ping-pongs between a and b.  Every thread of the block must call this.
// Returns the final node count; the result lives in *res.
__device__ __forceinline__ uint32_t lds_reduce(uint32_t (*a)[8], uint32_t (*b)[8], uint32_t cnt,
                                               uint32_t levels, uint32_t (**res)[8]) {
    const uint32_t t = threadIdx.x;
    for (uint32_t l = 0; l < levels; l++) {
        const uint32_t next = (cnt + 1) >> 1;
        if (t < next) {
            uint32_t L[8], R[8], o[8];
            const uint32_t ri = (2 * t + 1 < cnt) ? 2 * t + 1 : cnt - 1;
#pragma unroll
            for (int k = 0; k < 8; k++) { L[k] = a[2 * t][k]; R[k] = a[ri][k]; }
            node_hash(L, R, o);
#pragma unroll
            for (int k = 0; k < 8; k++) b[t][k] = o[k];
        }
        __syncthreads();
        uint32_t (*tmp)[8] = a; a = b; b = tmp;
        cnt = next;
    }
    *res = a;
    return cnt;
}

// One leaf as seen by one launch: its bytes inside the stripe [byte_off, byte_end) (single
// shot: the whole leaf), how many full blocks that is, and whether the leaf ends here.
struct LeafView {
    const uint8_t* p;   // first byte of this launch's part of the leaf
    uint64_t len;       // total leaf length (for the padding)
    uint64_t have;      // bytes of the leaf inside the stripe
    uint64_t nb;        // full 64-byte blocks to absorb in this launch
    bool fin;           // leaf ends inside this stripe: pad and emit the digest
    bool active;
};

template <bool TABLE>
__device__ __forceinline__ LeafView leaf_view(const LeafArgs& a, uint64_t i) {
    LeafView v{};
    v.active = i < a.nleaves;
    if (!v.active) {
        v.p = a.base;
        return v;
    }
    if constexpr (TABLE) {
        v.p = reinterpret_cast<const uint8_t*>(a.addrs[i]);
        v.len = a.lens[i];
    } else {
        v.p = a.base + i * a.pitch;
        v.len = (i + 1 == a.nleaves) ? a.last_len : a.leaf_len;
    }
    const uint64_t b0 = a.byte_off;
    const uint64_t end = v.len < a.byte_end ? v.len : a.byte_end;
    v.have = end > b0 ? end - b0 : 0;
    v.fin = (b0 < v.len && v.len <= a.byte_end) || (v.len == 0 && b0 == 0);
    v.nb = v.have / 64;   // not finishing: the stripe holds whole blocks only
    return v;
}

__device__ __forceinline__ void load_or_init_state(const LeafArgs& a, uint64_t i, uint32_t (&st)[8]) {
    if (a.state != nullptr && a.byte_off != 0) {
#pragma unroll
        for (int k = 0; k < 8; k++) st[k] = a.state[i * 8 + k];
    } else {
        init_state(st);
    }
}

// Finish a leaf after its full blocks: pad + digest, or save the chaining state for the next stripe.
template <bool ALIGNED>
__device__ __forceinline__ void leaf_epilogue(const LeafArgs& a, uint64_t i, const LeafView& v, uint32_t (&st)[8]) {
    if (v.fin) {
        absorb_tail<ALIGNED>(st, v.p + 64 * v.nb, (uint32_t)(v.have - 64 * v.nb), v.len);
        if (a.digests != nullptr) store_digest(a.digests + 32 * i, st);
    } else if (a.state != nullptr && v.have != 0) {
#pragma unroll
        for (int k = 0; k < 8; k++) a.state[i * 8 + k] = st[k];
    }
}

// Largest value over the 64 lanes of the wave (wave-uniform result).
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = __shfl_xor(x, o, 64);
        x = y > x ? y : x;
    }
    return x;
}

// K1: leaf SHA-256, one lane per leaf; optionally fused with the first tree levels.
template <bool TABLE, bool ALIGNED>
__global__ __launch_bounds__(kBlock) void leaf_kernel(LeafArgs a) {
    __shared__ uint32_t lds_a[kBlock][8];
    __shared__ uint32_t lds_b[kBlock / 2][8];
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const LeafView v = leaf_view<TABLE>(a, i);
    const bool active = v.active;
    uint32_t st[8];
    if (active) {
        load_or_init_state(a, i, st);
        absorb_blocks<ALIGNED>(st, v.p, v.nb);
        leaf_epilogue<ALIGNED>(a, i, v, st);
    }
    if (a.fuse_levels == 0) return;   // uniform across the grid
    const uint64_t first = (uint64_t)blockIdx.x * kBlock;
    const uint32_t cnt = (uint32_t)((a.nleaves - first) < kBlock ? (a.nleaves - first) : kBlock);
    if (active) {
#pragma unroll
        for (int k = 0; k < 8; k++) lds_a[threadIdx.x][k] = st[k];
    }
    __syncthreads();
    uint32_t (*res)[8];
    const uint32_t out_cnt = lds_reduce(lds_a, lds_b, cnt, a.fuse_levels, &res);
    if (threadIdx.x < out_cnt) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = res[threadIdx.x][k];
        const uint64_t o = (uint64_t)blockIdx.x * (kBlock >> a.fuse_levels) + threadIdx.x;
        store_digest(a.level_out + 32 * o, v);
    }
}

// ---------------------------------------------------------------------------------------------
// K1L: leaf SHA-256 for few, long leaves (latency regime).  A leaf's compressions form one serial
// chain, and a wave issues at most one instruction every ~4-6 cycles, so with < ~100 k leaves the
// root time is (instructions per block on the chain's wave) x (blocks per leaf).  K1L takes the
// message schedule off that wave: per 64 leaves, wave 0 ("producer") loads the blocks and writes
// K[t]+W[t] for all 64 rounds into an LDS ring; wave 1 ("consumer") only runs the rounds, reading
// 4 K+W words per ds_read_b128.  The consumer issues ~64 x 14 + 16 instructions per block instead
// of ~1,418.  Ring layout [slot][group of 4 rounds][lane] x 16 B: a wave's ds_read_b128 touches 64
// consecutive 16-byte slots (conflict-free).  Uniform-chunk, single-shot mode only.
constexpr int kLatLeaves = 64;      // leaves per workgroup (one consumer wave)
constexpr int kLatThreads = 128;    // producer wave + consumer wave
constexpr int kLatRing = 2;         // ring slots (producer runs one block ahead)
constexpr int kLatFuseMax = 6;      // 64 leaves -> 1 node

__device__ __forceinline__ void rounds_from_kw(uint32_t (&st)[8], const uint4 (*kw)[kLatLeaves], uint32_t lane) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    // K+W for 8 rounds in registers, the next 8 rounds' reads in flight (LDS latency hidden)
    uint4 x = kw[0][lane], y = kw[1][lane];
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
        uint4 nx = x, ny = y;
        if (q + 2 < 16) {
            nx = kw[q + 2][lane];
            ny = kw[q + 3][lane];
        }
        DM_SHA_ROUND(a, b, c, d, e, f, g, h, x.x);
        DM_SHA_ROUND(h, a, b, c, d, e, f, g, x.y);
        DM_SHA_ROUND(g, h, a, b, c, d, e, f, x.z);
        DM_SHA_ROUND(f, g, h, a, b, c, d, e, x.w);
        DM_SHA_ROUND(e, f, g, h, a, b, c, d, y.x);
        DM_SHA_ROUND(d, e, f, g, h, a, b, c, y.y);
        DM_SHA_ROUND(c, d, e, f, g, h, a, b, y.z);
        DM_SHA_ROUND(b, c, d, e, f, g, h, a, y.w);
        x = nx;
        y = ny;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Message schedule of one block, written as K[t]+W[t] groups of 4 into one ring slot.
__device__ __forceinline__ void schedule_to_lds(uint32_t (&w)[16], uint4 (*kw)[kLatLeaves], uint32_t lane) {
#pragma unroll
    for (int q = 0; q < 16; q++) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int t = 4 * q + j;
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {
                wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
                w[t & 15] = wt;
            }
            v[j] = kSha256K[t] + wt;
        }
        kw[q][lane] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

template <bool TABLE, bool ALIGNED>
__global__ __launch_bounds__(kLatThreads) void leaf_kernel_lat(LeafArgs a) {
    __shared__ uint4 ring[kLatRing][16][kLatLeaves];
    __shared__ uint32_t lds_a[kLatLeaves][8];
    __shared__ uint32_t lds_b[kLatLeaves / 2][8];
    const uint32_t lane = threadIdx.x & (kLatLeaves - 1);
    // wave-uniform role (readfirstlane makes the branch scalar, so the barriers below pair up)
    const bool producer = __builtin_amdgcn_readfirstlane(threadIdx.x) < kLatLeaves;
    const uint64_t first = (uint64_t)blockIdx.x * kLatLeaves;
    const uint64_t i = first + lane;
    const LeafView v = leaf_view<TABLE>(a, i);
    // trip count shared by both waves (each computes the same maximum over the 64 leaves)
    const uint64_t NB = wave_max_u64(v.nb);
    if (producer) {
        // One block (half a 128-B line) per iteration.  Loading whole lines here, as K1 does, took
        // the traffic at 64 KiB chunks from 1.047x to 1.000x but cost 3 % there and 6 % at 512 KiB
        // chunks (16,384 leaves, where K1L is chosen): profiles/r02/k1l_lines_ab/summary.log.
        Blk cur;
        if (v.nb > 0) cur = load_block<ALIGNED>(v.p);
        for (uint64_t b = 0; b < NB; b++) {
            if (b < v.nb) {
                uint32_t w[16];
                block_words(cur, w);
                if (b + 1 < v.nb) cur = load_block<ALIGNED>(v.p + 64 * (b + 1));
                schedule_to_lds(w, ring[b % kLatRing], lane);
            }
            __syncthreads();   // slot b full  /  slot b-1 free
        }
        __syncthreads();       // pairs with the consumer's final-iteration barrier
    } else {
        uint32_t st[8];
        if (v.active) load_or_init_state(a, i, st);
        else init_state(st);
        __syncthreads();       // wait for slot 0
        for (uint64_t b = 0; b < NB; b++) {
            if (b < v.nb) rounds_from_kw(st, ring[b % kLatRing], lane);
            __syncthreads();   // slot b consumed; slot b+1 full
        }
        if (v.active) {
            leaf_epilogue<ALIGNED>(a, i, v, st);
#pragma unroll
            for (int k = 0; k < 8; k++) lds_a[lane][k] = st[k];
        }
    }
    if (a.fuse_levels == 0) return;
    __syncthreads();
    const uint32_t cnt = (uint32_t)((a.nleaves - first) < kLatLeaves ? (a.nleaves - first) : kLatLeaves);
    uint32_t (*res)[8];
    const uint32_t out_cnt = lds_reduce(lds_a, lds_b, cnt, a.fuse_levels, &res);
    if (threadIdx.x < out_cnt) {
        uint32_t o8[8];
#pragma unroll
        for (int k = 0; k < 8; k++) o8[k] = res[threadIdx.x][k];
        const uint64_t o = (uint64_t)blockIdx.x * (kLatLeaves >> a.fuse_levels) + threadIdx.x;
        store_digest(a.level_out + 32 * o, o8);
    }
}

// ---------------------------------------------------------------------------------------------
// K1P: K1L with the rounds packed on lane pairs.  Consumer lanes 2c (A) and 2c+1 (B) run leaf c:
// A holds (e,f,g,h), B holds (a,b,c,d) in the same four registers X4..X7, and every instruction
// of a round does both halves with per-lane operands:
//   S = x3(rotr(X4,s1), rotr(X4,s2), rotr(X4,s3))  A: Sigma1(e)  B: Sigma0(a)   (per-lane shifts)
//   x = X4 ^ (X5 | M)                               A: ~e        B: a ^ b       (M = ~0 on A)
//   F = (x & X6) | (~x & X5)                        A: Ch(e,f,g) B: Maj(a,b,c)
//   T = S + F + (X7 & M) + KW                       A: T1        B: T2          (KW = 0 on B)
//   Y = B ? X7 : T                                  A: T1        B: d
//   X4' = T + Y[lane ^ 1]  (one DPP add)            A: d + T1    B: T1 + T2
// i.e. 11 instructions per round instead of 14; the message schedule stays on the producer.
constexpr int kPairLeaves = 32;     // leaves per workgroup (two consumer lanes per leaf)
constexpr int kPairFuseMax = 5;     // 32 leaves -> 1 node

__device__ __forceinline__ uint32_t dpp_swap_pairs(uint32_t v) {
    // quad_perm [1,0,3,2]: lane i reads lane i^1
    // old = 0 with bound_ctrl: the identity of the consuming add, so hipcc's DPP-combine pass can
    // fold this move into v_add_u32_dpp
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);
}

#define DM_PAIR_ROUND(X4, X5, X6, X7, kw)                                              \
    do {                                                                               \
        const uint32_t s_ = xor3(__builtin_amdgcn_alignbit(X4, X4, sh1),               \
                                 __builtin_amdgcn_alignbit(X4, X4, sh2),               \
                                 __builtin_amdgcn_alignbit(X4, X4, sh3));              \
        const uint32_t x_ = __builtin_amdgcn_bitop3_b32(X4, X5, msk, 0x1e);            \
        const uint32_t f_ = __builtin_amdgcn_bitop3_b32(x_, X6, X5, 0xca);             \
        const uint32_t t_ = s_ + f_ + ((X7 & msk) + (kw));                             \
        const uint32_t y_ = lane_b ? X7 : t_;                                          \
        X7 = t_ + dpp_swap_pairs(y_);                                                  \
    } while (0)

__device__ __forceinline__ void pair_rounds_from_kw(uint32_t (&x)[4], const uint4 (*kw)[kLatLeaves], uint32_t lane,
                                                    uint32_t sh1, uint32_t sh2, uint32_t sh3, uint32_t msk,
                                                    bool lane_b) {
    uint32_t x4 = x[0], x5 = x[1], x6 = x[2], x7 = x[3];
    uint4 q = kw[0][lane];
#pragma unroll
    for (int g = 0; g < 16; g++) {
        uint4 nq = q;
        if (g + 1 < 16) nq = kw[g + 1][lane];
        // register roles rotate: after a round, the new value X4' lands in the old X7 register
        DM_PAIR_ROUND(x4, x5, x6, x7, q.x);   // new x4 in x7
        DM_PAIR_ROUND(x7, x4, x5, x6, q.y);   // new in x6
        DM_PAIR_ROUND(x6, x7, x4, x5, q.z);   // new in x5
        DM_PAIR_ROUND(x5, x6, x7, x4, q.w);   // new in x4
        q = nq;
    }
    x[0] += x4; x[1] += x5; x[2] += x6; x[3] += x7;
}

template <bool TABLE, bool ALIGNED>
__global__ __launch_bounds__(kLatThreads) void leaf_kernel_pair(LeafArgs a) {
    __shared__ uint4 ring[kLatRing][16][kLatLeaves];
    __shared__ uint32_t lds_a[kPairLeaves][8];
    __shared__ uint32_t lds_b[kPairLeaves / 2][8];
    const uint32_t lane = threadIdx.x & (kLatLeaves - 1);
    const bool producer = __builtin_amdgcn_readfirstlane(threadIdx.x) < kLatLeaves;
    const bool lane_b = (lane & 1) != 0;
    const uint32_t c = lane >> 1;                           // leaf within the workgroup
    const uint64_t first = (uint64_t)blockIdx.x * kPairLeaves;
    const uint64_t i = first + c;
    const LeafView v = leaf_view<TABLE>(a, i);
    const uint64_t NB = wave_max_u64(v.nb);
    if (producer) {
        // even lanes compute leaf c's K+W; odd lanes publish zeros (the B half adds no K+W)
        Blk cur;
        if (v.nb > 0 && !lane_b) cur = load_block<ALIGNED>(v.p);
        for (uint64_t b = 0; b < NB; b++) {
            if (b < v.nb) {
                uint32_t w[16];
                block_words(cur, w);
                if (b + 1 < v.nb && !lane_b) cur = load_block<ALIGNED>(v.p + 64 * (b + 1));
                uint4 (*kw)[kLatLeaves] = ring[b % kLatRing];
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    uint32_t u[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int t = 4 * q + j;
                        uint32_t wt;
                        if (t < 16) {
                            wt = w[t];
                        } else {
                            wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
                            w[t & 15] = wt;
                        }
                        u[j] = lane_b ? 0u : kSha256K[t] + wt;
                    }
                    kw[q][lane] = make_uint4(u[0], u[1], u[2], u[3]);
                }
            }
            __syncthreads();
        }
        __syncthreads();
    } else {
        // per-lane constants of the packed round
        const uint32_t sh1 = lane_b ? 2 : 6, sh2 = lane_b ? 13 : 11, sh3 = lane_b ? 22 : 25;
        const uint32_t msk = lane_b ? 0u : ~0u;
        uint32_t st0[8];
        if (v.active) load_or_init_state(a, i, st0);
        else init_state(st0);
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; k++) x[k] = lane_b ? st0[k] : st0[4 + k];
        __syncthreads();
        for (uint64_t b = 0; b < NB; b++) {
            if (b < v.nb) pair_rounds_from_kw(x, ring[b % kLatRing], lane, sh1, sh2, sh3, msk, lane_b);
            __syncthreads();
        }
        // reassemble the full state on lane A: (a,b,c,d) from lane B, (e,f,g,h) own
        uint32_t st[8];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t other = dpp_swap_pairs(x[k]);
            st[k] = lane_b ? x[k] : other;
            st[4 + k] = lane_b ? other : x[k];
        }
        if (v.active && !lane_b) {
            leaf_epilogue<ALIGNED>(a, i, v, st);
#pragma unroll
            for (int k = 0; k < 8; k++) lds_a[c][k] = st[k];
        }
    }
    if (a.fuse_levels == 0) return;
    __syncthreads();
    const uint32_t cnt = (uint32_t)((a.nleaves - first) < kPairLeaves ? (a.nleaves - first) : kPairLeaves);
    uint32_t (*res)[8];
    const uint32_t out_cnt = lds_reduce(lds_a, lds_b, cnt, a.fuse_levels, &res);
    if (threadIdx.x < out_cnt) {
        uint32_t o8[8];
#pragma unroll
        for (int k = 0; k < 8; k++) o8[k] = res[threadIdx.x][k];
        const uint64_t o = (uint64_t)blockIdx.x * (kPairLeaves >> a.fuse_levels) + threadIdx.x;
        store_digest(a.level_out + 32 * o, o8);
    }
}

// ---------------------------------------------------------------------------------------------
// K1Q: the rounds of one leaf spread over 8 lanes, for the fewest, longest leaves.  In K1P the
// consumer wave still issues 3 rotations + an xor3 per Sigma; here each of three lanes does one
// rotation (one v_alignbit with a per-lane shift) and two DPP xors combine them, so every lane of
// the triple holds Sigma.  Leaf c owns two quads of one 16-lane row, 8 lanes apart: the e-triple
// (lanes 0..2 of the quad, holding e,f,g,h) and the a-triple (a,b,c,d); lane 3 of each quad idles.
// The a-triple runs two rounds behind the e-triple: round s of e needs d(s) = a(s-3), which the
// a-triple finished a step earlier, and round s-2 of a needs T1(s-2) = e(s-1) - d(s-2), which the
// e-triple finished a step earlier -- so one symmetric DPP add (row_ror:8) per step moves both,
// off the dependent chain.  Per step, with per-lane constants (e / a):
//   R  = rotr(X4, s)                        s = 6,11,25 / 2,13,22
//   S  = R ^ R[q1] ^ R[q2]  (two DPP xors)  Sigma1(e) / Sigma0(a)
//   F  = bitop3 pair of K1P                 Ch(e,f,g) / Maj(a,b,c)
//   X7 = S + F + H                          e(s+1) / a(s-1)
//   HN = (X6 ^ N) + V + X4[lane ^ 8]        next H: h + KW + d / T1 = e - d   (N = 0 / ~0, V = KW / 1)
// 8 instructions per step, a 4-deep chain (alignbit, xor, xor, add3); 66 steps per 64-byte block.
// The earlier lock-step form (both triples on one round, two bank-masked exchanges) took 9
// instructions and a 5-deep chain: 669.9 -> 625.7 ms for the 8 GiB / 32 MiB headline.  The
// producer wave gives each of a leaf's 8 lanes its own block (8 consecutive blocks per ring
// stage, 512 contiguous bytes per leaf per load), so one producer wave keeps up with the consumer.
// LDS: K+W ring [stage][group of 4 rounds][block][leaf] x 16 B (a producer store is 64
// consecutive uint4; a consumer load is 8 distinct uint4, each broadcast to a leaf's lanes), and
// a same-shaped region of ones that the a-triple reads instead (its V is the constant 1).
constexpr int kQuadLeaves = 8;      // leaves per workgroup (8 consumer lanes per leaf)
constexpr int kQuadBlocks = 8;      // blocks per leaf per ring stage (one producer lane each)
constexpr int kQuadFuseMax = 3;     // 8 leaves -> 1 node
// Two LDS footprints (template COMPACT), one ring layout: -(K+W) [stage][group][block][leaf].
// Wide reserves a second, unused 32 KiB region so that at most two workgroups share a CU and the
// dispatcher spreads them; compact (33 KiB, four per CU) is used for 4,097 .. 8,192 leaves.  The
// lock-step K1Q needed a region of ones for its a-triple (wide) or one broadcast ones entry per
// row (compact, 9-entry rows); the skewed step needs neither.
constexpr int kQuadRow = kQuadLeaves;
constexpr size_t kQuadLdsBytes = sizeof(uint4) * kLatRing * 16 * kQuadBlocks * kQuadRow + 4 * 8 * kQuadLeaves +
                                 4 * 8 * (kQuadLeaves / 2);
static_assert(4 * kQuadLdsBytes <= (160u << 10), "four compact K1Q workgroups must fit a CU's LDS");

// One skewed step, hand-scheduled (8 VALU, two of them half-rate): the e-triple runs round s,
// the a-triple round s-2.  H is this step's add3 term (made by the previous step), HN the next
// step's.  V = -(K+W) of round s+1 from the producer.
//   F  = Ch / Maj                    (reads X6 before it is reused)
//   X6 = V - X6   on the e-triple    -(h(s+1) + KW(s+1)); X6 is dead after F until the next
//                                    step's add3 overwrites it (it is that step's X7)
//   HN = X4[lane ^ 8] - X6           e: d(s+1) + h + KW          a: e(s) - d(s-1) = T1(s-1)
//   X7 = Sigma + F + H               e: e(s+1)                   a: a(s-1) = T1 + T2 of round s-2
// The row_ror:8 DPP subtract is the whole exchange: each leaf's e-quad and a-quad sit 8 lanes
// apart in one 16-lane row, so the same instruction hands a(s-2) to the e-triple and e(s) to the
// a-triple.  Both H instructions are full-rate DPP ops (a v_xad with a per-lane negate cost a
// half-rate slot).  hipcc re-associates DPP xors and cannot emit bank-masked DPP ops, so the
// steps are written out.  Wait states: every DPP source VGPR is written at least two
// instructions earlier.
#ifndef DM_QS_DEEP3
#define DM_QS_DEEP3 0
#endif
#if DM_QS_DEEP3
// Experiment ("3-deep e-chain"; A/B only, tools/deep3_ab.sh): every lane of a triple
// makes all three rotations itself (sh / sh2 / sh3 = 6,11,25 or 2,13,22) and one xor3 gives Sigma,
// so the chain is alignbit -> xor3 -> add3 (3 deep) at 9 instructions per step instead of 8.
#define DM_QS_HEAD(X4, X5, X6)                                                                   \
    "v_alignbit_b32 %[r], %[" X4 "], %[" X4 "], %[sh]\n\t"                                      \
    "v_alignbit_b32 %[s], %[" X4 "], %[" X4 "], %[sh2]\n\t"                                     \
    "v_alignbit_b32 %[t], %[" X4 "], %[" X4 "], %[sh3]\n\t"                                     \
    "v_bitop3_b32 %[f], %[" X4 "], %[" X5 "], %[msk] bitop3:0x1e\n\t"                          \
    "v_bitop3_b32 %[f], %[f], %[" X6 "], %[" X5 "] bitop3:0xca\n\t"
#define DM_QS_SIGMA "v_bitop3_b32 %[s], %[r], %[s], %[t] bitop3:0x96\n\t"
#else
#define DM_QS_HEAD(X4, X5, X6)                                                                   \
    "v_alignbit_b32 %[r], %[" X4 "], %[" X4 "], %[sh]\n\t"                                      \
    "v_bitop3_b32 %[f], %[" X4 "], %[" X5 "], %[msk] bitop3:0x1e\n\t"                          \
    "v_bitop3_b32 %[f], %[f], %[" X6 "], %[" X5 "] bitop3:0xca\n\t"                             \
    "v_xor_b32_dpp %[s], %[r], %[r] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t"
#define DM_QS_SIGMA "v_xor_b32_dpp %[s], %[r], %[s] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"
#endif
// VN's round comes from lane QP of the quad (QP = "[0,1,2,3]": every lane holds it, the generic
// path; "[j,j,j,j]": the register path's lane j holds it, see quad_block_regs)
#define DM_QS_STEP_Q(X4, X5, X6, X7, H, HN, VN, QP)                                             \
    DM_QS_HEAD(X4, X5, X6)                                                                       \
    "v_sub_u32_dpp %[" X6 "], %[" VN "], %[" X6 "] quad_perm:" QP " row_mask:0xf bank_mask:0x3\n\t" \
    DM_QS_SIGMA                                                                                  \
    "v_sub_u32_dpp %[" HN "], %[" X4 "], %[" X6 "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"    \
    "v_add3_u32 %[" X7 "], %[s], %[f], %[" H "]\n\t"
#define DM_QS_STEP(X4, X5, X6, X7, H, HN, VN) DM_QS_STEP_Q(X4, X5, X6, X7, H, HN, VN, "[0,1,2,3]")
// e-triple idle next step (steps 63, 64): keep X6 (the e-triple feeds forward from it), HN only
// matters on the a-triple
#define DM_QS_STEP_A(X4, X5, X6, X7, H, HN)                                                     \
    DM_QS_HEAD(X4, X5, X6)                                                                       \
    DM_QS_SIGMA                                                                                  \
    "v_sub_u32_dpp %[" HN "], %[" X4 "], %[" X6 "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"    \
    "v_add3_u32 %[" X7 "], %[s], %[f], %[" H "]\n\t"
// last step of a block: no next H
#define DM_QS_STEP_END(X4, X5, X6, X7, H)                                                       \
    DM_QS_HEAD(X4, X5, X6)                                                                       \
    DM_QS_SIGMA                                                                                  \
    "v_add3_u32 %[" X7 "], %[s], %[f], %[" H "]\n\t"
// four steps; the role registers rotate through P0..P3 = a, b, c, d and H alternates h / g
#define DM_QS_STEPS4V(V0, V1, V2, V3)                                                          \
    DM_QS_STEP("a", "b", "c", "d", "h", "g", V0) DM_QS_STEP("d", "a", "b", "c", "g", "h", V1)   \
    DM_QS_STEP("c", "d", "a", "b", "h", "g", V2) DM_QS_STEP("b", "c", "d", "a", "g", "h", V3)
// Every K1Q step instruction is 8 bytes, and where the stream sits mod 8 changes the rate.
// Measured on MI355X with one s_nop 0 shifted in front of otherwise identical code: a stream at
// addresses = 0 mod 8 runs the wide (<= 2 workgroups per CU) launch at 15.84 GiB/s (256 leaves)
// and the compact (4 per CU) launch at 320 GiB/s (8,192 leaves); at 4 mod 8 the wide launch
// drops to 12.85 and the compact one rises to 368 (reproducible over every odd and even shift,
// profiles/r01/r01f_align_ab.log).  So each step stream is pinned: 8-byte aligned, plus one 4-byte
// s_nop for the compact kernel (MIS).  Cause not isolated (instruction fetch / issue arbitration
// between the two waves sharing a SIMD in the compact case).
#define DM_QS_ALIGN ".p2align 3\n\t"
#define DM_QS_ALIGN_MIS ".p2align 3\n\t.if %[mis]\n\ts_nop 0\n\t.endif\n\t"
#define DM_QS_PROLOGUE(V) DM_QS_PROLOGUE_AT(V, DM_QS_ALIGN, "[0,1,2,3]")
// H of step 0, as if made by step -1 (X6 = P3, X4 = P1); P may have just been copied from x
#define DM_QS_PROLOGUE_AT(V, ALIGN, QP)                                                           \
    "s_nop 1\n\t" ALIGN                                                                          \
    "v_sub_u32_dpp %[d], %[" V "], %[d] quad_perm:" QP " row_mask:0xf bank_mask:0x3\n\t"         \
    "v_sub_u32_dpp %[h], %[b], %[d] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
// steps 0..3: the a-triple's first two steps run on stale values; their writes to P3 and P2 are
// replaced by b and a (a-quads only) before anything reads them
#define DM_QS_RESTORE_A(P, X) "v_mov_b32_dpp %[" P "], %[" X "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n\t"
#define DM_QS_GROUP0(V0, V1, V2, V3)                                                             \
    DM_QS_STEP("a", "b", "c", "d", "h", "g", V0) DM_QS_RESTORE_A("d", "x3")                      \
    DM_QS_STEP("d", "a", "b", "c", "g", "h", V1) DM_QS_RESTORE_A("c", "x2")                      \
    DM_QS_STEP("c", "d", "a", "b", "h", "g", V2) DM_QS_STEP("b", "c", "d", "a", "g", "h", V3)
// steps 60..65 and both feed-forwards: the e-triple after step 63 (P0 written last), the
// a-triple after step 65 (P2 written last).  FF: x += P on one lane type (bank 0x3 = e-quads,
// 0xc = a-quads).
#define DM_QS_FF(X, P, BANKS) "v_add_u32_dpp %[" X "], %[" P "], %[" X "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" BANKS "\n\t"
#define DM_QS_TAIL(V0, V1, V2)                                                                   \
    DM_QS_STEP("a", "b", "c", "d", "h", "g", V0) DM_QS_STEP("d", "a", "b", "c", "g", "h", V1)   \
    DM_QS_STEP("c", "d", "a", "b", "h", "g", V2) DM_QS_STEP_A("b", "c", "d", "a", "g", "h")      \
    DM_QS_FF("x3", "d", "0x3") DM_QS_FF("x2", "c", "0x3") DM_QS_FF("x1", "b", "0x3")             \
    DM_QS_FF("x0", "a", "0x3")                                                                   \
    DM_QS_STEP_A("a", "b", "c", "d", "h", "g") DM_QS_STEP_END("d", "a", "b", "c", "g")           \
    DM_QS_FF("x0", "a", "0xc") DM_QS_FF("x1", "b", "0xc") DM_QS_FF("x3", "d", "0xc")             \
    DM_QS_FF("x2", "c", "0xc")
// The same groups with each step's VN taken from a quad lane (quad_block_regs' register path)
#define DM_QS_STEPS4Q(V0, Q0, V1, Q1, V2, Q2, V3, Q3)                                          \
    DM_QS_STEP_Q("a", "b", "c", "d", "h", "g", V0, Q0) DM_QS_STEP_Q("d", "a", "b", "c", "g", "h", V1, Q1) \
    DM_QS_STEP_Q("c", "d", "a", "b", "h", "g", V2, Q2) DM_QS_STEP_Q("b", "c", "d", "a", "g", "h", V3, Q3)
#define DM_QS_GROUP0Q(V0, Q0, V1, Q1, V2, Q2, V3, Q3)                                          \
    DM_QS_STEP_Q("a", "b", "c", "d", "h", "g", V0, Q0) DM_QS_RESTORE_A("d", "x3")              \
    DM_QS_STEP_Q("d", "a", "b", "c", "g", "h", V1, Q1) DM_QS_RESTORE_A("c", "x2")              \
    DM_QS_STEP_Q("c", "d", "a", "b", "h", "g", V2, Q2) DM_QS_STEP_Q("b", "c", "d", "a", "g", "h", V3, Q3)
#define DM_QS_TAILQ(V0, Q0, V1, Q1, V2, Q2)                                                     \
    DM_QS_STEP_Q("a", "b", "c", "d", "h", "g", V0, Q0) DM_QS_STEP_Q("d", "a", "b", "c", "g", "h", V1, Q1) \
    DM_QS_STEP_Q("c", "d", "a", "b", "h", "g", V2, Q2) DM_QS_STEP_A("b", "c", "d", "a", "g", "h") \
    DM_QS_FF("x3", "d", "0x3") DM_QS_FF("x2", "c", "0x3") DM_QS_FF("x1", "b", "0x3")             \
    DM_QS_FF("x0", "a", "0x3")                                                                   \
    DM_QS_STEP_A("a", "b", "c", "d", "h", "g") DM_QS_STEP_END("d", "a", "b", "c", "g")           \
    DM_QS_FF("x0", "a", "0xc") DM_QS_FF("x1", "b", "0xc") DM_QS_FF("x3", "d", "0xc")             \
    DM_QS_FF("x2", "c", "0xc")
#if DM_QS_DEEP3
#define DM_QS_XOUT , [t] "=&v"(t_)
#define DM_QS_XIN , [sh2] "v"(sh.y), [sh3] "v"(sh.z)
#else
#define DM_QS_XOUT
#define DM_QS_XIN
#endif
#define DM_QS_OUT                                                                                \
    : [a] "+v"(p0), [b] "+v"(p1), [c] "+v"(p2), [d] "+v"(p3), [h] "+v"(h), [g] "+v"(g),           \
      [x0] "+v"(x[0]), [x1] "+v"(x[1]), [x2] "+v"(x[2]), [x3] "+v"(x[3]), [r] "=&v"(r_),          \
      [f] "=&v"(f_), [s] "=&v"(s_) DM_QS_XOUT
#define DM_QS_OPS DM_QS_OUT : [sh] "v"(sh.x), [msk] "v"(msk), [v0] "v"(v0), [v1] "v"(v1), [v2] "v"(v2), [v3] "v"(v3) DM_QS_XIN

// One 64-byte block from the ring: 66 skewed steps (the a-triple starts two steps late and
// finishes two steps after the e-triple).  x = this lane's chaining words: e-triple (e,f,g,h),
// a-triple (c,d,a,b) -- stored rotated so that both triples start from P = x and feed forward
// x += P.  kw(grp) gives -(K+W) of rounds 4grp..4grp+3 (an LDS read).
template <class KW>
__device__ __forceinline__ void quad_block_skewed(uint32_t (&x)[4], KW kw, uint3 sh, uint32_t msk) {
    uint32_t p0 = x[0], p1 = x[1], p2 = x[2], p3 = x[3], h = 0, g = 0, r_, f_, s_, t_;
    (void)t_;
    uint4 q = kw(0), nq = kw(1);
    {
        const uint32_t v0 = q.x, v1 = 0, v2 = 0, v3 = 0;
        asm volatile(DM_QS_PROLOGUE("v0") DM_QS_OPS);
    }
#pragma unroll
    for (int grp = 0; grp < 16; grp++) {
        // the group after next is loaded now, so its LDS latency hides behind this group's steps
        const uint4 nnq = grp + 2 < 16 ? kw(grp + 2) : nq;
        const uint32_t v0 = q.y, v1 = q.z, v2 = q.w, v3 = nq.x;
        if (grp == 0) {
            asm volatile(DM_QS_ALIGN DM_QS_GROUP0("v0", "v1", "v2", "v3") DM_QS_OPS);
        } else if (grp < 15) {
            asm volatile(DM_QS_ALIGN DM_QS_STEPS4V("v0", "v1", "v2", "v3") DM_QS_OPS);
        } else {
            asm volatile(DM_QS_ALIGN DM_QS_TAIL("v0", "v1", "v2") DM_QS_OPS);
        }
        q = nq;
        nq = nnq;
    }
}

constexpr int kLgkmWait0 = 0xC07F;   // s_waitcnt lgkmcnt(0), no wait on vmcnt / expcnt (gfx9 encoding)

// quad_block_skewed with the block's 64 words of -(K+W) in registers: the whole block is one asm
// statement (hipcc puts an s_nop between asm statements that share registers).  The 64 words are
// spread over the 4 lanes of a quad: lane j's K[t] holds rounds 16t + 4j .. 16t + 4j + 3, and
// round r's step reads its word from quad lane (r mod 16) / 4 by DPP (quad_perm [j,j,j,j]), so a
// block takes 4 ds_read_b128 per lane instead of 16 (issue slots on the chain's wave) and 16
// VGPRs instead of 64 (generated by the loop in this comment's commit: round r -> q{r/16}{r%4}).
template <bool MIS>
__device__ __forceinline__ void quad_block_regs(uint32_t (&x)[4], const uint4 (&K)[4], uint3 sh, uint32_t msk) {
    uint32_t p0 = x[0], p1 = x[1], p2 = x[2], p3 = x[3], h, g, r_, f_, s_, t_;
    (void)t_;
    asm volatile(DM_QS_PROLOGUE_AT("q00", DM_QS_ALIGN_MIS, "[0,0,0,0]")
                 DM_QS_GROUP0Q("q01", "[0,0,0,0]", "q02", "[0,0,0,0]", "q03", "[0,0,0,0]", "q00", "[1,1,1,1]")
                 DM_QS_STEPS4Q("q01", "[1,1,1,1]", "q02", "[1,1,1,1]", "q03", "[1,1,1,1]", "q00", "[2,2,2,2]")
                 DM_QS_STEPS4Q("q01", "[2,2,2,2]", "q02", "[2,2,2,2]", "q03", "[2,2,2,2]", "q00", "[3,3,3,3]")
                 DM_QS_STEPS4Q("q01", "[3,3,3,3]", "q02", "[3,3,3,3]", "q03", "[3,3,3,3]", "q10", "[0,0,0,0]")
                 DM_QS_STEPS4Q("q11", "[0,0,0,0]", "q12", "[0,0,0,0]", "q13", "[0,0,0,0]", "q10", "[1,1,1,1]")
                 DM_QS_STEPS4Q("q11", "[1,1,1,1]", "q12", "[1,1,1,1]", "q13", "[1,1,1,1]", "q10", "[2,2,2,2]")
                 DM_QS_STEPS4Q("q11", "[2,2,2,2]", "q12", "[2,2,2,2]", "q13", "[2,2,2,2]", "q10", "[3,3,3,3]")
                 DM_QS_STEPS4Q("q11", "[3,3,3,3]", "q12", "[3,3,3,3]", "q13", "[3,3,3,3]", "q20", "[0,0,0,0]")
                 DM_QS_STEPS4Q("q21", "[0,0,0,0]", "q22", "[0,0,0,0]", "q23", "[0,0,0,0]", "q20", "[1,1,1,1]")
                 DM_QS_STEPS4Q("q21", "[1,1,1,1]", "q22", "[1,1,1,1]", "q23", "[1,1,1,1]", "q20", "[2,2,2,2]")
                 DM_QS_STEPS4Q("q21", "[2,2,2,2]", "q22", "[2,2,2,2]", "q23", "[2,2,2,2]", "q20", "[3,3,3,3]")
                 DM_QS_STEPS4Q("q21", "[3,3,3,3]", "q22", "[3,3,3,3]", "q23", "[3,3,3,3]", "q30", "[0,0,0,0]")
                 DM_QS_STEPS4Q("q31", "[0,0,0,0]", "q32", "[0,0,0,0]", "q33", "[0,0,0,0]", "q30", "[1,1,1,1]")
                 DM_QS_STEPS4Q("q31", "[1,1,1,1]", "q32", "[1,1,1,1]", "q33", "[1,1,1,1]", "q30", "[2,2,2,2]")
                 DM_QS_STEPS4Q("q31", "[2,2,2,2]", "q32", "[2,2,2,2]", "q33", "[2,2,2,2]", "q30", "[3,3,3,3]")
                 DM_QS_TAILQ("q31", "[3,3,3,3]", "q32", "[3,3,3,3]", "q33", "[3,3,3,3]")
                 : [a] "+v"(p0), [b] "+v"(p1), [c] "+v"(p2), [d] "+v"(p3), [h] "=&v"(h), [g] "=&v"(g),
                   [x0] "+v"(x[0]), [x1] "+v"(x[1]), [x2] "+v"(x[2]), [x3] "+v"(x[3]), [r] "=&v"(r_),
                   [f] "=&v"(f_), [s] "=&v"(s_) DM_QS_XOUT
                 : [mis] "i"(MIS ? 1 : 0), [sh] "v"(sh.x), [msk] "v"(msk),
                   [q00] "v"(K[0].x), [q01] "v"(K[0].y), [q02] "v"(K[0].z), [q03] "v"(K[0].w),
                   [q10] "v"(K[1].x), [q11] "v"(K[1].y), [q12] "v"(K[1].z), [q13] "v"(K[1].w),
                   [q20] "v"(K[2].x), [q21] "v"(K[2].y), [q22] "v"(K[2].z), [q23] "v"(K[2].w),
                   [q30] "v"(K[3].x), [q31] "v"(K[3].y), [q32] "v"(K[3].z), [q33] "v"(K[3].w) DM_QS_XIN);
}

// One ring stage (8 blocks) when every leaf of the wave has all 8: each block's 64 K+W words go
// to registers in one burst while the previous block runs (one s_waitcnt per block instead of
// one per 4 rounds), and no per-block branch.  kw: this lane's column (quad lane p's groups
// 4t + p, see quad_block_regs).
template <int G, int ROW, bool MIS>
__device__ __forceinline__ void quad_stage_regs(uint32_t (&x)[4], const uint4* kw, uint3 sh, uint32_t msk) {
    uint4 A[4], B[4];
#pragma unroll
    for (int t = 0; t < 4; t++) A[t] = kw[4 * t * G];
#pragma unroll
    for (int k = 0; k < kQuadBlocks; k += 2) {
        __builtin_amdgcn_s_waitcnt(kLgkmWait0);
#pragma unroll
        for (int t = 0; t < 4; t++) B[t] = kw[(k + 1) * ROW + 4 * t * G];
        quad_block_regs<MIS>(x, A, sh, msk);
        __builtin_amdgcn_s_waitcnt(kLgkmWait0);
        if (k + 2 < kQuadBlocks) {
#pragma unroll
            for (int t = 0; t < 4; t++) A[t] = kw[(k + 2) * ROW + 4 * t * G];
        }
        quad_block_regs<MIS>(x, B, sh, msk);
    }
}

template <bool TABLE, bool ALIGNED, bool COMPACT>
__global__ __launch_bounds__(kLatThreads) void leaf_kernel_quad(LeafArgs a) {
    constexpr int ROW = COMPACT ? kQuadRow : kQuadLeaves;     // uint4 per (group, block) row
    constexpr int G = kQuadBlocks * ROW;                      // uint4 per group row
    // -(K+W) [stage][group][block][leaf (compact: + one unused entry)].  The wide layout reserves a
    // second, unused region: 64 KiB caps it at two workgroups per CU, so the dispatcher spreads
    // them (at 32 KiB it packed four on some CUs and none on others: 4,096 x 4 MiB measured
    // 96.6 instead of 65.4 ms).
    __shared__ uint4 ring[COMPACT ? 1 : 2][kLatRing][16][G];
    __shared__ uint32_t lds_a[kQuadLeaves][8];
    __shared__ uint32_t lds_b[kQuadLeaves / 2][8];
    const uint32_t lane = threadIdx.x & 63;
    const bool producer = __builtin_amdgcn_readfirstlane(threadIdx.x) < 64;
    const uint32_t c = lane >> 3;                             // leaf within the workgroup
    const uint32_t j = lane & 7;                              // producer: block j of leaf c
    const uint64_t first = (uint64_t)blockIdx.x * kQuadLeaves;
    const uint64_t i = first + c;
    const LeafView v = leaf_view<TABLE>(a, i);
    const uint64_t NB = wave_max_u64(v.nb);
    const uint64_t NI = (NB + kQuadBlocks - 1) / kQuadBlocks;
    if (producer) {
        // lane (c, j) schedules blocks j, j+8, j+16, ... of leaf c
        Blk cur;
        if (j < v.nb) cur = load_block<ALIGNED>(v.p + 64 * j);
        for (uint64_t it = 0; it < NI; it++) {
            const uint64_t b = it * kQuadBlocks + j;
            if (b < v.nb) {
                uint32_t w[16];
                block_words(cur, w);
                if (b + kQuadBlocks < v.nb) cur = load_block<ALIGNED>(v.p + 64 * (b + kQuadBlocks));
                uint4* kw = &ring[0][it % kLatRing][0][j * ROW + c];
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    uint32_t u[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int t = 4 * q + k;
                        uint32_t wt;
                        if (t < 16) {
                            wt = w[t];
                        } else {
                            wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
                            w[t & 15] = wt;
                        }
                        u[k] = 0u - (kSha256K[t] + wt);   // the consumer subtracts it
                    }
                    kw[q * G] = make_uint4(u[0], u[1], u[2], u[3]);
                }
            }
            __syncthreads();   // stage it full  /  stage it-1 free
        }
        __syncthreads();
    } else {
        // The consumer carries the serial chains: give it issue priority over a producer or a
        // second consumer on its SIMD.  Measured on MI355X (tools/ab_builds.sh,
        // profiles/r01/LOGS.md#r01g_prio_ab.log): 8,192 x 1 MiB leaves 367 -> 401 GiB/s, 256 x 32 MiB
        // 15.82 -> 15.90, other K1Q shapes unchanged (priority 1 and 3 alike).
        __builtin_amdgcn_s_setprio(1);
        // lanes: leaf cq's e-quad = row lanes 4*(cq&1)+0..3, its a-quad 8 lanes higher (row_ror:8)
        const uint32_t cq = 2 * (lane >> 4) + ((lane >> 2) & 1);
        const bool role_a = (lane >> 3) & 1;
        const uint32_t p = lane & 3;
        const uint64_t iq = first + cq;
        const LeafView vq = leaf_view<TABLE>(a, iq);
#if DM_QS_DEEP3
        const uint3 sh = role_a ? make_uint3(2, 13, 22) : make_uint3(6, 11, 25);
#else
        const uint3 sh = make_uint3(role_a ? (p == 0 ? 2 : p == 1 ? 13 : 22) : (p == 0 ? 6 : p == 1 ? 11 : 25), 0, 0);
#endif
        const uint32_t msk = role_a ? 0u : ~0u;
        uint32_t st0[8];
        if (vq.active) load_or_init_state(a, iq, st0);
        else init_state(st0);
        uint32_t x[4];   // e-triple (e,f,g,h); a-triple (c,d,a,b)
#pragma unroll
        for (int k = 0; k < 4; k++) x[k] = role_a ? st0[(k + 2) & 3] : st0[4 + k];
        const uint4* col = &ring[0][0][0][cq];   // the a-triple reads it too (and ignores it)
        __syncthreads();
        // xf: the leaf's state after its last block.  A stage takes the register path (all 8 blocks,
        // no per-block branch) unless some leaf of the wave ENDS strictly inside it; leaves that
        // ended in an earlier stage run it too, on stale ring words, and keep their result in xf.
        // (Before: the register path only while every leaf still had all 8 blocks, so a wave mixing
        // lengths -- a FullProcessing segment beside its 4x shorter fragments, a short last chunk --
        // ran its longest chain on the per-block path once the shortest leaf ended: 1 MiB upload
        // 490 -> 613-719 ms of leaf kernel.)
        uint32_t xf[4];
#pragma unroll
        for (int k = 0; k < 4; k++) xf[k] = x[k];
        // a leaf of the wave ends strictly inside stage it
        auto partial = [&](uint64_t it) {
            const uint64_t b0 = it * kQuadBlocks;
            return __any(vq.active && vq.nb > b0 && vq.nb < b0 + kQuadBlocks);
        };
        for (uint64_t it = 0; it < NI;) {
            // runs of whole stages: their own loop, so the register path compiles (and is counted
            // by deoss_amd/isa.py) without the per-block path inside it
            for (; it < NI && !partial(it); it++) {
                quad_stage_regs<G, ROW, COMPACT>(x, col + (it % kLatRing) * 16 * G + p * G, sh, msk);
                if (vq.nb > it * kQuadBlocks) {   // this stage advanced the leaf
#pragma unroll
                    for (int k = 0; k < 4; k++) xf[k] = x[k];
                }
                __syncthreads();
            }
            if (it == NI) break;
            const uint4* kw = col + (it % kLatRing) * 16 * G;
            const uint64_t b0 = it * kQuadBlocks;
            for (uint32_t k = 0; k < kQuadBlocks; k++) {
                const uint4* kb = kw + k * ROW;
                if (b0 + k < vq.nb)
                    quad_block_skewed(x, [kb](int g) { return kb[g * G]; }, sh, msk);
            }
            if (vq.nb > b0) {
#pragma unroll
                for (int k = 0; k < 4; k++) xf[k] = x[k];
            }
            __syncthreads();
            it++;
        }
        // full state on the e-quad's first lane: (a,b,c,d) from the a-quad 8 lanes up
        uint32_t st[8];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            st[k] = __shfl(xf[(k + 2) & 3], (int)(lane + 8), 64);
            st[4 + k] = xf[k];
        }
        if (vq.active && !role_a && p == 0) {
            leaf_epilogue<ALIGNED>(a, iq, vq, st);
#pragma unroll
            for (int k = 0; k < 8; k++) lds_a[cq][k] = st[k];
        }
    }
    if (a.fuse_levels == 0) return;
    __syncthreads();
    const uint32_t cnt = (uint32_t)((a.nleaves - first) < kQuadLeaves ? (a.nleaves - first) : kQuadLeaves);
    uint32_t (*res)[8];
    const uint32_t out_cnt = lds_reduce(lds_a, lds_b, cnt, a.fuse_levels, &res);
    if (threadIdx.x < out_cnt) {
        uint32_t o8[8];
#pragma unroll
        for (int k = 0; k < 8; k++) o8[k] = res[threadIdx.x][k];
        const uint64_t o = (uint64_t)blockIdx.x * (kQuadLeaves >> a.fuse_levels) + threadIdx.x;
        store_digest(a.level_out + 32 * o, o8);
    }
}

// Empty kernel with the compact K1Q's workgroup shape (128 threads, its LDS as dynamic LDS),
// launched just before it.  Measured on MI355X: a compact K1Q launch that directly follows a
// kernel of another shape (e.g. K3, 256-thread workgroups) runs with fewer workgroups resident
// -- 70.7 instead of 42.3 ms for 6,144 x 2 MiB leaves, same wave-cycles (PMC), no overlap in the
// kernel trace -- and one 4-per-CU grid of this no-op first restores it (42.3 ms).  The cause
// is in the dispatcher's state, not in the kernel; the primer costs microseconds.
__global__ __launch_bounds__(kLatThreads) void quad_shape_primer(int x) {
    extern __shared__ uint4 dyn[];
    if (x == 12345) dyn[threadIdx.x] = make_uint4(1, 1, 1, 1);
}

// K2: tree reduce, `levels` (1..9) levels over tiles of 512 input nodes; the first level reads
// global memory directly, the rest run in LDS.  Output: ceil(m / 2^levels) nodes.
__global__ __launch_bounds__(kBlock) void reduce_kernel(const uint8_t* in, uint64_t m, uint32_t levels,
                                                         uint8_t* out) {
    __shared__ uint32_t lds_a[kBlock][8];
    __shared__ uint32_t lds_b[kBlock / 2][8];
    const uint64_t base = (uint64_t)blockIdx.x * kReduceTile;
    const uint32_t cnt = (uint32_t)((m - base) < kReduceTile ? (m - base) : kReduceTile);
    const uint32_t t = threadIdx.x;
    const uint32_t next = (cnt + 1) >> 1;
    if (t < next) {
        uint32_t L[8], R[8], o[8];
        const uint32_t ri = (2 * t + 1 < cnt) ? 2 * t + 1 : cnt - 1;
        load_digest(in + 32 * (base + 2 * t), L);
        load_digest(in + 32 * (base + ri), R);
        node_hash(L, R, o);
#pragma unroll
        for (int k = 0; k < 8; k++) lds_a[t][k] = o[k];
    }
    __syncthreads();
    uint32_t (*res)[8];
    const uint32_t out_cnt = lds_reduce(lds_a, lds_b, next, levels - 1, &res);
    if (t < out_cnt) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = res[t][k];
        store_digest(out + 32 * ((uint64_t)blockIdx.x * (kReduceTile >> levels) + t), v);
    }
}

// K3: one workgroup per object, objects of <= 512 leaves: full tree to the root (>= 1 level).
// leaf_first[o] .. leaf_first[o+1] index the object's leaf digests.
__global__ __launch_bounds__(kBlock) void batch_root_kernel(const uint8_t* leaves, const uint64_t* leaf_first,
                                                             const uint32_t* obj_ids, uint8_t* roots) {
    __shared__ uint32_t lds_a[kBlock][8];
    __shared__ uint32_t lds_b[kBlock / 2][8];
    const uint32_t o = obj_ids[blockIdx.x];
    const uint64_t base = leaf_first[o];
    const uint32_t cnt = (uint32_t)(leaf_first[o + 1] - base);
    const uint32_t t = threadIdx.x;
    const uint32_t next = (cnt + 1) >> 1;
    if (t < next) {
        uint32_t L[8], R[8], h[8];
        const uint32_t ri = (2 * t + 1 < cnt) ? 2 * t + 1 : cnt - 1;
        load_digest(leaves + 32 * (base + 2 * t), L);
        load_digest(leaves + 32 * (base + ri), R);
        node_hash(L, R, h);
#pragma unroll
        for (int k = 0; k < 8; k++) lds_a[t][k] = h[k];
    }
    __syncthreads();
    uint32_t levels = 0;
    for (uint32_t c = next; c > 1; c = (c + 1) >> 1) levels++;
    uint32_t (*res)[8];
    lds_reduce(lds_a, lds_b, next, levels, &res);
    if (t == 0) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = res[0][k];
        store_digest(roots + 32 * (uint64_t)o, v);
    }
}

// Synthetic object bytes: word[i] = splitmix64(seed ^ i) (same as oracle/merkle_oracle.c).
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void fill_splitmix_kernel(uint64_t* dst, uint64_t word0, uint64_t nwords,
                                                                uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * 2;
    for (uint64_t j = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 2; j < nwords; j += stride) {
        if (j + 1 < nwords) {
            ulonglong2 v = make_ulonglong2(splitmix64(seed ^ (word0 + j)), splitmix64(seed ^ (word0 + j + 1)));
            *reinterpret_cast<ulonglong2*>(dst + j) = v;
        } else {
            dst[j] = splitmix64(seed ^ (word0 + j));
        }
    }
}

// HBM read-bandwidth probe (the measured read peak bench.py reports next to the 8 TB/s spec,
// SURVEY.md 8d): XOR of every 8-byte word of [p, p + 16 * n16).  Each workgroup streams one
// contiguous slab with 16 nontemporal 16-byte loads in flight per lane.  Measured A/B over 8 GiB
// (tools/read_peak_ab.hip, profiles/r02/LOGS.md#r02o_read_ab2.log): grid-stride with 4 loads 5.3 TB/s,
// slabs 5.7, slabs with nontemporal loads 6.7 TB/s.  One global atomic XOR per workgroup; *out
// must be zero before the launch.
constexpr int kProbeLoads = 16;
__global__ __launch_bounds__(kBlock) void read_probe_kernel(const uint8_t* p, uint64_t n16, uint64_t* out) {
    const u32x4_t* g = reinterpret_cast<const u32x4_t*>(p);
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < n16 ? lo + per : n16;
    u32x4_t acc[kProbeLoads];
#pragma unroll
    for (int u = 0; u < kProbeLoads; u++) acc[u] = u32x4_t{0u, 0u, 0u, 0u};
    uint64_t i = lo + threadIdx.x;
    for (; i + (kProbeLoads - 1) * kBlock < hi; i += kProbeLoads * kBlock) {
        u32x4_t x[kProbeLoads];
#pragma unroll
        for (int u = 0; u < kProbeLoads; u++) x[u] = __builtin_nontemporal_load(g + i + u * kBlock);
#pragma unroll
        for (int u = 0; u < kProbeLoads; u++) acc[u] ^= x[u];
    }
    for (; i < hi; i += kBlock) acc[0] ^= g[i];
#pragma unroll
    for (int u = 1; u < kProbeLoads; u++) acc[0] ^= acc[u];
    uint64_t v = (((uint64_t)acc[0].y << 32) | acc[0].x) ^ (((uint64_t)acc[0].w << 32) | acc[0].z);
    for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
    __shared__ uint64_t part[kBlock / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kBlock / 64; w++) t ^= part[w];
        atomicXor(reinterpret_cast<unsigned long long*>(out), (unsigned long long)t);
    }
}

}  // namespace dm
