// sha256_gfx950.hpp -- SHA-256 compression for CDNA4 (gfx950), one message per lane.
//
// Replaces the arithmetic of Go crypto/sha256 as used by DeOSS common/hashtree
// (reference: common/hashtree/hashtree.go:23-30 leaf hash; merkletree v0.2.0 node hash
// SHA-256(left||right), called from common/hashtree/types.go:38).
//
// Instruction mapping (checked in the ISA dump, see DESIGN.md "K1"):
//   rotr           -> v_alignbit_b32 x, x, n
//   x^y^z          -> v_bitop3_b32 ... bitop3:0x96
//   Ch(e,f,g)      -> v_bitop3_b32 ... bitop3:0xca
//   Maj(a,b,c)     -> v_bitop3_b32 ... bitop3:0xe8
//   a+b+c          -> v_add3_u32
//   byte swap      -> v_perm_b32
// Per 64-byte block: 64 rounds x 14 VALU + 48 schedule steps x 10 VALU + 8 state adds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dm {

__device__ __constant__ static const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

// Host-and-device constexpr copy, used to fold constant message schedules at compile time.
struct Sha256Consts {
    uint32_t k[64];
};
constexpr Sha256Consts kK = {{
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2}};

constexpr uint32_t kIV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                             0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

constexpr uint32_t c_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// K[t] + W[t] for the constant second block of every 64-byte (node) message:
// W = 0x80000000, 0 x 14, 512 (bit length).  Folded at compile time.
struct PadKW {
    uint32_t kw[64];
};
constexpr PadKW make_pad64_kw() {
    PadKW r{};
    uint32_t w[64] = {};
    w[0] = 0x80000000u;
    w[15] = 512u;
    for (int t = 16; t < 64; t++) {
        uint32_t s0 = c_rotr(w[t - 15], 7) ^ c_rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = c_rotr(w[t - 2], 17) ^ c_rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    for (int t = 0; t < 64; t++) r.kw[t] = kK.k[t] + w[t];
    return r;
}
constexpr PadKW kPad64KW = make_pad64_kw();

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xca);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xe8);
}
__device__ __forceinline__ uint32_t bsig0(uint32_t x) { return xor3(rotr(x, 2), rotr(x, 13), rotr(x, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t x) { return xor3(rotr(x, 6), rotr(x, 11), rotr(x, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }

// One round with the state kept as named registers rotated by the macro call order.
#define DM_SHA_ROUND(a, b, c, d, e, f, g, h, kw)                  \
    do {                                                          \
        uint32_t t1_ = h + bsig1(e) + ch(e, f, g) + (kw);         \
        uint32_t t2_ = bsig0(a) + maj(a, b, c);                   \
        d += t1_;                                                 \
        h = t1_ + t2_;                                            \
    } while (0)

// Eight rounds starting at round index T; KW(t) yields K[t] + W[t].
#define DM_SHA_8ROUNDS(T, KW)                                     \
    DM_SHA_ROUND(a, b, c, d, e, f, g, h, KW((T) + 0));            \
    DM_SHA_ROUND(h, a, b, c, d, e, f, g, KW((T) + 1));            \
    DM_SHA_ROUND(g, h, a, b, c, d, e, f, KW((T) + 2));            \
    DM_SHA_ROUND(f, g, h, a, b, c, d, e, KW((T) + 3));            \
    DM_SHA_ROUND(e, f, g, h, a, b, c, d, KW((T) + 4));            \
    DM_SHA_ROUND(d, e, f, g, h, a, b, c, KW((T) + 5));            \
    DM_SHA_ROUND(c, d, e, f, g, h, a, b, KW((T) + 6));            \
    DM_SHA_ROUND(b, c, d, e, f, g, h, a, KW((T) + 7))

// Compress one 64-byte block given as 16 big-endian-decoded words (w is clobbered).
__device__ __forceinline__ void compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#define DM_KW_MSG(t) (kSha256K[(t)] + dm_wt_((t)))
    // message word for round t (rolling 16-word window, computed in round order)
    auto dm_wt_ = [&](int t) __attribute__((always_inline)) -> uint32_t {
        if (t < 16) return w[t];
        uint32_t v = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
        w[t & 15] = v;
        return v;
    };
    DM_SHA_8ROUNDS(0, DM_KW_MSG);
    DM_SHA_8ROUNDS(8, DM_KW_MSG);
    DM_SHA_8ROUNDS(16, DM_KW_MSG);
    DM_SHA_8ROUNDS(24, DM_KW_MSG);
    DM_SHA_8ROUNDS(32, DM_KW_MSG);
    DM_SHA_8ROUNDS(40, DM_KW_MSG);
    DM_SHA_8ROUNDS(48, DM_KW_MSG);
    DM_SHA_8ROUNDS(56, DM_KW_MSG);
#undef DM_KW_MSG
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Compress the constant padding block of a 64-byte message (second block of every node hash):
// no message schedule at run time, K+W folded into literals.
__device__ __forceinline__ void compress_pad64(uint32_t (&st)[8]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#define DM_KW_PAD(t) (kPad64KW.kw[(t)])
    DM_SHA_8ROUNDS(0, DM_KW_PAD);
    DM_SHA_8ROUNDS(8, DM_KW_PAD);
    DM_SHA_8ROUNDS(16, DM_KW_PAD);
    DM_SHA_8ROUNDS(24, DM_KW_PAD);
    DM_SHA_8ROUNDS(32, DM_KW_PAD);
    DM_SHA_8ROUNDS(40, DM_KW_PAD);
    DM_SHA_8ROUNDS(48, DM_KW_PAD);
    DM_SHA_8ROUNDS(56, DM_KW_PAD);
#undef DM_KW_PAD
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__device__ __forceinline__ void init_state(uint32_t (&st)[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kIV[i];
}

// Merkle node: SHA-256(left || right) with left/right given as digest words (state form).
__device__ __forceinline__ void node_hash(const uint32_t (&l)[8], const uint32_t (&r)[8], uint32_t (&out)[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
    init_state(out);
    compress(out, w);
    compress_pad64(out);
}

}  // namespace dm
