// tree_kernels.hpp -- Merkle proof kernels for gfx950 (dm_merkle_paths_*, dm_verify_paths_*).
//
// merkletree v0.2.0 (go.mod:10, restated) keeps every node so GetMerklePath,
// VerifyContent and VerifyTree can walk the tree.  The GPU keeps the same nodes level-major:
// level 1 (ceil(n/2) nodes) .. the root, 32 B each, beside the n leaf digests (level 0).
// Both kernels are one lane per proof: a proof is `depth` dependent steps (gathers, or 2-block
// node hashes) and proofs are independent, so lanes = proofs fills the chip for large batches.
#pragma once

#include "merkle_kernels.hpp"

namespace dm {

constexpr int kProofBlock = 256;

__device__ __forceinline__ bool digest_eq(const uint8_t* a, const uint8_t* b) {
    const uint4* x = reinterpret_cast<const uint4*>(a);
    const uint4* y = reinterpret_cast<const uint4*>(b);
    const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
    return ((x0.x ^ y0.x) | (x0.y ^ y0.y) | (x0.z ^ y0.z) | (x0.w ^ y0.w) | (x1.x ^ y1.x) | (x1.y ^ y1.y) |
            (x1.z ^ y1.z) | (x1.w ^ y1.w)) == 0;
}

__device__ __forceinline__ void copy_digest(uint8_t* dst, const uint8_t* src) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    d[0] = s[0];
    d[1] = s[1];
}

// GetMerklePath for leaf idx[t]: at each level the parent of position p pairs (2j, min(2j+1, c-1));
// like merkletree's `bytes.Equal(currentParent.Left.Hash, current.Hash)`, the sibling is the RIGHT
// child (bit 1) whenever the left child's digest equals the current node's, else the left (bit 0).
// Out-of-range indices get an all-zero path and bits 0xff.
__global__ __launch_bounds__(kProofBlock) void paths_kernel(const uint8_t* leaves, const uint8_t* nodes, uint64_t n,
                                                            const uint64_t* idx, uint64_t q, uint32_t depth,
                                                            uint8_t* paths, uint8_t* bits) {
    const uint64_t t = (uint64_t)blockIdx.x * kProofBlock + threadIdx.x;
    if (t >= q) return;
    uint64_t p = idx[t];
    uint8_t* path = paths + 32 * depth * t;
    uint8_t* bt = bits + (uint64_t)depth * t;
    if (p >= n) {
        for (uint32_t l = 0; l < depth; l++) {
            reinterpret_cast<uint4*>(path + 32 * l)[0] = make_uint4(0, 0, 0, 0);
            reinterpret_cast<uint4*>(path + 32 * l)[1] = make_uint4(0, 0, 0, 0);
            bt[l] = 0xff;
        }
        return;
    }
    uint64_t c = n;
    const uint8_t* lev = leaves;
    uint64_t off = 0;   // offset (nodes) of the next level in `nodes`
    for (uint32_t l = 0; l < depth; l++) {
        const uint64_t j = p >> 1, li = 2 * j, ri = (2 * j + 1 < c) ? 2 * j + 1 : c - 1;
        const uint8_t* cur = lev + 32 * p;
        const uint8_t* left = lev + 32 * li;
        if (digest_eq(left, cur)) {
            copy_digest(path + 32 * l, lev + 32 * ri);
            bt[l] = 1;
        } else {
            copy_digest(path + 32 * l, left);
            bt[l] = 0;
        }
        lev = nodes + 32 * off;
        c = (c + 1) >> 1;
        off += c;
        p = j;
    }
}

// Fold q proofs: h = leaf digest; per level h = H(h || sib) (bit 1) or H(sib || h) (bit 0);
// ok[t] = (h == root of proof t).  roots advance by root_stride bytes per proof (0: one root).
__global__ __launch_bounds__(kProofBlock) void verify_kernel(const uint8_t* digests, const uint8_t* paths,
                                                             const uint8_t* bits, uint32_t depth, uint64_t q,
                                                             const uint8_t* roots, uint64_t root_stride,
                                                             uint8_t* ok) {
    const uint64_t t = (uint64_t)blockIdx.x * kProofBlock + threadIdx.x;
    if (t >= q) return;
    uint32_t h[8];
    load_digest(digests + 32 * t, h);
    const uint8_t* path = paths + 32 * depth * t;
    const uint8_t* bt = bits + (uint64_t)depth * t;
    bool good = true;
    for (uint32_t l = 0; l < depth; l++) {
        uint32_t s[8], L[8], R[8];
        load_digest(path + 32 * l, s);
        const uint8_t b = bt[l];
        good &= b <= 1;
#pragma unroll
        for (int k = 0; k < 8; k++) {   // operand select, one node hash per level (no divergence)
            L[k] = b == 1 ? h[k] : s[k];
            R[k] = b == 1 ? s[k] : h[k];
        }
        node_hash(L, R, h);
    }
    uint32_t r[8];
    load_digest(roots + root_stride * t, r);
    uint32_t diff = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) diff |= h[k] ^ r[k];
    ok[t] = (uint8_t)(good && diff == 0);
}

}  // namespace dm
