// tree_capi.inl -- Merkle tree levels and proofs (dm_tree_*, dm_merkle_paths*, dm_verify_paths*).
// Part of merkle_capi.hip (included at its end; shares dm_ctx, Dev and the helpers).
//
// merkletree v0.2.0 (go.mod:10; restated) builds Node objects for every level so that
//   GetMerklePath(content)  -> sibling digests + left/right indices up to the root,
//   VerifyContent(content)  -> recompute the content's leaf and its ancestors,
//   VerifyTree()            -> recompute every leaf from its content and the root
// work on the tree NewHashTree returns (common/hashtree/types.go:38).  DeOSS's fragment download
// path re-derives fragments and matches them by hash (node/fileHandler.go:962-1013); proofs let a
// caller check a fragment against a stored root instead.  Here the levels live in HBM
// (level-major, 32 B per node), paths are gathered and proofs folded on the GPU, one lane per proof.
#include "tree_kernels.hpp"

namespace {

uint64_t tree_nodes(uint64_t n) {
    if (n == 0) return 0;
    uint64_t total = 0, c = n;
    do {
        c = (c + 1) >> 1;
        total += c;
    } while (c > 1);
    return total;
}

uint32_t tree_depth(uint64_t n) { return n == 0 ? 0 : std::max<uint32_t>(1, ceil_log2(n)); }

// Levels 1 .. root of n leaf digests at `leaves` into `nodes` (level-major), one launch per level.
int tree_levels_dev(dm_ctx* c, hipStream_t s, const uint8_t* leaves, uint64_t n, uint8_t* nodes) {
    const uint8_t* in = leaves;
    uint64_t m = n, off = 0;
    const uint32_t D = tree_depth(n);
    for (uint32_t l = 0; l < D; l++) {
        uint8_t* out = nodes + 32 * off;
        hipLaunchKernelGGL(dm::reduce_kernel, dim3((uint32_t)ceil_div(m, dm::kReduceTile)), dim3(dm::kBlock), 0, s,
                           in, m, 1u, out);
        HIP_TRY(hipGetLastError());
        m = ceil_div(m, 2);
        off += m;
        in = out;
    }
    return DM_OK;
}

int paths_dev(dm_ctx* c, hipStream_t s, const uint8_t* leaves, const uint8_t* nodes, uint64_t n, const uint64_t* idx,
              uint64_t q, uint8_t* paths, uint8_t* bits) {
    if (q == 0) return DM_OK;
    hipLaunchKernelGGL(dm::paths_kernel, dim3((uint32_t)ceil_div(q, dm::kProofBlock)), dim3(dm::kProofBlock), 0, s,
                       leaves, nodes, n, idx, q, tree_depth(n), paths, bits);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

// Leaf digests of q device contents (table mode) into d.leaves, then the fold.
int verify_dev(dm_ctx* c, Dev& d, hipStream_t s, const void* const* contents, const uint64_t* lens, uint64_t q,
               const uint8_t* paths, const uint8_t* bits, uint32_t depth, const uint8_t* roots, uint64_t root_stride,
               uint8_t* ok) {
    std::vector<uint64_t> addr(q), len(q);
    bool aligned = true;
    for (uint64_t t = 0; t < q; t++) {
        addr[t] = reinterpret_cast<uint64_t>(contents[t]);
        len[t] = lens[t];
        aligned &= (addr[t] & 15) == 0;
    }
    RC_TRY(tables_begin(c, d, q * 16 + 1024));
    HIP_TRY(d.leaves.ensure(q * 32));
    RC_TRY(upload(c, d, s, d.tab_addr, addr.data(), q * 8));
    RC_TRY(upload(c, d, s, d.tab_len, len.data(), q * 8));
    dm::LeafArgs la{};
    la.addrs = static_cast<const uint64_t*>(d.tab_addr.p);
    la.lens = static_cast<const uint64_t*>(d.tab_len.p);
    la.nleaves = q;
    la.byte_end = ~0ull;
    la.digests = d.leaves.u8();
    RC_TRY(launch_leaves(c, d, s, la, true, aligned, pick_leaf_kernel(c, d, q)));
    hipLaunchKernelGGL(dm::verify_kernel, dim3((uint32_t)ceil_div(q, dm::kProofBlock)), dim3(dm::kProofBlock), 0, s,
                       d.leaves.u8(), paths, bits, depth, q, roots, root_stride, ok);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

// Uniform layout: the n chunks of one object (leaf i at dev + i * chunk, the last one short).
int verify_object_dev(dm_ctx* c, Dev& d, hipStream_t s, const void* dev, uint64_t len, uint64_t chunk,
                      const uint8_t* paths, const uint8_t* bits, uint32_t depth, const uint8_t* roots,
                      uint64_t root_stride, uint8_t* ok) {
    dm::LeafArgs la = uniform_args(dev, len, chunk);
    const uint64_t q = la.nleaves;
    HIP_TRY(d.leaves.ensure(q * 32));
    la.byte_end = ~0ull;
    la.digests = d.leaves.u8();
    const bool aligned = is_aligned16(dev) && chunk % 16 == 0;
    hipEvent_t* tr = timing_record(c, d);
    if (tr) HIP_TRY(hipEventRecord(tr[0], s));
    RC_TRY(launch_leaves(c, d, s, la, false, aligned, pick_leaf_kernel(c, d, q)));
    if (tr) HIP_TRY(hipEventRecord(tr[1], s));
    hipLaunchKernelGGL(dm::verify_kernel, dim3((uint32_t)ceil_div(q, dm::kProofBlock)), dim3(dm::kProofBlock), 0, s,
                       d.leaves.u8(), paths, bits, depth, q, roots, root_stride, ok);
    HIP_TRY(hipGetLastError());
    if (tr) HIP_TRY(hipEventRecord(tr[2], s));
    return DM_OK;
}

bool aligned_all(std::initializer_list<const void*> ps) {
    for (const void* p : ps)
        if (!p || !is_aligned16(p)) return false;
    return true;
}

}  // namespace

extern "C" {

uint64_t dm_tree_node_count(uint64_t n) { return tree_nodes(n); }

uint32_t dm_tree_depth(uint64_t n) { return tree_depth(n); }

int dm_tree_levels_device_async(dm_ctx* ctx, const void* dev_leaves, uint64_t n, void* dev_nodes, void* stream) {
    if (!ctx) return bad_arg();
    const int g = device_of(ctx, dev_nodes);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (n == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    if (!aligned_all({dev_leaves, dev_nodes}))
        return fail(c, DM_ERR_INVALID, "dm_tree_levels_device_async: need 16-byte aligned device buffers");
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    return tree_levels_dev(c, s, static_cast<const uint8_t*>(dev_leaves), n, static_cast<uint8_t*>(dev_nodes));
}

int dm_tree_levels(dm_ctx* ctx, const uint8_t* leaf_digests, uint64_t n, uint8_t* nodes_out) {
    if (!ctx || (n && (!leaf_digests || !nodes_out))) return bad_arg();
    const int g = pick_device(ctx);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (n == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    Dev& d = c->devs[g];
    hipStream_t s = d.stream;
    RC_TRY(begin_call(c, d, s));
    const uint64_t T = tree_nodes(n);
    HIP_TRY(d.leaves.ensure(n * 32));
    HIP_TRY(d.gather.ensure(T * 32));
    HIP_TRY(hipMemcpyAsync(d.leaves.p, leaf_digests, n * 32, hipMemcpyHostToDevice, s));
    RC_TRY(tree_levels_dev(c, s, d.leaves.u8(), n, d.gather.u8()));
    HIP_TRY(hipMemcpyAsync(nodes_out, d.gather.p, T * 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return DM_OK;
}

int dm_merkle_paths_device_async(dm_ctx* ctx, const void* dev_leaves, const void* dev_nodes, uint64_t n,
                                 const void* dev_idx, uint64_t q, void* dev_paths, void* dev_bits, void* stream) {
    if (!ctx) return bad_arg();
    const int g = device_of(ctx, dev_paths);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (n == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    if (q == 0) return DM_OK;
    if (!aligned_all({dev_leaves, dev_nodes, dev_paths}) || !dev_idx || !dev_bits ||
        (reinterpret_cast<uintptr_t>(dev_idx) & 7))
        return fail(c, DM_ERR_INVALID, "dm_merkle_paths_device_async: null or misaligned device buffer");
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    return paths_dev(c, s, static_cast<const uint8_t*>(dev_leaves), static_cast<const uint8_t*>(dev_nodes), n,
                     static_cast<const uint64_t*>(dev_idx), q, static_cast<uint8_t*>(dev_paths),
                     static_cast<uint8_t*>(dev_bits));
}

int dm_merkle_paths(dm_ctx* ctx, const uint8_t* leaf_digests, uint64_t n, const uint64_t* idx, uint64_t q,
                    uint8_t* paths, uint8_t* bits) {
    if (!ctx || (n && !leaf_digests) || (q && (!idx || !paths || !bits))) return bad_arg();
    const int g = pick_device(ctx);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (n == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    if (q == 0) return DM_OK;
    Dev& d = c->devs[g];
    hipStream_t s = d.stream;
    RC_TRY(begin_call(c, d, s));
    const uint64_t T = tree_nodes(n);
    const uint32_t D = tree_depth(n);
    HIP_TRY(d.leaves.ensure(n * 32));
    HIP_TRY(d.gather.ensure(T * 32));
    HIP_TRY(d.proof_paths.ensure(q * D * 32));
    HIP_TRY(d.proof_bits.ensure(q * D));
    HIP_TRY(d.proof_roots.ensure(q * 8));   // holds the leaf indices here
    HIP_TRY(hipMemcpyAsync(d.leaves.p, leaf_digests, n * 32, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.proof_roots.p, idx, q * 8, hipMemcpyHostToDevice, s));
    RC_TRY(tree_levels_dev(c, s, d.leaves.u8(), n, d.gather.u8()));
    RC_TRY(paths_dev(c, s, d.leaves.u8(), d.gather.u8(), n, static_cast<const uint64_t*>(d.proof_roots.p), q,
                     d.proof_paths.u8(), d.proof_bits.u8()));
    HIP_TRY(hipMemcpyAsync(paths, d.proof_paths.p, q * D * 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(bits, d.proof_bits.p, q * D, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return DM_OK;
}

int dm_verify_paths_device_async(dm_ctx* ctx, const void* const* dev_contents, const uint64_t* lens, uint64_t q,
                                 const void* dev_paths, const void* dev_bits, uint32_t depth, const void* dev_roots,
                                 uint64_t root_stride, void* dev_ok, void* stream) {
    if (!ctx) return bad_arg();
    const int g = device_of(ctx, dev_ok);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (q == 0) return DM_OK;
    if (!dev_contents || !lens || !dev_bits || !dev_ok || depth == 0 || !aligned_all({dev_paths, dev_roots}) ||
        root_stride % 16)
        return fail(c, DM_ERR_INVALID, "dm_verify_paths_device_async: null or misaligned argument, or depth 0");
    for (uint64_t t = 0; t < q; t++)
        if (lens[t] && !dev_contents[t])
            return fail(c, DM_ERR_INVALID, "content %llu: NULL pointer", (unsigned long long)t);
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    return verify_dev(c, d, s, dev_contents, lens, q, static_cast<const uint8_t*>(dev_paths),
                      static_cast<const uint8_t*>(dev_bits), depth, static_cast<const uint8_t*>(dev_roots),
                      root_stride, static_cast<uint8_t*>(dev_ok));
}

int dm_verify_object_device_async(dm_ctx* ctx, const void* dev_obj, uint64_t len, uint64_t chunk,
                                  const void* dev_paths, const void* dev_bits, uint32_t depth, const void* dev_roots,
                                  uint64_t root_stride, void* dev_ok, void* stream) {
    if (!ctx) return bad_arg();
    const int g = device_of(ctx, dev_obj);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (len == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    if (chunk == 0 || !dev_obj || !dev_bits || !dev_ok || depth == 0 || !aligned_all({dev_paths, dev_roots}) ||
        root_stride % 16)
        return fail(c, DM_ERR_INVALID, "dm_verify_object_device_async: null or misaligned argument, or depth 0");
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    return verify_object_dev(c, d, s, dev_obj, len, chunk, static_cast<const uint8_t*>(dev_paths),
                             static_cast<const uint8_t*>(dev_bits), depth, static_cast<const uint8_t*>(dev_roots),
                             root_stride, static_cast<uint8_t*>(dev_ok));
}

int dm_verify_paths(dm_ctx* ctx, const void* const* contents, const uint64_t* lens, uint64_t q, const uint8_t* paths,
                    const uint8_t* bits, uint32_t depth, const uint8_t* roots, uint64_t root_stride, uint8_t* ok) {
    if (!ctx || (q && (!contents || !lens || !paths || !bits || !roots || !ok)) || depth == 0 ||
        (root_stride != 0 && root_stride != 32))
        return bad_arg();
    const int g = pick_device(ctx);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (q == 0) return DM_OK;
    for (uint64_t t = 0; t < q; t++)
        if (lens[t] && !contents[t]) return fail(c, DM_ERR_INVALID, "content %llu: NULL pointer", (unsigned long long)t);
    Dev& d = c->devs[g];
    hipStream_t s = d.stream;
    RC_TRY(begin_call(c, d, s));
    std::vector<uint64_t> addr;
    RC_TRY(pack_chunks(c, d, contents, lens, q, addr));
    const uint64_t nroots = root_stride ? q : 1;
    HIP_TRY(d.proof_paths.ensure(q * depth * 32));
    HIP_TRY(d.proof_bits.ensure(q * depth + q));   // bits, then ok flags
    HIP_TRY(d.proof_roots.ensure(nroots * 32));
    HIP_TRY(hipMemcpyAsync(d.proof_paths.p, paths, q * depth * 32, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.proof_bits.p, bits, q * depth, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.proof_roots.p, roots, nroots * 32, hipMemcpyHostToDevice, s));
    std::vector<const void*> dptr(q);
    for (uint64_t t = 0; t < q; t++) dptr[t] = reinterpret_cast<const void*>(addr[t]);
    uint8_t* dok = d.proof_bits.u8() + q * depth;
    RC_TRY(verify_dev(c, d, s, dptr.data(), lens, q, d.proof_paths.u8(), d.proof_bits.u8(), depth,
                      d.proof_roots.u8(), root_stride ? 32 : 0, dok));
    HIP_TRY(hipMemcpyAsync(ok, dok, q, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return DM_OK;
}

}  // extern "C"
