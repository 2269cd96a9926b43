// process_capi.inl -- FullProcessing on the GPU (dm_process_*, include/deoss_merkle.h).
// Part of merkle_capi.hip (included after rs_capi.inl; shares dm_ctx, Dev, dm_rs and the helpers).
//
// Replaces cess-go-sdk process.FullProcessing(file, cipher = "", savedir) (go.mod:8), which every
// upload handler runs to get the fid and the fragment names (node/objectHandler.go:168,
// node/fileHandler.go:771, node/filesHandler.go:201, node/resumeHandler.go:326,
// node/tracker.go:767-769) and the fragment download path re-runs (node/fileHandler.go:964,997).
// One call, all on the device:
//   1. zero the last segment's padding in place (hipMemsetAsync);
//   2. rs_code_kernel codes every segment into its parity fragments (one launch, all segments);
//   3. ONE table-mode leaf-kernel launch hashes the nseg segments (32 MiB leaves, listed first so
//      they start first) and the nseg x (data + parity) fragments (8 MiB leaves) together: the
//      segment chains set the time, the fragment chains run beside them on otherwise idle SIMDs;
//   4. the segment digests reduce to the fid (K2 / finish).
// Oracle: oracle/process_oracle.c (restated composition; parity of the composition unpinned).

namespace {

// nseg segments at `obj` (segment-contiguous, padding already zeroed) belonging to objects whose
// segments start at first[o] (first.size() == nobj + 1): RS coding, one leaf launch over every
// segment and fragment, one fid per object into fids (nobj x 32, device).  Digests land in
// d.leaves: segment s at s, fragment (s, j) at nseg + s * total + j.  after_rs (nullable) is
// recorded once the parity is written, so a caller can copy it out while the leaf kernel runs.
int process_segments(dm_rs* r, Dev& d, hipStream_t s, uint8_t* obj, uint64_t segment, uint8_t* parity,
                     const std::vector<uint64_t>& first, uint8_t* fids, hipEvent_t after_rs = nullptr) {
    dm_ctx* c = r->c;
    const int k = r->k, m = r->m, total = k + m;
    const uint64_t nseg = first.back(), frag = segment / (uint64_t)k, nobj = first.size() - 1;
    dm::RsArgs a{};
    for (int j = 0; j < k; j++) a.in[j] = obj + (uint64_t)j * frag;
    for (int i = 0; i < m; i++) a.out[i] = parity + (uint64_t)i * frag;
    a.in_seg_stride = segment;
    a.out_seg_stride = (uint64_t)m * frag;
    a.units_per_seg = frag / 16;
    a.nseg = nseg;
    a.table = static_cast<const uint2*>(r->enc_tab.p);
    a.nout = (uint32_t)m;
    launch_rs(d, s, k, a);
    HIP_TRY(hipGetLastError());
    if (after_rs) HIP_TRY(hipEventRecord(after_rs, s));
    // leaf table: segments first (their chains are the longest: they start first), then fragments
    const uint64_t T = nseg * (1 + (uint64_t)total);
    std::vector<uint64_t> addr(T), lens(T);
    for (uint64_t i = 0; i < nseg; i++) {
        addr[i] = reinterpret_cast<uint64_t>(obj + i * segment);
        lens[i] = segment;
    }
    for (uint64_t i = 0; i < nseg; i++)
        for (int j = 0; j < total; j++) {
            const uint64_t t = nseg + i * total + j;
            addr[t] = reinterpret_cast<uint64_t>(j < k ? obj + i * segment + (uint64_t)j * frag
                                                       : parity + (i * m + (j - k)) * frag);
            lens[t] = frag;
        }
    RC_TRY(tables_begin(c, d, T * 16 + (nobj + 1) * 12 + 2048));
    HIP_TRY(d.leaves.ensure(T * 32));
    RC_TRY(upload(c, d, s, d.tab_addr, addr.data(), T * 8));
    RC_TRY(upload(c, d, s, d.tab_len, lens.data(), T * 8));
    dm::LeafArgs la{};
    la.addrs = static_cast<const uint64_t*>(d.tab_addr.p);
    la.lens = static_cast<const uint64_t*>(d.tab_len.p);
    la.nleaves = T;
    la.byte_end = ~0ull;
    la.digests = d.leaves.u8();
    hipEvent_t* tr = timing_record(c, d);
    if (tr) HIP_TRY(hipEventRecord(tr[0], s));
    RC_TRY(launch_leaves(c, d, s, la, true, true, pick_leaf_kernel(c, d, T)));
    if (tr) HIP_TRY(hipEventRecord(tr[1], s));
    if (nobj == 1) RC_TRY(finish(c, d, s, d.leaves.u8(), nseg, true, fids));
    else RC_TRY(batch_roots_from_leaves(c, d, s, d.leaves.u8(), first, fids));
    if (tr) HIP_TRY(hipEventRecord(tr[2], s));
    return DM_OK;
}

int process_dev(dm_rs* r, Dev& d, hipStream_t s, uint8_t* obj, uint64_t len, uint64_t segment, uint8_t* parity,
                uint8_t* seg_hashes, uint8_t* frag_hashes, uint8_t* fid) {
    dm_ctx* c = r->c;
    const int total = r->k + r->m;
    const uint64_t nseg = ceil_div(len, segment);
    RC_TRY(begin_call(c, d, s));
    if (nseg * segment > len) HIP_TRY(hipMemsetAsync(obj + len, 0, nseg * segment - len, s));
    RC_TRY(process_segments(r, d, s, obj, segment, parity, {0, nseg}, fid));
    if (seg_hashes) HIP_TRY(hipMemcpyAsync(seg_hashes, d.leaves.p, nseg * 32, hipMemcpyDeviceToDevice, s));
    if (frag_hashes)
        HIP_TRY(hipMemcpyAsync(frag_hashes, d.leaves.u8() + nseg * 32, nseg * total * 32, hipMemcpyDeviceToDevice, s));
    return DM_OK;
}

// Host objects -> device (segment-aligned, zero-padded) -> process_segments -> host outputs.
// Per-object outputs are nullable (frags_out / seg_hashes / frag_hashes may be NULL arrays or hold
// NULL entries); fids (nobj x 32) is required.  Runs on d.stream, synchronous.
int process_host(dm_rs* r, Dev& d, const void* const* objs, const uint64_t* lens, uint64_t nobj, uint64_t segment,
                 void* const* frags_out, uint8_t* const* seg_hashes, uint8_t* const* frag_hashes, uint8_t* fids) {
    dm_ctx* c = r->c;
    hipStream_t s = d.stream;
    RC_TRY(begin_call(c, d, s));
    const int k = r->k, m = r->m, total = k + m;
    const uint64_t frag = segment / (uint64_t)k;
    std::vector<uint64_t> first(nobj + 1, 0), off(nobj);
    for (uint64_t o = 0; o < nobj; o++) {
        first[o + 1] = first[o] + ceil_div(lens[o], segment);
        off[o] = first[o] * segment;
    }
    const uint64_t S = first[nobj];
    HIP_TRY(d.data.ensure(S * segment + kAlign));
    RC_TRY(h2d_at(c, d, objs, lens, nobj, off));
    for (uint64_t o = 0; o < nobj; o++) {
        const uint64_t pad = (first[o + 1] - first[o]) * segment - lens[o];
        if (pad) HIP_TRY(hipMemsetAsync(d.data.u8() + off[o] + lens[o], 0, pad, s));
    }
    DevBuf& work = rs_ln(r, d).work;
    HIP_TRY(work.ensure(S * (uint64_t)m * frag + nobj * 32));
    uint8_t* parity = work.u8();
    uint8_t* dfid = parity + S * (uint64_t)m * frag;
    RC_TRY(process_segments(r, d, s, d.data.u8(), segment, parity, first, dfid));
    HIP_TRY(hipMemcpyAsync(fids, dfid, nobj * 32, hipMemcpyDeviceToHost, s));
    for (uint64_t o = 0; o < nobj; o++) {
        const uint64_t f0 = first[o], ns = first[o + 1] - first[o];
        if (seg_hashes && seg_hashes[o])
            HIP_TRY(hipMemcpyAsync(seg_hashes[o], d.leaves.u8() + f0 * 32, ns * 32, hipMemcpyDeviceToHost, s));
        if (frag_hashes && frag_hashes[o])
            HIP_TRY(hipMemcpyAsync(frag_hashes[o], d.leaves.u8() + (S + f0 * total) * 32, ns * total * 32,
                                   hipMemcpyDeviceToHost, s));
        if (frags_out && frags_out[o]) {
            uint8_t* out = static_cast<uint8_t*>(frags_out[o]);
            for (uint64_t i = 0; i < ns; i++) {
                HIP_TRY(hipMemcpyAsync(out + i * total * frag, d.data.u8() + (f0 + i) * segment, segment,
                                       hipMemcpyDeviceToHost, s));
                HIP_TRY(hipMemcpyAsync(out + i * total * frag + segment, parity + (f0 + i) * m * frag, m * frag,
                                       hipMemcpyDeviceToHost, s));
            }
        }
    }
    HIP_TRY(hipStreamSynchronize(s));
    return DM_OK;
}

int process_check(dm_rs* r, uint64_t len, uint64_t segment) {
    dm_ctx* c = r->c;
    if (len == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    if (segment == 0 || segment % (16ull * (uint64_t)r->k))
        return fail(c, DM_ERR_INVALID, "segment size %llu must be a non-zero multiple of 16 x %d data shards",
                    (unsigned long long)segment, r->k);
    return DM_OK;
}

}  // namespace

extern "C" {

int dm_process_device_async(dm_rs* r, void* dev_obj, uint64_t len, uint64_t segment, void* dev_parity,
                            void* dev_seg_hashes, void* dev_frag_hashes, void* dev_fid, void* stream) {
    if (!r) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    RC_TRY(process_check(r, len, segment));
    if (!dev_obj || !dev_parity || !dev_fid || !is_aligned16(dev_obj) || !is_aligned16(dev_parity))
        return fail(c, DM_ERR_INVALID, "dm_process_device_async: need 16-byte aligned object and parity buffers");
    Dev& d = c->devs[g];
    return process_dev(r, d, pick_stream(d, stream), static_cast<uint8_t*>(dev_obj), len, segment,
                       static_cast<uint8_t*>(dev_parity), static_cast<uint8_t*>(dev_seg_hashes),
                       static_cast<uint8_t*>(dev_frag_hashes), static_cast<uint8_t*>(dev_fid));
}

int dm_process_buffer(dm_rs* r, const void* host, uint64_t len, uint64_t segment, void* frags_out,
                      uint8_t* seg_hashes, uint8_t* frag_hashes, uint8_t fid[32]) {
    if (!r) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    if (!fid || (!host && len)) return fail(c, DM_ERR_INVALID, "dm_process_buffer: null argument");
    RC_TRY(process_check(r, len, segment));
    return process_host(r, c->devs[g], &host, &len, 1, segment, &frags_out, &seg_hashes, &frag_hashes, fid);
}

int dm_process_batch(dm_rs* r, const void* const* objs, const uint64_t* lens, uint64_t nobj, uint64_t segment,
                     void* const* frags_out, uint8_t* const* seg_hashes, uint8_t* const* frag_hashes, uint8_t* fids) {
    if (!r) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    if (nobj == 0) return DM_OK;
    if (!objs || !lens || !fids) return fail(c, DM_ERR_INVALID, "dm_process_batch: null argument");
    for (uint64_t o = 0; o < nobj; o++) {
        if (lens[o] == 0) return fail(c, DM_ERR_EMPTY, "Empty data (object %llu has no bytes)", (unsigned long long)o);
        if (!objs[o]) return fail(c, DM_ERR_INVALID, "object %llu: NULL pointer", (unsigned long long)o);
    }
    RC_TRY(process_check(r, lens[0], segment));
    return process_host(r, c->devs[g], objs, lens, nobj, segment, frags_out, seg_hashes, frag_hashes, fids);
}

}  // extern "C"
