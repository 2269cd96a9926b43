// fragment_capi.inl -- one fragment of a stored object, found by its name (dm_fragment_lookup,
// include/deoss_merkle.h).  Part of merkle_capi.hip (included after fullproc_capi.inl).
//
// DeOSS's fragment download handler (node/fileHandler.go:958-1013) serves ONE 8 MiB fragment of an
// object it holds locally: it runs FullProcessing(fpath, "", cacheDir) -- every 32 MiB segment
// hashed, every fragment coded, hashed and WRITTEN to cacheDir -- scans the names for the requested
// hash, streams that file and deletes cacheDir.  The answer needs only the fragment names, so this
// entry point computes exactly those: the file is read window by window into pinned memory
// (double-buffered: window w + 1 is read while the GPU codes and hashes window w), the segments are
// RS-coded on the device, every fragment is hashed (8 MiB chains, one table-mode leaf launch per
// window; no 32 MiB segment chains, no fid, no files), and the scan stops at the first window that
// holds the wanted name.  The matching fragment's bytes come back in `out`.
// Same fragments and names as dm_full_processing (oracle: oracle/process_oracle.c).

namespace {

constexpr uint64_t kFlWindowBytes = 1ull << 30;   // file bytes per GPU pass (hides the GPU under the reads)

}  // namespace

extern "C" {

int dm_fragment_lookup(dm_rs* r, const char* path, uint64_t segment, const uint8_t want[32], void* out,
                       uint64_t out_cap, int* found, uint64_t* seg_idx, int* frag_idx) {
    if (!r || !path || !want || !found) return bad_arg();
    *found = 0;
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    FileSet fs;
    RC_TRY(open_files(c, &path, 1, fs));   // "open <path>: ..." as os.Open would fail
    const uint64_t size = fs.size[0];
    if (size == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    RC_TRY(process_check(r, size, segment));
    const int k = r->k, m = r->m, total = k + m;
    const uint64_t frag = segment / (uint64_t)k, pbytes = (uint64_t)m * frag;
    if (out && out_cap < frag)
        return fail(c, DM_ERR_INVALID, "dm_fragment_lookup: out holds %llu bytes, a fragment is %llu",
                    (unsigned long long)out_cap, (unsigned long long)frag);
    const uint64_t nseg = ceil_div(size, segment);
    const uint64_t win = std::min(nseg, std::max<uint64_t>(1, env_bytes("DEOSS_FL_WINDOW_BYTES", kFlWindowBytes) / segment));
    const uint64_t nwin = ceil_div(nseg, win), per = win * (uint64_t)total;   // fragments per full window
    Dev& d = c->devs[g];
    RsLane& L = rs_ln(r, d);
    hipStream_t s = d.stream;
    RC_TRY(begin_call(c, d, s));
    struct SyncOnExit {   // on every return: nothing queued outlives the call (the pinned slots are reused)
        hipStream_t s;
        ~SyncOnExit() { (void)hipStreamSynchronize(s); }
    } sync_on_exit{s};
    // two of everything: pinned window slots, device segments, parity and digests (window w uses w % 2)
    HIP_TRY(pinned_grow(c, d.id, L.fp_slot[0], win * segment));
    HIP_TRY(pinned_grow(c, d.id, L.fp_slot[1], win * segment));
    HIP_TRY(pinned_grow(c, d.id, L.fp_slot[2], 2 * per * 32));
    HIP_TRY(d.data.ensure(2 * win * segment));
    HIP_TRY(L.work.ensure(2 * win * pbytes));
    HIP_TRY(d.leaves.ensure(2 * per * 32));
    uint8_t* data[2] = {d.data.u8(), d.data.u8() + win * segment};
    uint8_t* par[2] = {L.work.u8(), L.work.u8() + win * pbytes};
    uint8_t* hdig = L.fp_slot[2].u8();
    // one leaf table for both halves: fragment j of segment t of half b (data fragments are
    // segment slices, parity fragments live in the parity half)
    std::vector<uint64_t> addr(2 * per), lens(2 * per, frag);
    for (int b = 0; b < 2; b++)
        for (uint64_t t = 0; t < win; t++)
            for (int j = 0; j < total; j++)
                addr[b * per + t * total + j] = reinterpret_cast<uint64_t>(
                    j < k ? data[b] + t * segment + (uint64_t)j * frag : par[b] + t * pbytes + (uint64_t)(j - k) * frag);
    RC_TRY(tables_begin(c, d, 2 * per * 16 + 1024));
    RC_TRY(upload(c, d, s, d.tab_addr, addr.data(), addr.size() * 8));
    RC_TRY(upload(c, d, s, d.tab_len, lens.data(), lens.size() * 8));
    const int readers = (int)std::min<uint64_t>(64, env_bytes("DEOSS_FP_READERS", kFpReaders));
    // window w's names (in segment, fragment order) against `want`: 1 found (its bytes copied to
    // out), 0 not in this window, -1 the copy failed
    auto scan = [&](uint64_t w) -> int {
        const uint64_t ns = std::min(win, nseg - w * win);
        const uint8_t* dg = hdig + (w % 2) * per * 32;
        for (uint64_t i = 0; i < ns * (uint64_t)total; i++) {
            if (std::memcmp(dg + 32 * i, want, 32) != 0) continue;
            const uint64_t t = i / (uint64_t)total;
            const int j = (int)(i % (uint64_t)total);
            *found = 1;
            if (seg_idx) *seg_idx = w * win + t;
            if (frag_idx) *frag_idx = j;
            const uint8_t* src = j < k ? data[w % 2] + t * segment + (uint64_t)j * frag
                                       : par[w % 2] + t * pbytes + (uint64_t)(j - k) * frag;
            if (!out) return 1;
            const bool ok = hipMemcpyAsync(out, src, frag, hipMemcpyDeviceToHost, s) == hipSuccess &&
                            hipStreamSynchronize(s) == hipSuccess;
            return ok ? 1 : -1;
        }
        return 0;
    };
    hipEvent_t ev_dig[2] = {d.ev_step[0], d.ev_step[1]};
    int rc = DM_OK;
    for (uint64_t w = 0; w < nwin && rc == DM_OK; w++) {
        const int b = (int)(w % 2);
        const uint64_t s0 = w * win, ns = std::min(win, nseg - s0);
        // host: read window w into slot b while the GPU runs window w - 1 (slot b's last H2D, from
        // window w - 2, finished before window w - 1's digests were scanned)
        uint8_t* slot = L.fp_slot[b].u8();
        std::vector<FilePart> parts;
        for (uint64_t t = 0; t < ns; t++) {
            const uint64_t off = (s0 + t) * segment, have = std::min(segment, size - off);
            parts.push_back({0, off, have, slot + t * segment});
            if (have < segment) std::memset(slot + t * segment + have, 0, segment - have);   // zero padding
        }
        if ((rc = read_parts(c, fs, parts, readers)) != DM_OK) break;
        if (w > 0) {   // window w - 1's names first: stop before launching w when it holds the fragment
            if (hipEventSynchronize(ev_dig[(w - 1) % 2]) != hipSuccess) {
                rc = fail(c, DM_ERR_HIP, "dm_fragment_lookup: window %llu", (unsigned long long)(w - 1));
                break;
            }
            const int hit = scan(w - 1);
            if (hit < 0) rc = fail(c, DM_ERR_HIP, "dm_fragment_lookup: fragment copy");
            if (hit != 0) break;
        }
        HIP_TRY(hipMemcpyAsync(data[b], slot, ns * segment, hipMemcpyHostToDevice, s));
        dm::RsArgs a{};
        for (int j = 0; j < k; j++) a.in[j] = data[b] + (uint64_t)j * frag;
        for (int i = 0; i < m; i++) a.out[i] = par[b] + (uint64_t)i * frag;
        a.in_seg_stride = segment;
        a.out_seg_stride = pbytes;
        a.units_per_seg = frag / 16;
        a.nseg = ns;
        a.table = static_cast<const uint2*>(r->enc_tab.p);
        a.nout = (uint32_t)m;
        launch_rs(d, s, k, a);
        HIP_TRY(hipGetLastError());
        dm::LeafArgs la{};
        la.addrs = static_cast<const uint64_t*>(d.tab_addr.p) + b * per;
        la.lens = static_cast<const uint64_t*>(d.tab_len.p) + b * per;
        la.nleaves = ns * (uint64_t)total;
        la.byte_end = ~0ull;
        la.digests = d.leaves.u8() + b * per * 32;
        RC_TRY(launch_leaves(c, d, s, la, true, true, pick_leaf_kernel(c, d, la.nleaves)));
        HIP_TRY(hipMemcpyAsync(hdig + b * per * 32, la.digests, la.nleaves * 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipEventRecord(ev_dig[b], s));
        if (w + 1 == nwin) {   // the last window: nothing left to read, wait for its names
            HIP_TRY(hipEventSynchronize(ev_dig[b]));
            if (scan(w) < 0) rc = fail(c, DM_ERR_HIP, "dm_fragment_lookup: fragment copy");
        }
    }
    if (hipStreamSynchronize(s) != hipSuccess && rc == DM_OK) rc = fail(c, DM_ERR_HIP, "dm_fragment_lookup: sync");
    return rc;
}

}  // extern "C"
