// fragment_capi.inl -- one fragment of a stored object, found by its name (dm_fragment_lookup,
// include/deoss_merkle.h).  Part of merkle_capi.hip (included after fullproc_capi.inl).
//
// DeOSS's fragment download handler (node/fileHandler.go:958-1013) serves ONE 8 MiB fragment of an
// object it holds locally: it runs FullProcessing(fpath, "", cacheDir) -- every 32 MiB segment
// hashed, every fragment coded, hashed and WRITTEN to cacheDir -- scans the names for the requested
// hash, streams that file and deletes cacheDir.  The answer needs only the fragment names, so this
// entry point computes exactly those.  The file is read in pieces into the rs lane's small pinned
// slots (the FullProcessing slots, 64 MiB) and copied on the lane's copy stream into a device ring
// of two windows; each window (>= 1 GiB, so that few windows pay the 8 MiB fragment chain) gets one
// RS launch and one table-mode leaf launch over its fragments on the lane's compute stream (no
// 32 MiB segment chains, no fid, no files) while the next window is read; the names come back and
// are scanned in window order, and the call stops at the first window holding the wanted one.
// The matching fragment's bytes come back in `out`.  Same fragments and names as
// dm_full_processing (oracle: oracle/process_oracle.c).

namespace {

constexpr uint64_t kFlWindowBytes = 1ull << 30;      // smallest window (file bytes per leaf launch)
constexpr uint64_t kFlWindowMaxBytes = 4ull << 30;   // largest window (2 in HBM + 2x parity: 24 GiB)
constexpr int kFlSlots = 3;                          // pinned read slots (of dm_rs's 4; the 4th holds names)
constexpr uint64_t kFlPartBytes = 8ull << 20;        // pread size (one reader thread each)

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
    // window: a quarter of the file, within [kFlWindowBytes, kFlWindowMaxBytes] (test hook:
    // DEOSS_FL_WINDOW_BYTES fixes it); slot: the FullProcessing slot size, at least one segment
    const uint64_t want_win = std::getenv("DEOSS_FL_WINDOW_BYTES")
                                  ? env_bytes("DEOSS_FL_WINDOW_BYTES", kFlWindowBytes)
                                  : std::min(kFlWindowMaxBytes, std::max(kFlWindowBytes, size / 4));
    const uint64_t win = std::min(nseg, std::max<uint64_t>(1, want_win / segment));
    const uint64_t spd = std::min(win, std::max<uint64_t>(1, env_bytes("DEOSS_FP_SLOT_BYTES", kFpSlotBytes) / segment));
    const uint64_t nwin = ceil_div(nseg, win), per = win * (uint64_t)total;   // fragments per full window
    Dev& d = c->devs[g];
    RsLane& L = rs_ln(r, d);
    hipStream_t s = d.stream, cp = d.copy;
    RC_TRY(begin_call(c, d, s));
    // events: pinned slot free again, window copied, window hashed (created per call)
    struct Events {
        hipEvent_t slot[kFlSlots] = {}, copied[2] = {}, hashed[2] = {};
        ~Events() {
            for (hipEvent_t e : slot) if (e) (void)hipEventDestroy(e);
            for (int i = 0; i < 2; i++) {
                if (copied[i]) (void)hipEventDestroy(copied[i]);
                if (hashed[i]) (void)hipEventDestroy(hashed[i]);
            }
        }
    } ev;
    struct SyncOnExit {   // on every return: nothing queued outlives the call (slots and buffers are reused)
        hipStream_t a, b;
        ~SyncOnExit() {
            (void)hipStreamSynchronize(a);
            (void)hipStreamSynchronize(b);
        }
    } sync_on_exit{s, cp};
    for (hipEvent_t& e : ev.slot) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int i = 0; i < 2; i++) {
        HIP_TRY(hipEventCreateWithFlags(&ev.copied[i], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&ev.hashed[i], hipEventDisableTiming));
    }
    for (int i = 0; i < kFlSlots; i++) HIP_TRY(pinned_grow(c, d.id, L.fp_slot[i], spd * segment));
    HIP_TRY(pinned_grow(c, d.id, L.fp_slot[kFlSlots], 2 * per * 32));
    HIP_TRY(d.data.ensure(2 * win * segment));
    HIP_TRY(L.work.ensure(2 * win * pbytes));
    HIP_TRY(d.leaves.ensure(2 * per * 32));
    uint8_t* data[2] = {d.data.u8(), d.data.u8() + win * segment};
    uint8_t* par[2] = {L.work.u8(), L.work.u8() + win * pbytes};
    uint8_t* hdig = L.fp_slot[kFlSlots].u8();
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
    // out), 0 not in this window, -1 the copy failed.  Window w's half is neither re-filled nor its
    // names overwritten before w is scanned (window w + 1 is launched, and w + 2 read, after that).
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
            // on the copy stream: the compute stream may already hold the next window's chains
            const bool ok = hipMemcpyAsync(out, src, frag, hipMemcpyDeviceToHost, cp) == hipSuccess &&
                            hipStreamSynchronize(cp) == hipSuccess;
            return ok ? 1 : -1;
        }
        return 0;
    };
    int rc = DM_OK;
    uint64_t next_scan = 0, piece = 0;
    bool slot_used[kFlSlots] = {};
    // scan windows [next_scan, upto) in order, waiting for each; 1 = found, -1 = error
    auto scan_upto = [&](uint64_t upto, bool wait) -> int {
        while (next_scan < upto) {
            hipEvent_t e = ev.hashed[next_scan % 2];
            if (wait) {
                if (hipEventSynchronize(e) != hipSuccess) return -1;
            } else if (hipEventQuery(e) != hipSuccess) {
                (void)hipGetLastError();
                return 0;
            }
            const int hit = scan(next_scan++);
            if (hit != 0) return hit;
        }
        return 0;
    };
    int hit = 0;
    for (uint64_t w = 0; w < nwin && hit == 0; w++) {
        const int b = (int)(w % 2);
        const uint64_t s0 = w * win, ns = std::min(win, nseg - s0);
        // half b is free: window w - 2 was hashed and scanned before window w - 1 was launched.
        // Read the window through the pinned slots; each piece's H2D runs while the next is read,
        // and the GPU hashes window w - 1 meanwhile.
        for (uint64_t p0 = 0; p0 < ns; p0 += spd, piece++) {
            const int sl = (int)(piece % kFlSlots);
            const uint64_t np = std::min(spd, ns - p0);
            if (slot_used[sl]) HIP_TRY(hipEventSynchronize(ev.slot[sl]));
            uint8_t* slot = L.fp_slot[sl].u8();
            std::vector<FilePart> parts;
            for (uint64_t t = 0; t < np; t++) {   // 8 MiB parts, so every reader thread has work
                const uint64_t off = (s0 + p0 + t) * segment, have = off < size ? std::min(segment, size - off) : 0;
                for (uint64_t q = 0; q < have; q += kFlPartBytes)
                    parts.push_back({0, off + q, std::min(kFlPartBytes, have - q), slot + t * segment + q});
                if (have < segment) std::memset(slot + t * segment + have, 0, segment - have);   // zero padding
            }
            if ((rc = read_parts(c, fs, parts, readers)) != DM_OK) return rc;
            HIP_TRY(hipMemcpyAsync(data[b] + p0 * segment, slot, np * segment, hipMemcpyHostToDevice, cp));
            HIP_TRY(hipEventRecord(ev.slot[sl], cp));
            slot_used[sl] = true;
        }
        HIP_TRY(hipEventRecord(ev.copied[b], cp));
        // window w - 1's names before window w is launched: a hit there ends the call without
        // waiting for another window's chains (a window's chain, ~0.13 s, is about its read time)
        if ((hit = scan_upto(w, true)) != 0) break;
        HIP_TRY(hipStreamWaitEvent(s, ev.copied[b], 0));
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
        HIP_TRY(hipEventRecord(ev.hashed[b], s));
    }
    if (hit == 0) hit = scan_upto(nwin, true);   // the windows still in flight, in order
    if (hit < 0) rc = fail(c, DM_ERR_HIP, "dm_fragment_lookup: waiting for or copying a window");
    // the parity ring of a large file does not stay resident (the lane trims its object buffer
    // itself at unlock); the reaper's free waits for the work still queued
    if (L.work.cap > kFpKeepBytes) c->reaper.put(d.id, L.work);
    return rc;
}

}  // extern "C"
