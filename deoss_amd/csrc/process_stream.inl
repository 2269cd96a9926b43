// process_stream.inl -- dm_pstream_*: FullProcessing while the upload body arrives (SURVEY.md 8f
// #1 + #2).  The upload handlers write the body to a file (node/objectHandler.go:248-266
// saveObjectToFile, node/fileHandler.go:899-937) and only then run cess-go-sdk
// FullProcessing(fpath, cipher, cacheDir) over it (node/objectHandler.go:168,
// node/fileHandler.go:771), which reads the file again.  A pstream takes the body in pieces of any
// size (io.MultiWriter beside the file) and does the FullProcessing work as the bytes arrive:
//   - pieces fill a pinned slot of whole segments; a full slot is copied to its own device chunk
//     (segments + room for their parity), its data fragments and segment files are written to
//     temporary names by background writers, and one RS launch codes the chunk;
//   - a chunk's parity comes back through a free slot and is written as soon as its RS launch
//     (on its own stream, in chunk order) has finished (checked whenever a slot is taken);
//   - every kPsBatchChunks chunks, one table-mode leaf launch hashes their segments and fragments
//     on one of two compute streams (the 32 MiB segment chains of one batch run while later
//     batches arrive);
//   - close pads the last segment, launches the last chunk and batch, drains the parity, builds
//     the fid over all segment digests and renames every temporary to savedir/<hex SHA-256>.
// Device memory is bounded, not proportional to the body: a chunk's buffer (3 x its segments at
// 4 + 8) returns to the stream's spare list once its parity has been written out and the leaf
// launch that hashed it has finished, and new chunks reuse spare buffers.  When the buffers held
// reach the cap (DEOSS_PS_DEVICE_CAP, default kPsDeviceCap), write blocks: it launches the pending
// batch early and waits for the oldest chunk to be reclaimable.
// Results are those of dm_full_processing on the same bytes.  Part of merkle_capi.hip (after
// fullproc_capi.inl: SlotWrites, write_whole, mkdir_all, hex32, env_bytes).

namespace {

constexpr int kPsSlots = 4;
static_assert(kPsSlots == StreamKit::kSlots && StreamKit::kEvents >= 2 + kPsSlots, "pstream kit layout");
constexpr uint64_t kPsSlotBytes = 64ull << 20;
constexpr uint64_t kPsBatchChunks = 32;   // 64 segments = 2 GiB of body per leaf launch (32 MiB segments)
// Device bytes one pstream may hold: two 6 GiB batches in flight (32 chunks x 2 segments x 96 MiB)
// plus the chunks arriving meanwhile, so both leaf lanes stay busy at full rate.
constexpr uint64_t kPsDeviceCap = 16ull << 30;

struct PsBatch;

struct PsChunk {
    uint64_t s0 = 0, ns = 0;      // segments [s0, s0 + ns)
    DevBuf mem;                   // ns * seg of data, then ns * pbytes of parity
    hipEvent_t ev_rs = nullptr;   // RS done: parity may be copied out
    bool drained = false;         // parity written out (its D2H has completed)
    PsBatch* batch = nullptr;     // the leaf launch that hashes this chunk (nullptr: not launched yet)
};

struct PsBatch {
    uint64_t c0 = 0, nc = 0, s0 = 0, ns = 0;   // chunks [c0, c0 + nc) = segments [s0, s0 + ns)
    DevBuf tab, dig;                            // leaf table; digests: ns segments, then ns x total fragments
    int lane = 0;
    hipEvent_t ev_done = nullptr;               // the leaf launch has finished reading its chunks
};

}  // namespace

struct dm_pstream {
    dm_rs* r = nullptr;
    StreamKit* kit = nullptr;   // pooled streams, events, pinned slots (borrowed for the stream's life)
    int k = 0, m = 0, total = 0, flags = 0;
    uint64_t seg = 0, frag = 0, pbytes = 0, spd = 1, spp = 1, slot_len = 0, batch_chunks = kPsBatchChunks;
    std::string dir, base;
    PinnedBuf slot[kPsSlots];
    hipEvent_t ev_slot[kPsSlots] = {};
    SlotWrites wr[kPsSlots];
    bool busy[kPsSlots] = {};
    uint64_t next_slot = 0;
    int cur = -1;              // slot being filled, -1: none
    uint64_t fill = 0;
    uint64_t received = 0;
    hipStream_t copy = nullptr, code = nullptr, comp[2] = {nullptr, nullptr};   // H2D/D2H, RS, leaf lanes
    hipEvent_t ev_copy = nullptr, ev_code = nullptr;
    std::vector<PsChunk*> chunks;
    std::vector<PsBatch*> batches;
    uint64_t hashed_chunks = 0;     // chunks covered by leaf launches
    uint64_t drained_upto = 0;      // chunks [0, drained_upto) have their parity written
    uint64_t reclaimed_upto = 0;    // chunks [0, reclaimed_upto) gave their device buffer back
    std::vector<DevBuf> spare;      // reclaimed chunk buffers, reused by later chunks
    uint64_t dev_cap = kPsDeviceCap, dev_held = 0, dev_peak = 0;   // chunk buffers allocated (in use + spare)
    std::vector<std::pair<std::string, uint64_t>> pend;   // temporary, digest index (~: segment)
    std::string err;
    int failed = DM_OK;   // sticky: after a failed write the stream only aborts (close returns this)
    Dev tree;             // the stream's own fid scratch: close takes no context lock
};

namespace {

int pfail(dm_pstream* st, int code, const std::string& msg) {
    st->err = msg;
    t_err = msg;
    return code;
}

#define PSHIP(expr)                                                                              \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return pfail(st, e_ == hipErrorOutOfMemory ? DM_ERR_NOMEM : DM_ERR_HIP,               \
                         std::string(#expr) + ": " + hipGetErrorString(e_));                     \
    } while (0)

Dev& ps_dev(dm_pstream* st) { return st->r->c->devs[0]; }

// A free slot (its H2D / D2H finished and its writes joined).  Slots are pinned on first use, so a
// small body holds one slot, not four.
int ps_take_slot(dm_pstream* st, int* out) {
    int sl;
    do {   // never the slot being filled / flushed (a drain inside ps_flush must not reuse it)
        sl = (int)(st->next_slot++ % kPsSlots);
    } while (sl == st->cur);
    PSHIP(pinned_grow(st->r->c, ps_dev(st).id, st->slot[sl], std::max(st->slot_len, st->spp * st->pbytes)));
    if (st->busy[sl]) {
        PSHIP(hipEventSynchronize(st->ev_slot[sl]));
        const std::string e = st->wr[sl].wait();
        if (!e.empty()) return pfail(st, DM_ERR_IO, e);
        st->busy[sl] = false;
    }
    *out = sl;
    return DM_OK;
}

// Copy chunk ci's parity out through a slot and write its parity fragments (RS must be done).
int ps_drain_chunk(dm_pstream* st, uint64_t ci) {
    PsChunk* ch = st->chunks[ci];
    if (!ch->mem.p) return pfail(st, DM_ERR_INVALID, "pstream: draining a chunk without device memory");
    uint8_t* parity = ch->mem.u8() + ch->ns * st->seg;
    for (uint64_t t0 = 0; t0 < ch->ns; t0 += st->spp) {
        const uint64_t nt = std::min(st->spp, ch->ns - t0);
        int sl;
        int rc = ps_take_slot(st, &sl);
        if (rc != DM_OK) return rc;
        uint8_t* buf = st->slot[sl].u8();
        PSHIP(hipStreamWaitEvent(st->copy, ch->ev_rs, 0));
        PSHIP(hipMemcpyAsync(buf, parity + t0 * st->pbytes, nt * st->pbytes, hipMemcpyDeviceToHost, st->copy));
        PSHIP(hipEventRecord(st->ev_slot[sl], st->copy));
        PSHIP(hipEventSynchronize(st->ev_slot[sl]));
        std::vector<FpFile> files;
        for (uint64_t u = 0; u < nt; u++) {
            const uint64_t gs = ch->s0 + t0 + u;
            for (int i = 0; i < st->m; i++) {
                const uint64_t id = gs * (uint64_t)st->total + (uint64_t)(st->k + i);
                files.push_back({buf + u * st->pbytes + (uint64_t)i * st->frag, st->frag,
                                 st->base + "f" + std::to_string(id)});
                st->pend.emplace_back(files.back().tmp, 32 * id);
            }
        }
        st->wr[sl].start(std::move(files));
        st->busy[sl] = true;
    }
    ch->drained = true;
    return DM_OK;
}

// Drain every chunk, in order, whose RS launch has finished (all of them when `all`).
int ps_drain(dm_pstream* st, bool all) {
    while (st->drained_upto < st->chunks.size()) {
        PsChunk* ch = st->chunks[st->drained_upto];
        if (!all) {
            const hipError_t q = hipEventQuery(ch->ev_rs);
            if (q == hipErrorNotReady) break;
            PSHIP(q);
        }
        int rc = ps_drain_chunk(st, st->drained_upto);
        if (rc != DM_OK) return rc;
        st->drained_upto++;
    }
    return DM_OK;
}

// One table-mode leaf launch over chunks [hashed_chunks, upto): segments first, then fragments.
int ps_launch_batch(dm_pstream* st, uint64_t upto) {
    if (upto <= st->hashed_chunks) return DM_OK;
    Dev& d = ps_dev(st);
    PsBatch* b = new PsBatch();
    st->batches.push_back(b);
    b->c0 = st->hashed_chunks;
    b->nc = upto - b->c0;
    b->s0 = st->chunks[b->c0]->s0;
    for (uint64_t c = b->c0; c < upto; c++) {
        if (!st->chunks[c]->mem.p)   // every chunk of a launch holds its data (host-side guard)
            return pfail(st, DM_ERR_INVALID, "pstream: chunk without device memory in a leaf launch");
        b->ns += st->chunks[c]->ns;
    }
    const uint64_t T = b->ns * (1 + (uint64_t)st->total);
    uint8_t* htab = kit_table(st->r->c, d.id, st->kit, 16 * T);   // host side of the leaf table
    if (!htab) return pfail(st, DM_ERR_NOMEM, "pstream: pinned table arena");
    PSHIP(b->tab.ensure(16 * T));
    PSHIP(b->dig.ensure(32 * T));
    uint64_t* addr = reinterpret_cast<uint64_t*>(htab);
    uint64_t* lens = addr + T;
    uint64_t i = 0;
    for (uint64_t c = b->c0; c < upto; c++) {
        PsChunk* ch = st->chunks[c];
        for (uint64_t u = 0; u < ch->ns; u++, i++) {
            addr[i] = reinterpret_cast<uint64_t>(ch->mem.u8() + u * st->seg);
            lens[i] = st->seg;
        }
    }
    for (uint64_t c = b->c0; c < upto; c++) {
        PsChunk* ch = st->chunks[c];
        const uint8_t* parity = ch->mem.u8() + ch->ns * st->seg;
        for (uint64_t u = 0; u < ch->ns; u++)
            for (int j = 0; j < st->total; j++, i++) {
                addr[i] = reinterpret_cast<uint64_t>(
                    j < st->k ? ch->mem.u8() + u * st->seg + (uint64_t)j * st->frag
                              : parity + (u * st->m + (uint64_t)(j - st->k)) * st->frag);
                lens[i] = st->frag;
            }
    }
    b->lane = (int)(st->batches.size() % 2);
    hipStream_t s = st->comp[b->lane];
    // after the RS launches of these chunks (in order on the code stream); batches on the two
    // lanes overlap, so one batch's segment chains run while the next batch arrives
    PSHIP(hipEventRecord(st->ev_code, st->code));
    PSHIP(hipStreamWaitEvent(s, st->ev_code, 0));
    PSHIP(hipMemcpyAsync(b->tab.p, htab, 16 * T, hipMemcpyHostToDevice, s));
    dm::LeafArgs la{};
    la.addrs = static_cast<const uint64_t*>(b->tab.p);
    la.lens = la.addrs + T;
    la.nleaves = T;
    la.byte_end = ~0ull;
    la.digests = b->dig.u8();
    launch_leaves_t<true, true>(s, la, pick_leaf_kernel(st->r->c, d, T), d.cus);
    PSHIP(hipGetLastError());
    PSHIP(hipEventCreateWithFlags(&b->ev_done, hipEventDisableTiming));
    PSHIP(hipEventRecord(b->ev_done, s));
    for (uint64_t c = b->c0; c < upto; c++) st->chunks[c]->batch = b;
    st->hashed_chunks = upto;
    return DM_OK;
}

// Return the buffers of chunks whose parity is written out and whose leaf launch has finished to
// the spare list, oldest first (drains and launches run in chunk order).  wait: block for the
// oldest chunk that is still in use (after launching its batch and draining its parity).
int ps_reclaim(dm_pstream* st, bool wait) {
    while (st->reclaimed_upto < st->chunks.size()) {
        PsChunk* ch = st->chunks[st->reclaimed_upto];
        if (wait && !ch->batch) RC_TRY(ps_launch_batch(st, st->chunks.size()));
        if (wait && !ch->drained) RC_TRY(ps_drain(st, true));
        if (!ch->batch || !ch->drained) break;
        if (wait) {
            PSHIP(hipEventSynchronize(ch->batch->ev_done));
        } else {
            const hipError_t q = hipEventQuery(ch->batch->ev_done);
            if (q == hipErrorNotReady) break;
            PSHIP(q);
        }
        st->spare.push_back(ch->mem);
        ch->mem = DevBuf();
        st->reclaimed_upto++;
        wait = false;   // one chunk freed is enough to make progress
    }
    return DM_OK;
}

// A device buffer of `bytes` for the next chunk: a spare one, a new one within the cap, or (cap
// reached) the oldest in-use buffer once it can be reclaimed.
int ps_chunk_buffer(dm_pstream* st, uint64_t bytes, DevBuf* out) {
    RC_TRY(ps_reclaim(st, false));
    for (;;) {
        for (size_t i = 0; i < st->spare.size(); i++)
            if (st->spare[i].cap >= bytes) {
                *out = st->spare[i];
                st->spare.erase(st->spare.begin() + (ptrdiff_t)i);
                return DM_OK;
            }
        const uint64_t sz = round_up(std::max<uint64_t>(bytes, 4096), 2ull << 20);
        if (st->dev_held + sz <= st->dev_cap || st->reclaimed_upto == st->chunks.size()) {
            DevBuf b;
            PSHIP(b.ensure(sz));
            st->dev_held += b.cap;
            st->dev_peak = std::max(st->dev_peak, st->dev_held);
            *out = b;
            return DM_OK;
        }
        if (!st->spare.empty()) {   // spare buffers too small for this chunk: give them back first
            for (auto& b : st->spare) {
                st->dev_held -= b.cap;
                st->r->c->reaper.put(ps_dev(st).id, b);
            }
            st->spare.clear();
            continue;
        }
        const uint64_t before = st->reclaimed_upto;
        RC_TRY(ps_reclaim(st, true));
        if (st->reclaimed_upto == before) return pfail(st, DM_ERR_NOMEM, "pstream: device cap reached, nothing to reclaim");
    }
}

// The current slot holds `len` bytes (whole segments, the last one zero-padded at close): copy it
// to a new device chunk, write its data fragments and segments, code it.
int ps_flush(dm_pstream* st) {
    if (st->cur < 0 || st->fill == 0) return DM_OK;
    Dev& d = ps_dev(st);
    const int sl = st->cur;
    const uint64_t ns = ceil_div(st->fill, st->seg), len = ns * st->seg;
    uint8_t* buf = st->slot[sl].u8();
    if (len > st->fill) std::memset(buf + st->fill, 0, len - st->fill);
    // the buffer first: reclaiming may launch and drain every chunk already in the list, and a
    // chunk joins the list only once it has memory (its H2D and RS follow right below)
    DevBuf mem;
    RC_TRY(ps_chunk_buffer(st, ns * (st->seg + st->pbytes), &mem));
    PsChunk* ch = new PsChunk();
    ch->mem = mem;
    ch->s0 = st->chunks.empty() ? 0 : st->chunks.back()->s0 + st->chunks.back()->ns;
    ch->ns = ns;
    st->chunks.push_back(ch);
    PSHIP(hipEventCreateWithFlags(&ch->ev_rs, hipEventDisableTiming));
    PSHIP(hipMemcpyAsync(ch->mem.p, buf, len, hipMemcpyHostToDevice, st->copy));
    PSHIP(hipEventRecord(st->ev_slot[sl], st->copy));
    std::vector<FpFile> files;
    for (uint64_t u = 0; u < ns; u++) {
        const uint64_t gs = ch->s0 + u;
        for (int j = 0; j < st->k; j++) {
            const uint64_t id = gs * (uint64_t)st->total + (uint64_t)j;
            files.push_back({buf + u * st->seg + (uint64_t)j * st->frag, st->frag, st->base + "f" + std::to_string(id)});
            st->pend.emplace_back(files.back().tmp, 32 * id);
        }
        if (st->flags & DM_FP_SEGMENT_FILES) {
            files.push_back({buf + u * st->seg, st->seg, st->base + "s" + std::to_string(gs)});
            st->pend.emplace_back(files.back().tmp, ~(32 * gs));
        }
    }
    st->wr[sl].start(std::move(files));
    st->busy[sl] = true;
    st->cur = -1;
    st->fill = 0;
    // RS on the code stream after the H2D
    hipStream_t s = st->code;
    PSHIP(hipEventRecord(st->ev_copy, st->copy));
    PSHIP(hipStreamWaitEvent(s, st->ev_copy, 0));
    dm::RsArgs a{};
    for (int j = 0; j < st->k; j++) a.in[j] = ch->mem.u8() + (uint64_t)j * st->frag;
    uint8_t* parity = ch->mem.u8() + len;
    for (int i = 0; i < st->m; i++) a.out[i] = parity + (uint64_t)i * st->frag;
    a.in_seg_stride = st->seg;
    a.out_seg_stride = st->pbytes;
    a.units_per_seg = st->frag / 16;
    a.nseg = ns;
    a.table = static_cast<const uint2*>(st->r->enc_tab.p);
    a.nout = (uint32_t)st->m;
    launch_rs(d, s, st->k, a);
    PSHIP(hipGetLastError());
    PSHIP(hipEventRecord(ch->ev_rs, s));
    if (st->chunks.size() - st->hashed_chunks >= st->batch_chunks) return ps_launch_batch(st, st->chunks.size());
    return DM_OK;
}

// End of a pstream: wait for its own streams only, hand its device buffers to the reaper (a
// hipFree here would wait for every other caller's kernels on the GPU) and its kit to the pool.
void ps_free(dm_pstream* st) {
    if (!st) return;
    dm_ctx* c = st->r->c;
    const int id = ps_dev(st).id;
    (void)hipSetDevice(id);
    bool idle = true;
    if (st->kit)
        for (hipStream_t s : {st->copy, st->code, st->comp[0], st->comp[1]})
            if (s && hipStreamSynchronize(s) != hipSuccess) idle = false;
    for (auto& w : st->wr) (void)w.wait();
    for (PsChunk* ch : st->chunks) {
        c->reaper.put(id, ch->mem);
        if (ch->ev_rs) (void)hipEventDestroy(ch->ev_rs);
        delete ch;
    }
    for (auto& b : st->spare) c->reaper.put(id, b);
    for (PsBatch* b : st->batches) {
        c->reaper.put(id, b->tab);
        c->reaper.put(id, b->dig);
        if (b->ev_done) (void)hipEventDestroy(b->ev_done);
        delete b;
    }
    for (DevBuf* b : {&st->tree.leaves, &st->tree.nodes_a, &st->tree.nodes_b, &st->tree.root}) c->reaper.put(id, *b);
    if (st->kit) {
        for (int i = 0; i < kPsSlots; i++) st->kit->slot[i] = st->slot[i];
        if (idle) kit_release(c, 0, st->kit);
        else kit_destroy(st->kit);   // a failed stream's kit is not reused
    } else {
        for (auto& b : st->slot) c->reaper.put(id, b);
    }
    delete st;
}

void ps_unlink_pending(dm_pstream* st) {
    for (const auto& p : st->pend)
        if (!p.first.empty()) ::unlink(p.first.c_str());
}

int pstream_write(dm_pstream* st, const void* data, uint64_t len);
int pstream_close(dm_pstream* st, uint8_t* seg_hashes, uint8_t* frag_hashes, uint64_t cap, uint64_t* nseg_out,
                  uint8_t fid[32]);

}  // namespace

extern "C" {

int dm_pstream_open(dm_rs* r, uint64_t segment, const char* savedir, int flags, dm_pstream** out) {
    if (!r || !savedir || !out) return bad_arg();
    *out = nullptr;
    dm_ctx* c = r->c;
    {
        CallLock lk(c, 0);
        RC_TRY(process_check(r, 1, segment));
    }
    DeviceRestore dev;
    dm_pstream* st = new dm_pstream();
    st->r = r;
    st->k = r->k;
    st->m = r->m;
    st->total = r->k + r->m;
    st->flags = flags;
    st->seg = segment;
    st->frag = segment / (uint64_t)r->k;
    st->pbytes = (uint64_t)r->m * st->frag;
    // test hooks (env, read at open): small slots / batches exercise slot reuse and many launches
    const uint64_t slot_bytes = env_bytes("DEOSS_FP_SLOT_BYTES", kPsSlotBytes);
    st->batch_chunks = env_bytes("DEOSS_PS_BATCH_CHUNKS", kPsBatchChunks);
    st->dev_cap = env_bytes("DEOSS_PS_DEVICE_CAP", kPsDeviceCap);
    st->spd = std::max<uint64_t>(1, slot_bytes / segment);
    st->spp = std::max<uint64_t>(1, slot_bytes / st->pbytes);
    st->slot_len = st->spd * segment;
    st->dir = savedir;
    while (st->dir.size() > 1 && st->dir.back() == '/') st->dir.pop_back();
    st->base = st->dir + "/.dm-ps-" + std::to_string((long long)::getpid()) + "-" +
               std::to_string((unsigned long long)g_fp_seq++) + "-";
    int rc = DM_OK;
    do {
        const std::string me = mkdir_all(st->dir);
        if (!me.empty()) { rc = pfail(st, DM_ERR_IO, me); break; }
        if (hipSetDevice(ps_dev(st).id) != hipSuccess) { rc = pfail(st, DM_ERR_HIP, "hipSetDevice"); break; }
        if ((rc = kit_acquire(c, 0, &st->kit)) != DM_OK) {
            st->err = t_err;
            break;
        }
        StreamKit* k = st->kit;
        st->copy = k->copy;   // H2D / D2H on the kit's high-priority stream
        st->code = k->code;
        st->comp[0] = k->comp[0];
        st->comp[1] = k->comp[1];
        st->ev_copy = k->ev[0];
        st->ev_code = k->ev[1];
        for (int i = 0; i < kPsSlots; i++) {
            st->ev_slot[i] = k->ev[2 + i];
            st->slot[i] = k->slot[i];   // pinned on first use (ps_take_slot)
            k->slot[i] = PinnedBuf();
        }
    } while (0);
    if (rc != DM_OK) {
        ps_free(st);
        return rc;
    }
    *out = st;
    return DM_OK;
}

int dm_pstream_write(dm_pstream* st, const void* data, uint64_t len) {
    if (!st || (!data && len)) return bad_arg();
    if (st->failed != DM_OK) return pfail(st, st->failed, st->err);
    const int rc = pstream_write(st, data, len);
    if (rc != DM_OK) st->failed = rc;
    return rc;
}

int dm_pstream_close(dm_pstream* st, uint8_t* seg_hashes, uint8_t* frag_hashes, uint64_t cap, uint64_t* nseg_out,
                     uint8_t fid[32]) {
    if (!st) return bad_arg();
    if (st->failed != DM_OK) {   // a write failed: nothing of this stream may reach the GPU again
        const int rc = pfail(st, st->failed, st->err);
        dm_pstream_abort(st);
        return rc;
    }
    return pstream_close(st, seg_hashes, frag_hashes, cap, nseg_out, fid);
}

}  // extern "C"

namespace {

int pstream_write(dm_pstream* st, const void* data, uint64_t len) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    // fast path (most calls: Go's io.Copy hands over 32 KiB at a time): the piece fits the slot
    // being filled, so it is one memcpy with no HIP call at all
    if (st->cur >= 0 && len < st->slot_len - st->fill) {
        std::memcpy(st->slot[st->cur].u8() + st->fill, p, len);
        st->fill += len;
        st->received += len;
        return DM_OK;
    }
    DeviceRestore dev;
    PSHIP(hipSetDevice(ps_dev(st).id));
    while (len) {
        if (st->cur < 0) {
            int rc = ps_drain(st, false);   // parity of coded chunks out first: frees slots early
            if (rc == DM_OK) rc = ps_take_slot(st, &st->cur);
            if (rc != DM_OK) return rc;
        }
        const uint64_t take = std::min(len, st->slot_len - st->fill);
        std::memcpy(st->slot[st->cur].u8() + st->fill, p, take);
        st->fill += take;
        st->received += take;
        p += take;
        len -= take;
        if (st->fill == st->slot_len) {
            int rc = ps_flush(st);
            if (rc != DM_OK) return rc;
        }
    }
    return DM_OK;
}

int pstream_close(dm_pstream* st, uint8_t* seg_hashes, uint8_t* frag_hashes, uint64_t cap, uint64_t* nseg_out,
                  uint8_t fid[32]) {
    DeviceRestore dev;
    dm_ctx* c = st->r->c;
    const uint64_t nseg = ceil_div(st->received, st->seg);
    if (nseg_out) *nseg_out = nseg;
    int rc = DM_OK;
    do {
        if (!fid) { rc = bad_arg(); break; }
        if (st->received == 0) { rc = pfail(st, DM_ERR_EMPTY, "Empty data"); break; }
        if ((seg_hashes || frag_hashes) && cap < nseg) {
            rc = pfail(st, DM_ERR_INVALID, "dm_pstream_close: " + std::to_string(nseg) + " segments, digest arrays hold " +
                                               std::to_string(cap));
            break;
        }
        if (hipSetDevice(ps_dev(st).id) != hipSuccess) { rc = pfail(st, DM_ERR_HIP, "hipSetDevice"); break; }
        if ((rc = ps_flush(st)) != DM_OK) break;
        if ((rc = ps_launch_batch(st, st->chunks.size())) != DM_OK) break;
        if ((rc = ps_drain(st, true)) != DM_OK) break;
        // digests: batch b holds its ns segments, then ns x total fragments
        std::vector<uint8_t> segd(32 * nseg), fragd(32 * nseg * st->total);
        for (PsBatch* b : st->batches) {
            hipStream_t s = st->comp[b->lane];
            hipError_t e;
            if ((e = hipMemcpyAsync(segd.data() + 32 * b->s0, b->dig.p, 32 * b->ns, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                (e = hipMemcpyAsync(fragd.data() + 32 * b->s0 * st->total, b->dig.u8() + 32 * b->ns,
                                    32 * b->ns * st->total, hipMemcpyDeviceToHost, s)) != hipSuccess) {
                rc = pfail(st, DM_ERR_HIP, std::string("digests: ") + hipGetErrorString(e));
                break;
            }
        }
        if (rc != DM_OK) break;
        for (hipStream_t s : {st->comp[0], st->comp[1], st->code, st->copy})
            if (hipStreamSynchronize(s) != hipSuccess) { rc = pfail(st, DM_ERR_HIP, "stream sync"); break; }
        if (rc != DM_OK) break;
        for (auto& w : st->wr) {
            const std::string e = w.wait();
            if (!e.empty() && rc == DM_OK) rc = pfail(st, DM_ERR_IO, e);
        }
        if (rc != DM_OK) break;
        {   // fid: the tree over every segment digest, in the stream's own scratch on its code stream
            // (no context lock: a close never waits behind a dm_full_processing on the same GPU)
            Dev& d = st->tree;
            d.id = ps_dev(st).id;
            d.cus = ps_dev(st).cus;
            hipStream_t s = st->code;
            hipError_t e;
            if ((e = d.root.ensure(32)) != hipSuccess || (e = d.leaves.ensure(32 * nseg)) != hipSuccess ||
                (e = hipMemcpyAsync(d.leaves.p, segd.data(), 32 * nseg, hipMemcpyHostToDevice, s)) != hipSuccess) {
                rc = pfail(st, DM_ERR_HIP, std::string("fid: ") + hipGetErrorString(e));
                break;
            }
            if ((rc = finish(c, d, s, d.leaves.u8(), nseg, true, d.root.u8())) != DM_OK) break;
            if ((e = hipMemcpyAsync(fid, d.root.p, 32, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                (e = hipStreamSynchronize(s)) != hipSuccess) {
                rc = pfail(st, DM_ERR_HIP, std::string("fid: ") + hipGetErrorString(e));
                break;
            }
        }
        for (auto& p : st->pend) {
            const uint64_t at = p.second;
            const uint8_t* dig = (at >> 63) ? segd.data() + ~at : fragd.data() + at;
            const std::string to = st->dir + "/" + hex32(dig);
            if (::rename(p.first.c_str(), to.c_str()) != 0) {
                rc = pfail(st, DM_ERR_IO, "rename " + p.first + " " + to + ": " + go_errno(errno));
                break;
            }
            p.first.clear();
        }
        if (rc != DM_OK) break;
        if (seg_hashes) std::memcpy(seg_hashes, segd.data(), segd.size());
        if (frag_hashes) std::memcpy(frag_hashes, fragd.data(), fragd.size());
    } while (0);
    if (rc != DM_OK) {
        t_err = st->err.empty() ? t_err : st->err;
        for (auto& w : st->wr) (void)w.wait();
        ps_unlink_pending(st);
    }
    ps_free(st);
    return rc;
}

}  // namespace

extern "C" {

int dm_pstream_stats(dm_pstream* st, uint64_t* device_bytes, uint64_t* peak_device_bytes) {
    if (!st) return bad_arg();
    if (device_bytes) *device_bytes = st->dev_held;
    if (peak_device_bytes) *peak_device_bytes = st->dev_peak;
    return DM_OK;
}

void dm_pstream_abort(dm_pstream* st) {
    if (!st) return;
    DeviceRestore dev;
    for (auto& w : st->wr) (void)w.wait();
    ps_unlink_pending(st);
    ps_free(st);
}

}  // extern "C"
