// merkle_stream.inl -- incremental Merkle root of one object whose bytes arrive in pieces
// (hash the upload body while it is received instead of after
// node/objectHandler.go:248-266 / node/fileHandler.go:899-937 have written it to a temp file).
// Included by merkle_capi.hip (shares its internal helpers).
//
// Host pieces -> pinned staging (2 slots) -> H2D into leaf-aligned device segments (copy
// stream) -> as soon as enough whole leaves are on the device, a leaf-kernel launch over them
// on one of kStreamLanes compute streams (so several batches hash concurrently while more bytes
// arrive) -> at close, the last partial leaf, then the tree over all leaf digests.

namespace {

constexpr uint64_t kStreamStage = 64ull << 20;   // pinned staging slot
constexpr int kStreamLanes = 2;                  // concurrent compute streams per object
// A batch launches once it can fill the chip by itself (32 leaves per CU in the pair kernel) or
// holds this many bytes: every launch of a long-leaf object then runs ~one leaf-time, and
// staging copies are not queued behind a stream of small latency-bound launches.
constexpr uint64_t kStreamLeavesPerCu = 32;
constexpr uint64_t kStreamMinBytes = 4ull << 30;

struct StreamSeg {
    DevBuf data;      // seg_leaves * chunk bytes
};

// One leaf-kernel launch: its leaves may span segments (table mode), its digests are its own.
struct StreamBatch {
    uint64_t first = 0, count = 0;
    DevBuf tab;       // count x (address, length)
    DevBuf digests;   // count x 32 bytes
};

}  // namespace

struct dm_stream {
    dm_ctx* c = nullptr;
    int dev = 0;
    StreamKit* kit = nullptr;   // pooled streams, events, staging (borrowed for the stream's life)
    uint64_t chunk = 0;
    uint64_t seg_leaves = 0;
    std::vector<StreamSeg*> segs;
    std::vector<StreamBatch*> batches;
    PinnedBuf stage[2];
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    int slot = 0;
    uint64_t fill = 0;
    hipStream_t copy = nullptr;
    hipStream_t comp[kStreamLanes] = {};
    hipEvent_t ev_copy = nullptr;
    hipEvent_t ev_comp[kStreamLanes] = {};
    int next_comp = 0;
    uint64_t received = 0;   // bytes handed to dm_stream_write
    uint64_t on_device = 0;  // bytes whose H2D is enqueued
    uint64_t launched = 0;   // leaves whose hashing is enqueued
    std::string err;
    int failed = DM_OK;      // sticky: after a failed write nothing more reaches the GPU; close returns it
    Dev tree;                // the stream's own tree scratch (leaves, K2 nodes, root): close takes no context lock
};

namespace {

int sfail(dm_stream* st, int code, const char* what, hipError_t e) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    st->err = buf;
    t_err = buf;
    return code;
}

#define SHIP(expr)                                                                               \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return sfail(st, e_ == hipErrorOutOfMemory ? DM_ERR_NOMEM : DM_ERR_HIP, #expr, e_); \
    } while (0)

int stream_seg_for(dm_stream* st, uint64_t leaf, StreamSeg** out) {
    const uint64_t si = leaf / st->seg_leaves;
    while (st->segs.size() <= si) {
        StreamSeg* g = new StreamSeg();
        st->segs.push_back(g);
        SHIP(g->data.ensure(st->seg_leaves * st->chunk));
    }
    *out = st->segs[si];
    return DM_OK;
}

// Enqueue hashing of leaves [launched, upto) as ONE launch (table mode across segments, so a
// batch of long leaves runs concurrently, never as a serial chain of per-segment launches); the
// leaf upto-1 may be the short last one.
int stream_launch(dm_stream* st, uint64_t upto, uint64_t last_len) {
    if (upto <= st->launched) return DM_OK;
    StreamBatch* bt = new StreamBatch();
    st->batches.push_back(bt);
    bt->first = st->launched;
    bt->count = upto - st->launched;
    const uint64_t n = bt->count;
    uint8_t* htab = kit_table(st->c, st->c->devs[st->dev].id, st->kit, 16 * n);   // host side of tab
    if (!htab) return sfail(st, DM_ERR_NOMEM, "pinned table arena", hipErrorOutOfMemory);
    SHIP(bt->tab.ensure(16 * n));
    SHIP(bt->digests.ensure(32 * n));
    uint64_t* h = reinterpret_cast<uint64_t*>(htab);
    for (uint64_t j = 0; j < n; j++) {
        const uint64_t leaf = bt->first + j;
        StreamSeg* g;
        int rc = stream_seg_for(st, leaf, &g);
        if (rc != DM_OK) return rc;
        h[j] = reinterpret_cast<uint64_t>(g->data.u8() + (leaf % st->seg_leaves) * st->chunk);
        h[n + j] = (leaf + 1 == upto) ? last_len : st->chunk;
    }
    SHIP(hipEventRecord(st->ev_copy, st->copy));
    const int k = st->next_comp++ % kStreamLanes;
    hipStream_t s = st->comp[k];
    SHIP(hipStreamWaitEvent(s, st->ev_copy, 0));
    SHIP(hipMemcpyAsync(bt->tab.p, htab, 16 * n, hipMemcpyHostToDevice, s));
    dm::LeafArgs la{};
    la.addrs = static_cast<const uint64_t*>(bt->tab.p);
    la.lens = la.addrs + n;
    la.nleaves = n;
    la.byte_end = ~0ull;
    la.digests = bt->digests.u8();
    const int kind = pick_leaf_kernel(st->c, st->c->devs[st->dev], n);
    launch_leaves_t<true, true>(s, la, kind, st->c->devs[st->dev].cus);
    SHIP(hipGetLastError());
    st->launched = upto;
    SHIP(hipEventRecord(st->ev_comp[k], s));
    return DM_OK;
}

// Move the filled staging slot to the device and launch whatever whole leaves are ready.
int stream_flush(dm_stream* st) {
    if (st->fill == 0) return DM_OK;
    const uint8_t* src = st->stage[st->slot].u8();
    uint64_t pos = st->on_device, left = st->fill;
    while (left) {
        StreamSeg* g;
        int rc = stream_seg_for(st, pos / st->chunk, &g);
        if (rc != DM_OK) return rc;
        const uint64_t seg_off = pos - (pos / st->chunk / st->seg_leaves) * st->seg_leaves * st->chunk;
        const uint64_t room = st->seg_leaves * st->chunk - seg_off;
        const uint64_t n = std::min(left, room);
        SHIP(hipMemcpyAsync(g->data.u8() + seg_off, src, n, hipMemcpyHostToDevice, st->copy));
        src += n;
        pos += n;
        left -= n;
    }
    SHIP(hipEventRecord(st->ev_stage[st->slot], st->copy));
    st->busy[st->slot] = true;
    st->on_device += st->fill;
    st->slot ^= 1;
    st->fill = 0;
    const uint64_t ready = st->on_device / st->chunk;
    const uint64_t pending = ready > st->launched ? ready - st->launched : 0;
    const uint64_t fill_leaves = kStreamLeavesPerCu * (uint64_t)st->c->devs[st->dev].cus;
    if (pending >= fill_leaves || pending * st->chunk >= kStreamMinBytes)
        return stream_launch(st, ready, st->chunk);
    return DM_OK;
}

// End of a stream: wait for its own work only, hand its device buffers to the reaper (freeing
// them here would wait for every other caller's kernels on the device) and its kit back to the pool.
void stream_free(dm_stream* st) {
    if (!st) return;
    dm_ctx* c = st->c;
    const int id = c->devs[st->dev].id;
    (void)hipSetDevice(id);
    bool idle = true;
    if (st->kit)
        for (hipStream_t s : {st->copy, st->comp[0], st->comp[1]})
            if (s && hipStreamSynchronize(s) != hipSuccess) idle = false;
    for (StreamSeg* g : st->segs) {
        c->reaper.put(id, g->data);
        delete g;
    }
    for (StreamBatch* b : st->batches) {
        c->reaper.put(id, b->tab);
        c->reaper.put(id, b->digests);
        delete b;
    }
    for (DevBuf* b : {&st->tree.leaves, &st->tree.nodes_a, &st->tree.nodes_b, &st->tree.root}) c->reaper.put(id, *b);
    if (st->kit) {
        for (int i = 0; i < 2; i++) st->kit->slot[i] = st->stage[i];
        if (idle) kit_release(c, st->dev, st->kit);
        else kit_destroy(st->kit);   // a failed stream's kit is not reused
    }
    c->slots[st->dev].load--;   // the stream's hold on its device's load (dm_stream_open)
    delete st;
}

int stream_write(dm_stream* st, const void* data, uint64_t len);

}  // namespace

extern "C" {

int dm_stream_open(dm_ctx* ctx, uint64_t chunk, dm_stream** out) {
    if (!ctx || !out || chunk == 0) return bad_arg();
    *out = nullptr;
    DeviceRestore dev;
    if (chunk % 16 != 0) return fail(ctx, DM_ERR_INVALID, "dm_stream: chunk must be a multiple of 16 bytes");
    dm_stream* st = new dm_stream();
    st->c = ctx;
    // a stream keeps one lane busy while the body arrives: the least-loaded one, counted in its
    // load until the stream is freed, so concurrent uploads spread over the context's GPUs and lanes
    st->dev = pick_device(ctx);
    st->tree.id = ctx->devs[st->dev].id;
    st->tree.cus = ctx->devs[st->dev].cus;
    st->chunk = chunk;
    st->seg_leaves = std::max<uint64_t>(1, (1ull << 30) / chunk);
    int rc = DM_OK;
    do {
        hipError_t e;
        if ((e = hipSetDevice(ctx->devs[st->dev].id)) != hipSuccess) { rc = sfail(st, DM_ERR_HIP, "hipSetDevice", e); break; }
        if ((rc = kit_acquire(ctx, st->dev, &st->kit)) != DM_OK) {
            st->err = t_err;
            break;
        }
        StreamKit* k = st->kit;
        st->copy = k->copy;   // copies on the kit's high-priority stream (its own hardware queue)
        for (int i = 0; i < kStreamLanes; i++) {
            st->comp[i] = k->comp[i];
            st->ev_comp[i] = k->ev[1 + i];
        }
        st->ev_copy = k->ev[0];
        st->ev_stage[0] = k->ev[3];
        st->ev_stage[1] = k->ev[4];
        for (int i = 0; i < 2; i++) {
            st->stage[i] = k->slot[i];
            k->slot[i] = PinnedBuf();
            if ((e = pinned_grow(ctx, ctx->devs[st->dev].id, st->stage[i], kStreamStage)) != hipSuccess) {
                rc = sfail(st, DM_ERR_NOMEM, "pinned staging", e);
                break;
            }
        }
    } while (0);
    if (rc != DM_OK) {
        {
            std::lock_guard<std::mutex> lk(ctx->err_mu);
            ctx->err = st->err;
        }
        t_err = st->err;
        stream_free(st);
        return rc;
    }
    *out = st;
    return DM_OK;
}

int dm_stream_write(dm_stream* st, const void* data, uint64_t len) {
    if (!st || (!data && len)) return bad_arg();
    if (st->failed != DM_OK) {
        t_err = st->err;
        return st->failed;
    }
    const int rc = stream_write(st, data, len);
    if (rc != DM_OK) st->failed = rc;
    return rc;
}

}  // extern "C"

namespace {

int stream_write(dm_stream* st, const void* data, uint64_t len) {
    // fast path: the piece fits the staging slot being filled (no slot wait, no flush): one
    // memcpy and no HIP call (Go's io.Copy hands over 32 KiB at a time)
    if (len < kStreamStage - st->fill && !(st->fill == 0 && st->busy[st->slot])) {
        std::memcpy(st->stage[st->slot].u8() + st->fill, data, len);
        st->fill += len;
        st->received += len;
        return DM_OK;
    }
    DeviceRestore dev;
    SHIP(hipSetDevice(st->c->devs[st->dev].id));
    const uint8_t* p = static_cast<const uint8_t*>(data);
    while (len) {
        if (st->fill == 0 && st->busy[st->slot]) {
            SHIP(hipEventSynchronize(st->ev_stage[st->slot]));
            st->busy[st->slot] = false;
        }
        const uint64_t take = std::min(len, kStreamStage - st->fill);
        std::memcpy(st->stage[st->slot].u8() + st->fill, p, take);
        st->fill += take;
        st->received += take;
        p += take;
        len -= take;
        if (st->fill == kStreamStage) {
            int rc = stream_flush(st);
            if (rc != DM_OK) return rc;
        }
    }
    return DM_OK;
}

}  // namespace

extern "C" {

const char* dm_stream_error(dm_stream* st) { return st ? st->err.c_str() : ""; }

int dm_stream_close(dm_stream* st, uint8_t* leaf_out, uint64_t leaf_cap, uint64_t* nleaves, uint8_t root[32]) {
    if (!st || !root) return bad_arg();
    if (st->failed != DM_OK) {   // a write failed: free the stream, report that failure
        const int rc = st->failed;
        t_err = st->err;
        DeviceRestore dev;
        stream_free(st);
        return rc;
    }
    DeviceRestore dev;
    dm_ctx* c = st->c;
    int rc = DM_OK;
    t_err.clear();
    do {
        if (st->received == 0) {
            rc = DM_ERR_EMPTY;
            st->err = "Empty data";
            break;
        }
        if (hipSetDevice(c->devs[st->dev].id) != hipSuccess) { rc = DM_ERR_HIP; break; }
        if ((rc = stream_flush(st)) != DM_OK) break;
        const uint64_t n = ceil_div(st->received, st->chunk);
        if ((rc = stream_launch(st, n, st->received - (n - 1) * st->chunk)) != DM_OK) break;
        if (nleaves) *nleaves = n;
        // tree over all leaf digests on the stream's first compute lane, after the other lane, in
        // the stream's own scratch: no context lock, so a close never waits behind another call
        Dev& d = st->tree;
        hipStream_t s = st->comp[0];
        for (int k = 1; k < kStreamLanes; k++) {
            hipError_t e = hipStreamWaitEvent(s, st->ev_comp[k], 0);
            if (e != hipSuccess) { rc = fail(c, DM_ERR_HIP, "hipStreamWaitEvent: %s", hipGetErrorString(e)); break; }
        }
        if (rc != DM_OK) break;
        hipError_t e = d.leaves.ensure(n * 32);
        if (e == hipSuccess) e = d.root.ensure(32);
        if (e != hipSuccess) { rc = fail(c, DM_ERR_NOMEM, "leaf digests: %s", hipGetErrorString(e)); break; }
        for (StreamBatch* b : st->batches) {
            e = hipMemcpyAsync(d.leaves.u8() + 32 * b->first, b->digests.p, b->count * 32, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) { rc = fail(c, DM_ERR_HIP, "digest gather: %s", hipGetErrorString(e)); break; }
        }
        if (rc != DM_OK) break;
        if ((rc = finish(c, d, s, d.leaves.u8(), n, true, d.root.u8())) != DM_OK) break;
        if ((e = hipMemcpyAsync(root, d.root.p, 32, hipMemcpyDeviceToHost, s)) != hipSuccess) {
            rc = fail(c, DM_ERR_HIP, "root copy: %s", hipGetErrorString(e));
            break;
        }
        if (leaf_out && leaf_cap) {
            e = hipMemcpyAsync(leaf_out, d.leaves.p, std::min(leaf_cap, n) * 32, hipMemcpyDeviceToHost, s);
            if (e != hipSuccess) { rc = fail(c, DM_ERR_HIP, "leaf copy: %s", hipGetErrorString(e)); break; }
        }
        if ((e = hipStreamSynchronize(s)) != hipSuccess) rc = fail(c, DM_ERR_HIP, "close sync: %s", hipGetErrorString(e));
    } while (0);
    if (rc != DM_OK && !st->err.empty()) {
        std::lock_guard<std::mutex> lk(c->err_mu);
        if (c->err.empty() || rc == DM_ERR_EMPTY) c->err = st->err;
        if (t_err.empty() || rc == DM_ERR_EMPTY) t_err = st->err;
    }
    stream_free(st);
    return rc;
}

void dm_stream_abort(dm_stream* st) {
    DeviceRestore dev;
    stream_free(st);
}

}  // extern "C"
