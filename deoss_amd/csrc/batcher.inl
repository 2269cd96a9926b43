// batcher.inl -- coalescing executor for concurrent callers (dm_batcher_*, include/deoss_merkle.h).
// Part of merkle_capi.hip (included after process_capi.inl).
//
// DeOSS serves every upload on its own gin goroutine and each one runs FullProcessing on its own
// file (node/objectHandler.go:168, node/fileHandler.go:771, node/filesHandler.go:201).  One
// request is one or a few 32 MiB segments: 13 serial SHA-256 chains, two K1Q workgroups -- a
// GPU used one request at a time runs < 1 % of its SIMDs, and separate streams do not fix that
// (GPU_MAX_HW_QUEUES = 4 per process).  The batcher takes blocking calls from any number of
// threads, queues them, and lets `slots` worker threads (each with its own context, streams and
// scratch) turn whatever is queued into ONE batched pass (dm_process_batch / root batch): one RS
// launch, one leaf launch over every request's leaves, one tree per request.  While one slot's
// batch runs, the next slot collects the requests that arrived meanwhile, so under load batches
// grow to the leaf budget and the GPU runs them back to back or side by side.

#include <memory>

#include "batch_queue.hpp"

namespace {

struct BatchReq : dm_batch::Req {
    const void* host = nullptr;
    uint64_t len = 0;
    uint8_t* out32 = nullptr;       // root (ROOT) or fid (PROCESS)
    uint8_t* leaf_out = nullptr;    // ROOT: leaf digests (nullable)
    void* frags_out = nullptr;      // PROCESS (nullable)
    uint8_t* seg_hashes = nullptr;  // PROCESS (nullable)
    uint8_t* frag_hashes = nullptr; // PROCESS (nullable)
};

thread_local std::string t_batcher_err;

}  // namespace

struct dm_batcher {
    int mode = DM_BATCH_ROOT;
    uint64_t unit = 0;
    int k = 0, m = 0;
    std::vector<dm_ctx*> ctxs;
    std::vector<dm_rs*> coders;
    std::vector<std::thread> workers;
    std::unique_ptr<dm_batch::Queue> q;   // requests, batching and linger (batch_queue.hpp)
};

namespace {

// ROOT batch on one slot context: per-object roots and (optionally) leaf digests.
int batch_roots_host(dm_ctx* c, const std::vector<BatchReq*>& reqs, uint64_t chunk) {
    CallLock lk(c, 0);
    Dev& d = c->devs[0];
    RC_TRY(begin_call(c, d, d.stream));
    const uint64_t n = reqs.size();
    std::vector<const void*> ptrs(n), dptr(n);
    std::vector<uint64_t> lens(n), first(n + 1, 0), addr;
    for (uint64_t o = 0; o < n; o++) {
        ptrs[o] = reqs[o]->host;
        lens[o] = reqs[o]->len;
        first[o + 1] = first[o] + ceil_div(lens[o], chunk);
    }
    // request bodies in page-locked memory are read in place by K1Q over PCIe (as dm_root_batch
    // does): no copy to HBM, and no per-request hipMemcpyAsync (4,096 pinned 1 MiB requests took
    // 292 ms through per-request copies, 191 ms pageable through the ring)
    const bool zc = zero_copy_regime(c, d, first[n]) && pinned_view(ptrs.data(), lens.data(), n, &addr);
    if (!zc) RC_TRY(pack_chunks(c, d, ptrs.data(), lens.data(), n, addr));
    for (uint64_t o = 0; o < n; o++) dptr[o] = reinterpret_cast<const void*>(addr[o]);
    HIP_TRY(d.gather.ensure(n * 32));
    RC_TRY(batch_device(c, d, d.stream, dptr.data(), lens.data(), n, chunk, d.gather.u8(), zc ? DM_LEAF_QUAD : -1));
    for (uint64_t o = 0; o < n; o++) {
        HIP_TRY(hipMemcpyAsync(reqs[o]->out32, d.gather.u8() + 32 * o, 32, hipMemcpyDeviceToHost, d.stream));
        if (reqs[o]->leaf_out)
            HIP_TRY(hipMemcpyAsync(reqs[o]->leaf_out, d.leaves.u8() + 32 * first[o], 32 * (first[o + 1] - first[o]),
                                   hipMemcpyDeviceToHost, d.stream));
    }
    HIP_TRY(hipStreamSynchronize(d.stream));
    return DM_OK;
}

int batch_process_host(dm_rs* r, const std::vector<BatchReq*>& reqs, uint64_t segment) {
    dm_ctx* c = r->c;
    CallLock lk(c, 0);
    const uint64_t n = reqs.size();
    std::vector<const void*> ptrs(n);
    std::vector<uint64_t> lens(n);
    std::vector<void*> frags(n);
    std::vector<uint8_t*> segh(n), fragh(n);
    std::vector<uint8_t> fids(32 * n);
    for (uint64_t o = 0; o < n; o++) {
        ptrs[o] = reqs[o]->host;
        lens[o] = reqs[o]->len;
        frags[o] = reqs[o]->frags_out;
        segh[o] = reqs[o]->seg_hashes;
        fragh[o] = reqs[o]->frag_hashes;
    }
    RC_TRY(process_host(r, c->devs[0], ptrs.data(), lens.data(), n, segment, frags.data(), segh.data(), fragh.data(),
                        fids.data()));
    for (uint64_t o = 0; o < n; o++) std::memcpy(reqs[o]->out32, fids.data() + 32 * o, 32);
    return DM_OK;
}

void batcher_worker(dm_batcher* b, size_t slot) {
    dm_ctx* c = b->ctxs[slot];
    std::vector<dm_batch::Req*> taken;
    std::vector<BatchReq*> batch;
    while (b->q->take(taken)) {
        batch.clear();
        for (dm_batch::Req* r : taken) batch.push_back(static_cast<BatchReq*>(r));
        const int rc = b->mode == DM_BATCH_PROCESS ? batch_process_host(b->coders[slot], batch, b->unit)
                                                   : batch_roots_host(c, batch, b->unit);
        b->q->finish(taken, rc, rc == DM_OK ? std::string() : c->err);
    }
}

int batcher_submit(dm_batcher* b, BatchReq& r) {
    if (!b->q->submit(r)) {
        t_batcher_err = "batcher is shutting down";
        return DM_ERR_INVALID;
    }
    t_batcher_err = r.err;
    return r.rc;
}

}  // namespace

extern "C" {

void dm_batcher_destroy(dm_batcher* b) {
    if (!b) return;
    if (b->q) b->q->stop();
    for (auto& t : b->workers)
        if (t.joinable()) t.join();
    for (dm_rs* r : b->coders) dm_rs_destroy(r);
    for (dm_ctx* c : b->ctxs) dm_destroy(c);
    delete b;
}

int dm_batcher_create(const int* devs, int ndev, int mode, uint64_t unit, int data_shards, int parity_shards,
                      int slots, uint64_t max_leaves, uint64_t max_bytes, uint32_t linger_us, dm_batcher** out) {
    if (!out) return DM_ERR_INVALID;
    *out = nullptr;
    std::vector<int> dl;
    if (devs) {
        dl.assign(devs, devs + std::max(ndev, 0));
    } else {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
            (void)hipGetLastError();
            t_batcher_err = "dm_batcher_create: no usable GPU";
            return DM_ERR_NODEV;
        }
        for (int i = 0; i < n; i++) dl.push_back(i);
    }
    if (dl.empty() || (mode != DM_BATCH_ROOT && mode != DM_BATCH_PROCESS) || unit == 0 || slots < 0 || slots > 8) {
        t_batcher_err = "dm_batcher_create: bad mode, unit or slot count";
        return DM_ERR_INVALID;
    }
    if (mode == DM_BATCH_PROCESS && (data_shards < 1 || unit % (16ull * (uint64_t)data_shards))) {
        t_batcher_err = "dm_batcher_create: segment must be a non-zero multiple of 16 x data shards";
        return DM_ERR_INVALID;
    }
    dm_batcher* b = new (std::nothrow) dm_batcher();
    if (!b) return DM_ERR_NOMEM;
    b->mode = mode;
    b->unit = unit;
    b->k = data_shards;
    b->m = parity_shards;
    // default 4 slots per GPU: each slot's context has its own hardware queue (a CU-masked lane
    // stream), so 4 batches run side by side; measured 2 / 3 / 4 / 6 / 8 slots: 0.278 / 0.370 /
    // 0.400 / 0.398 / 0.402 GiB/s of 1 MiB FullProcessing uploads, roots 8.2 (2) / 9.1 (4) / 8.4 (8)
    // GiB/s (profiles/r03/LOGS.md (r03y_*.log), r03z_*.log)
    const int per = slots ? slots : 4;
    const int ns = per * (int)dl.size();
    for (int i = 0; i < ns; i++) {   // slot i on device dl[i % ndev]: consecutive slots alternate GPUs
        dm_ctx* c = nullptr;
        int rc = dm_create_lanes(&c, &dl[i % dl.size()], 1, 1);   // the slots are the batcher's lanes
        if (rc != DM_OK) {
            t_batcher_err = std::string("dm_batcher_create: ") + dm_strerror(rc);
            dm_batcher_destroy(b);
            return rc;
        }
        b->ctxs.push_back(c);
        if (mode == DM_BATCH_PROCESS) {
            dm_rs* r = nullptr;
            rc = dm_rs_create(c, data_shards, parity_shards, &r);
            if (rc != DM_OK) {
                t_batcher_err = std::string("dm_batcher_create: ") + dm_last_error(c);
                dm_batcher_destroy(b);
                return rc;
            }
            b->coders.push_back(r);
        }
    }
    // default budget: half of what K1Q keeps resident (four 37 KiB workgroups x 8 leaves per CU),
    // so two slots' batches fit side by side
    b->q.reset(new dm_batch::Queue(ns, max_leaves ? max_leaves : 4096, max_bytes ? max_bytes : (16ull << 30),
                                   (double)linger_us, dm_plan::chain_ns_per_block(dm_plan::kQuad)));
    for (int i = 0; i < ns; i++) b->workers.emplace_back(batcher_worker, b, (size_t)i);
    *out = b;
    return DM_OK;
}

int dm_batcher_root(dm_batcher* b, const void* host, uint64_t len, uint8_t* leaf_out, uint8_t root[32]) {
    if (!b || !root || (!host && len) || b->mode != DM_BATCH_ROOT) {
        t_batcher_err = "dm_batcher_root: bad argument or not a ROOT batcher";
        return DM_ERR_INVALID;
    }
    if (len == 0) {
        t_batcher_err = "Empty data";
        return DM_ERR_EMPTY;
    }
    BatchReq r;
    r.host = host;
    r.len = len;
    r.leaves = ceil_div(len, b->unit);
    r.bytes = len;
    r.chain_bytes = std::min(len, b->unit);
    r.out32 = root;
    r.leaf_out = leaf_out;
    return batcher_submit(b, r);
}

int dm_batcher_process(dm_batcher* b, const void* host, uint64_t len, void* frags_out, uint8_t* seg_hashes,
                       uint8_t* frag_hashes, uint8_t fid[32]) {
    if (!b || !fid || (!host && len) || b->mode != DM_BATCH_PROCESS) {
        t_batcher_err = "dm_batcher_process: bad argument or not a PROCESS batcher";
        return DM_ERR_INVALID;
    }
    if (len == 0) {
        t_batcher_err = "Empty data";
        return DM_ERR_EMPTY;
    }
    BatchReq r;
    r.host = host;
    r.len = len;
    r.leaves = ceil_div(len, b->unit) * (1 + (uint64_t)(b->k + b->m));
    r.bytes = ceil_div(len, b->unit) * b->unit * 3;   // segments + parity in device memory
    r.chain_bytes = b->unit;                          // every segment is one full chain
    r.out32 = fid;
    r.frags_out = frags_out;
    r.seg_hashes = seg_hashes;
    r.frag_hashes = frag_hashes;
    return batcher_submit(b, r);
}

int dm_batcher_stats(dm_batcher* b, uint64_t* requests, uint64_t* batches, uint64_t* max_batch) {
    if (!b) return DM_ERR_INVALID;
    const dm_batch::Stats st = b->q->stats();
    if (requests) *requests = st.requests;
    if (batches) *batches = st.batches;
    if (max_batch) *max_batch = st.max_batch;
    return DM_OK;
}

const char* dm_batcher_last_error(void) { return t_batcher_err.c_str(); }

}  // extern "C"
