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

#include <chrono>
#include <condition_variable>
#include <deque>

namespace {

struct BatchReq {
    const void* host = nullptr;
    uint64_t len = 0;
    uint64_t leaves = 0;            // leaves this request adds to a batch
    uint8_t* out32 = nullptr;       // root (ROOT) or fid (PROCESS)
    uint8_t* leaf_out = nullptr;    // ROOT: leaf digests (nullable)
    void* frags_out = nullptr;      // PROCESS (nullable)
    uint8_t* seg_hashes = nullptr;  // PROCESS (nullable)
    uint8_t* frag_hashes = nullptr; // PROCESS (nullable)
    int rc = DM_OK;
    std::string err;
    bool done = false;
    std::chrono::steady_clock::time_point arrived{};
};

thread_local std::string t_batcher_err;

}  // namespace

struct dm_batcher {
    int mode = DM_BATCH_ROOT;
    uint64_t unit = 0;
    int k = 0, m = 0;
    uint64_t max_leaves = 0, max_bytes = 0;
    uint32_t linger_us = 0;
    std::vector<dm_ctx*> ctxs;
    std::vector<dm_rs*> coders;
    std::vector<std::thread> workers;
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::deque<BatchReq*> q;
    uint64_t q_leaves = 0;   // leaves queued
    int busy = 0;            // slots running a batch
    int nslots = 0;          // worker slots (set before any worker starts)
    bool stop = false;
    uint64_t n_req = 0, n_batch = 0, max_batch = 0;
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
    for (;;) {
        std::vector<BatchReq*> batch;
        {
            std::unique_lock<std::mutex> lk(b->mu);
            b->cv_work.wait(lk, [&] { return b->stop || !b->q.empty(); });
            if (b->q.empty()) return;   // stop requested and nothing left to drain
            // let a burst accumulate before launching (dm_plan::batch_linger_us), re-evaluated
            // whenever a slot frees up or the queue fills a batch
            while (!b->stop && !b->q.empty() && b->q_leaves < b->max_leaves) {
                double chain_us = 0;
                if (b->busy > 0) {
                    uint64_t longest = 0;
                    for (const BatchReq* r : b->q)
                        longest = std::max(longest, b->mode == DM_BATCH_PROCESS ? b->unit : std::min(r->len, b->unit));
                    chain_us = (double)ceil_div(longest + 9, 64) * dm_plan::chain_ns_per_block(dm_plan::kQuad) * 1e-3;
                }
                const double w = dm_plan::batch_linger_us(b->linger_us, chain_us, b->busy, b->nslots);
                const auto until = b->q.front()->arrived + std::chrono::microseconds((int64_t)w);
                if (std::chrono::steady_clock::now() >= until) break;
                const int busy0 = b->busy;
                b->cv_work.wait_until(lk, until, [&] {
                    return b->stop || b->q.empty() || b->q_leaves >= b->max_leaves || b->busy != busy0;
                });
            }
            if (b->q.empty()) continue;    // another slot took them meanwhile
            uint64_t leaves = 0, bytes = 0;
            while (!b->q.empty()) {
                BatchReq* r = b->q.front();
                const uint64_t rb = b->mode == DM_BATCH_PROCESS ? ceil_div(r->len, b->unit) * b->unit * 3 : r->len;
                if (!batch.empty() && (leaves + r->leaves > b->max_leaves || bytes + rb > b->max_bytes)) break;
                batch.push_back(r);
                leaves += r->leaves;
                bytes += rb;
                b->q_leaves -= r->leaves;
                b->q.pop_front();
            }
            b->busy++;
            b->n_batch++;
            b->max_batch = std::max<uint64_t>(b->max_batch, batch.size());
            if (!b->q.empty()) b->cv_work.notify_one();   // another slot can start on the rest
        }
        const int rc = b->mode == DM_BATCH_PROCESS ? batch_process_host(b->coders[slot], batch, b->unit)
                                                   : batch_roots_host(c, batch, b->unit);
        const std::string msg = rc == DM_OK ? std::string() : c->err;
        {
            std::lock_guard<std::mutex> lk(b->mu);
            b->busy--;
            for (BatchReq* r : batch) {
                r->rc = rc;
                r->err = msg;
                r->done = true;
            }
        }
        b->cv_done.notify_all();
        b->cv_work.notify_all();   // a lingering slot re-evaluates with one busy slot fewer
    }
}

int batcher_submit(dm_batcher* b, BatchReq& r) {
    {
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->stop) {
            t_batcher_err = "batcher is shutting down";
            return DM_ERR_INVALID;
        }
        r.arrived = std::chrono::steady_clock::now();
        b->q.push_back(&r);
        b->q_leaves += r.leaves;
        b->n_req++;
    }
    b->cv_work.notify_all();   // idle slots start; a lingering one re-checks the leaf budget
    std::unique_lock<std::mutex> lk(b->mu);
    b->cv_done.wait(lk, [&] { return r.done; });
    t_batcher_err = r.err;
    return r.rc;
}

}  // namespace

extern "C" {

void dm_batcher_destroy(dm_batcher* b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
    }
    b->cv_work.notify_all();
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
    // default budget: half of what K1Q keeps resident (four 37 KiB workgroups x 8 leaves per CU),
    // so two slots' batches fit side by side
    b->max_leaves = max_leaves ? max_leaves : 4096;
    b->max_bytes = max_bytes ? max_bytes : (16ull << 30);
    b->linger_us = linger_us;
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
    b->nslots = ns;
    b->workers.reserve(ns);
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
    r.out32 = fid;
    r.frags_out = frags_out;
    r.seg_hashes = seg_hashes;
    r.frag_hashes = frag_hashes;
    return batcher_submit(b, r);
}

int dm_batcher_stats(dm_batcher* b, uint64_t* requests, uint64_t* batches, uint64_t* max_batch) {
    if (!b) return DM_ERR_INVALID;
    std::lock_guard<std::mutex> lk(b->mu);
    if (requests) *requests = b->n_req;
    if (batches) *batches = b->n_batch;
    if (max_batch) *max_batch = b->max_batch;
    return DM_OK;
}

const char* dm_batcher_last_error(void) { return t_batcher_err.c_str(); }

}  // extern "C"
