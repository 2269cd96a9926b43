// merkle_capi.hip -- host runtime and C ABI (include/deoss_merkle.h) of the MI355X Merkle path.
//
// Replaces, behind a C ABI, DeOSS common/hashtree (common/hashtree/types.go:19-39,
// common/hashtree/hashtree.go:18-35) and the tree construction of cbergoon/merkletree v0.2.0
// (go.mod:10).  Every entry point returns an error code; there is no CPU fallback: a missing
// or failing GPU is reported as DM_ERR_NODEV / DM_ERR_HIP.
//
// Layout of one call (single device):
//   object bytes in HBM --K1 leaf_kernel (SHA-256 per chunk, first <=8 levels fused in LDS)-->
//   level-L nodes --K2 reduce_kernel (<=9 levels per launch)--> ... --> 32-byte root.
// Multi-device (one process, ndev > 1): aligned chunk ranges per device, per-device subtree
// roots, one RCCL all-gather of the 32-byte roots, final levels on the first device.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cerrno>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "deoss_merkle.h"
#include "merkle_kernels.hpp"
#include "copy_pool.hpp"
#include "shard_plan.hpp"

namespace {

constexpr uint64_t kAlign = 256;                    // leaf start alignment when packing chunks
constexpr uint64_t kStageBytes = 64ull << 20;       // pinned staging slot
constexpr uint64_t kStripeBudget = 256ull << 20;    // bytes per H2D stripe / batch (e2e path)
constexpr int kMaxLanes = 8;                        // call lanes per GPU (dm_create_lanes)
constexpr uint64_t kLaneKeepBytes = 16ull << 30;    // object buffer a lane keeps between calls (a batcher batch fits)

uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
uint64_t round_up(uint64_t a, uint64_t b) { return ceil_div(a, b) * b; }
uint32_t ceil_log2(uint64_t n) {
    uint32_t d = 0;
    while ((1ull << d) < n) d++;
    return d;
}
uint64_t ceil_shift(uint64_t n, uint32_t k) { return k >= 64 ? (n ? 1 : 0) : (n + (1ull << k) - 1) >> k; }

struct Reaper;
void reaper_put(Reaper* r, int dev, void* p, bool pinned);
void reaper_drain(Reaper* r);

// Device memory an allocation leaves free for the HIP runtime and everything else (dev_alloc).
constexpr size_t kMallocHeadroom = 256ull << 20;

// Free / total memory of device `dev` (the current device when dev < 0), whatever device the
// calling thread has current; false (and the error cleared) when the query fails.
inline bool free_on(int dev, size_t* fr, size_t* tot) {
    int cur = -1;
    if (dev >= 0 && (hipGetDevice(&cur) != hipSuccess || cur != dev)) {
        if (hipSetDevice(dev) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
    } else {
        cur = -1;   // already current: nothing to restore
    }
    const bool ok = hipMemGetInfo(fr, tot) == hipSuccess;
    if (!ok) (void)hipGetLastError();
    if (cur >= 0) (void)hipSetDevice(cur);
    return ok;
}

inline int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) {
        (void)hipGetLastError();
        d = 0;
    }
    return d;
}

// The process's one allocator: every hipMalloc / hipFree of device memory this library makes
// (DevBuf growth and release, the reapers' deferred frees, every context's) runs under its HIP
// device's mutex, and every hipHostMalloc / hipHostFree under the host mutex.  Round 4 saw four
// segfaults inside the HSA runtime (pthread_mutex_lock under hipMalloc) when a DevBuf growth ran
// out of memory while a reaper's hipFree of a large block was still pending behind a running
// chain.  A round-5 probe separated the conditions (profiles/r05/LOGS.md#oom_free_race.log);
// whatever its verdict,
// under these locks the library never has a hipMalloc in flight beside one of its own hipFrees on
// that device, and dev_alloc never issues a hipMalloc that hipMemGetInfo says cannot succeed --
// not on the first try and not on the retry after a reaper drain.  The cost: an allocation waits
// behind a reaper free of the same device, which waits for the device's queued work (growth only;
// steady-state calls reuse their buffers and allocate nothing).
struct AllocLocks {
    static constexpr int kDevs = 64;
    std::mutex dev[kDevs];
    std::mutex host;
};
AllocLocks& alloc_locks() {
    static AllocLocks* a = new AllocLocks();   // never destroyed: reapers may free during exit
    return *a;
}
std::mutex& dev_mutex(int dev) { return alloc_locks().dev[(unsigned)dev % AllocLocks::kDevs]; }

// hipMalloc(n) on device `dev` (current on the calling thread), or hipErrorOutOfMemory without
// calling hipMalloc when less than n + kMallocHeadroom is free.  DM_ALLOC_PRECHECK=0 builds an A/B
// variant without the free-memory check (the lock alone), never the shipped library.
#ifndef DM_ALLOC_PRECHECK
#define DM_ALLOC_PRECHECK 1
#endif
hipError_t dev_alloc(int dev, void** p, size_t n) {
    *p = nullptr;
    std::lock_guard<std::mutex> lk(dev_mutex(dev));
    size_t fr = 0, tot = 0;
    if (DM_ALLOC_PRECHECK && free_on(dev, &fr, &tot) && fr < n + kMallocHeadroom) return hipErrorOutOfMemory;
    hipError_t e = hipMalloc(p, n);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
    }
    return e;
}

void dev_release(int dev, void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(dev_mutex(dev));
    (void)hipFree(p);   // waits for the device's queued work
    (void)hipGetLastError();
}

hipError_t host_alloc(void** p, size_t n, unsigned flags) {
    *p = nullptr;
    std::lock_guard<std::mutex> lk(alloc_locks().host);
    hipError_t e = hipHostMalloc(p, n, flags);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
    }
    return e;
}

void host_release(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(alloc_locks().host);
    (void)hipHostFree(p);
    (void)hipGetLastError();
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    Reaper* rp = nullptr;   // set (context scratch): growth hands the old buffer to the context's reaper
    int dev = -1;           // HIP device (-1: the device current at each ensure / release)
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        const int id = dev >= 0 ? dev : current_device();
        if (p) {
            if (rp) {   // freed once the work queued so far has finished; this caller does not wait
                reaper_put(rp, id, p, false);
            } else {
                hipError_t e = hipDeviceSynchronize();   // scratch may still be in use by queued work
                if (e != hipSuccess) return e;
                dev_release(id, p);
            }
            p = nullptr;
            cap = 0;
        }
        const size_t c = round_up(std::max<size_t>(n, 4096), 2ull << 20);
        hipError_t e = dev_alloc(id, &p, c);
        if (e == hipErrorOutOfMemory && rp) {
            // the memory this growth needs may still sit in the reaper's queue (this buffer's old
            // block among it, freed only once every stream of the device has drained): wait for
            // those frees, then try once more -- dev_alloc checks free memory again first
            reaper_drain(rp);
            e = dev_alloc(id, &p, c);
        }
        if (e != hipSuccess) return e;
        cap = c;
        return hipSuccess;
    }
    uint8_t* u8() { return static_cast<uint8_t*>(p); }
    void release() {
        dev_release(dev >= 0 ? dev : current_device(), p);
        p = nullptr;
        cap = 0;
    }
};

struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        host_release(p);
        p = nullptr;
        cap = 0;
        hipError_t e = host_alloc(&p, n, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        cap = n;
        return hipSuccess;
    }
    uint8_t* u8() { return static_cast<uint8_t*>(p); }
    void release() {
        host_release(p);
        p = nullptr;
        cap = 0;
    }
};

// Deferred release.  hipFree, hipFreeAsync and hipHostFree wait for ALL work queued on the device
// (profiles/r03/LOGS.md#free_sync_probe.log: ~280 ms behind an unrelated 300 ms
// kernel on another stream; hipMalloc and event calls do not wait).  So buffers a call no longer
// needs go to the context's reaper thread, which frees them in order: the caller never waits for
// other callers' kernels.  The same device-wide wait makes it safe: every use of a buffer was
// queued before the buffer was handed over.
struct Reaper {
    std::mutex mu;
    std::condition_variable cv;
    struct Item {
        int dev;
        void* p;
        bool pinned;
    };
    std::deque<Item> q;
    bool stop = false;
    int active = 0;                   // items popped but not yet freed
    std::condition_variable idle;     // q empty and nothing being freed (drain)
    std::thread th;
    void put(int dev, void* p, bool pinned) {
        if (!p) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back({dev, p, pinned});
            if (!th.joinable()) th = std::thread([this] { run(); });
        }
        cv.notify_one();
    }
    void put(int dev, DevBuf& b) {
        put(dev, b.p, false);
        b.p = nullptr;
        b.cap = 0;
    }
    void put(int dev, PinnedBuf& b) {
        put(dev, b.p, true);
        b.p = nullptr;
        b.cap = 0;
    }
    void run() {
        for (;;) {
            Item it;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;   // stop requested and drained
                it = q.front();
                q.pop_front();
                active++;
            }
            // hipFree resolves the allocation from the pointer; a failed hipSetDevice must not leak it
            (void)hipSetDevice(it.dev);
            (void)hipGetLastError();
            if (it.pinned) host_release(it.p);
            else dev_release(it.dev, it.p);
            {
                std::lock_guard<std::mutex> lk(mu);
                active--;
            }
            idle.notify_all();
        }
    }
    // Block until everything queued so far has been freed (an allocation that failed for lack of
    // memory retries after this).  Each free goes through dev_release / host_release: it takes that
    // device's allocation mutex (or the host one) and holds it across a hipFree / hipHostFree that
    // waits for the device's queued work, so meanwhile every allocation on that device (for a host
    // free: every pinned allocation of the process) waits too.  Deadlock-free because those mutexes
    // are leaves: no code holds a device or host allocation mutex while calling reaper_drain or
    // taking any other library lock (DevBuf::ensure drains the reaper between two dev_alloc calls,
    // holding neither mutex).
    void drain() {
        std::unique_lock<std::mutex> lk(mu);
        idle.wait(lk, [&] { return q.empty() && active == 0; });
    }
    void finish() {   // free everything queued, then end the thread (dm_destroy)
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_one();
        if (th.joinable()) th.join();
    }
    ~Reaper() { finish(); }
};

void reaper_put(Reaper* r, int dev, void* p, bool pinned) { r->put(dev, p, pinned); }
void reaper_drain(Reaper* r) { r->drain(); }

void par_copy(const std::vector<dm_copy::CopyItem>& items) { dm_copy::CopyPool::get().run(items); }

// The HIP resources of one streaming upload (dm_stream / dm_pstream), pooled per device and reused
// by the next stream: creating streams and pinning staging costs ~10 ms per object
// (profiles/r03/LOGS.md#free_sync_probe.log), and destroying / unpinning waits for the whole device.
struct StreamKit {
    static constexpr int kEvents = 10, kSlots = 4;
    hipStream_t copy = nullptr;          // high priority: staging reuse never waits behind leaf kernels
    hipStream_t code = nullptr, comp[2] = {nullptr, nullptr};
    hipEvent_t ev[kEvents] = {};
    PinnedBuf slot[kSlots];              // staging slots, pinned on first use
    PinnedBuf tabs;                      // pinned arena for per-launch leaf tables
    uint64_t tabs_used = 0;
};

struct Dev {
    int id = 0;
    int cus = 256;                      // compute units (leaf-kernel choice)
    hipStream_t stream = nullptr;       // compute stream
    hipStream_t copy = nullptr;         // H2D stream
    DevBuf data, nodes_a, nodes_b, leaves, tab_addr, tab_len, tab_first, tab_ids, root, gather;
    DevBuf proof_paths, proof_bits, proof_roots;   // host-API proof staging (tree_capi.inl)
    PinnedBuf stage[2];
    PinnedBuf htab;                     // pinned bounce buffer for per-call index tables
    uint64_t htab_used = 0;
    hipEvent_t ev_done = nullptr;
    hipEvent_t ev_copy[2] = {nullptr, nullptr}, ev_step[2] = {nullptr, nullptr}, ev_htab = nullptr;
    bool has_last = false;              // the lane has run a call (ev_tail is recorded)
    // end of the lane's last call on the GPU (recorded when its lock is released): an async call's
    // kernels outlive its lock, so routing counts a lane whose tail has not completed as busy
    hipEvent_t ev_tail = nullptr;
    hipStream_t tail_stream = nullptr;  // set by begin_call, recorded into ev_tail at unlock
    uint64_t keep_bytes = kLaneKeepBytes;   // object buffer kept between calls (test hook: DEOSS_LANE_KEEP_BYTES)
    // timing records: (K1 begin, K1 end, call end) per timed call, reused across resets
    std::vector<hipEvent_t> tev;
    size_t ntimed = 0;
};

}  // namespace

// Per-device call state of a context: the lock a call holds on the device it runs on, and the
// device's load (calls running or waiting on it, plus open streams) for least-busy routing.
struct DevSlot {
    std::mutex mu;
    std::atomic<int> load{0};
    std::mutex kit_mu;
    std::vector<StreamKit*> kits;          // idle stream kits of this device
};

inline uint64_t next_ctx_serial() {
    static std::atomic<uint64_t> n{0};
    return ++n;
}

struct dm_ctx {
    // Call lanes: devs holds `lanes` entries per GPU, lane-major (devs[l * nphys + p] is lane l of
    // GPU p), each with its own streams, scratch and lock, so up to `lanes` calls run on one GPU at
    // once (an 8 GiB object at 32 MiB chunks keeps 32 of 256 CUs busy for its whole chain).  Lane 0
    // of every GPU comes first, so a sharded call over G' GPUs locks and uses devs [0, G').
    std::vector<Dev> devs;
    int nphys = 1;                         // GPUs (distinct devices) of the context
    int lanes = 1;                         // call lanes per GPU (DEOSS_LANES, dm_create_lanes)
    std::unique_ptr<DevSlot[]> slots;      // one per lane (absent in private error-sink contexts)
    std::atomic<uint32_t> rr{0};           // round-robin start of the least-busy scan
    std::mutex route_mu;                   // a lane choice and its reservation are one step
    std::mutex comm_mu;
    std::map<int, std::vector<ncclComm_t>> comms;   // RCCL communicators over devices [0, G'), by G'
    std::mutex err_mu;
    std::string err;
    Reaper reaper;                         // deferred hipFree / hipHostFree (never in a caller's path)
    bool timing = false;                   // written with every device locked
    std::atomic<int> leaf_mode{DM_LEAF_AUTO};
    // Test hook (env DEOSS_FORCE_SHARDED=1 at dm_create): run host-memory objects through the
    // multi-device path (partition, RCCL all-gather, compaction, finish) even with one device.
    bool force_sharded = false;
    // The routing model's all-gather and host-bandwidth terms: estimates, or the values an N = 8
    // bench line measured, from DEOSS_ALLGATHER_US / DEOSS_HOST_BYTES_PER_S at dm_create.
    dm_plan::RouteConstants route_k;
    // Test hook (env DEOSS_TEST_RCCL_INIT_FAIL=1 at dm_create of a multi-device context that is not
    // forced sharded): comms_for fails the way a failing ncclCommInitAll does, just before calling
    // it, so dm_create's degraded path runs end to end on one GPU (virtual devices otherwise never
    // build communicators).
    bool fail_comm_init = false;
    // Test hook (env DEOSS_VIRTUAL_DEVICES=N at dm_create): N context devices on the first GPU, each
    // with its own streams, scratch and lock, so routing, range locks, multi_root's partition and
    // compaction and the batch split run with G = N on a one-GPU box.  RCCL rejects duplicate
    // GPUs, so the gather of subtree roots is then a D2D copy to device 0 (real GPUs: RCCL).
    bool virtual_devs = false;
    // false when ncclCommInitAll failed at dm_create on an unforced multi-GPU context: every call
    // then runs whole on one GPU (routing never shards an object; batches still split by objects,
    // which needs no exchange) instead of the context failing outright.
    bool shard_ok = true;
    // process-unique, never reused (dm_last_call_devices' thread-local record names it)
    const uint64_t serial = next_ctx_serial();
    bool keep_claimed = false;             // its lanes' keep bytes count in g_keep_claimed (dm_create)
    // Exchange timing of multi-device calls while timing is on (dm_exchange_timing): host clock
    // from every device's subtree roots being ready to the gathered slots being on every device.
    std::mutex xmu;
    uint64_t x_n = 0;
    double x_sum_us = 0, x_max_us = 0;
    int x_last_G = 0;
};

namespace {

// Detailed message of the calling thread's last failing call (dm_last_error).  Thread-local, so a
// reader never races another thread's failure (Go: runtime.LockOSThread around call + read), and
// every error return below sets it, so it is never a stale message from an older call.
thread_local std::string t_err;

int set_err(int code, const char* msg) {
    t_err = msg;
    return code;
}

int bad_arg() { return set_err(DM_ERR_INVALID, "invalid argument"); }

// Where the calling thread's last lane-holding call ran (dm_last_call_devices): context device
// indices (one for a whole call, [0, G) for a call sharded over G GPUs) and the lane.
thread_local std::vector<int> t_call_devs;
thread_local int t_call_lane = -1;
// the context is named by its serial (dm_ctx::serial), not its address: a context created where a
// destroyed one lived must not see that one's last call
thread_local uint64_t t_call_ctx = 0;

void note_call(const dm_ctx* c, int g, int G) {
    t_call_ctx = c->serial;
    t_call_devs.clear();
    if (G == 1) {
        t_call_devs.push_back(g % c->nphys);
        t_call_lane = g / c->nphys;
    } else {
        for (int i = 0; i < G; i++) t_call_devs.push_back(i);
        t_call_lane = 0;
    }
}

int fail(dm_ctx* c, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) {
        std::lock_guard<std::mutex> lk(c->err_mu);
        c->err = buf;
    }
    t_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(c, e_ == hipErrorOutOfMemory ? DM_ERR_NOMEM : DM_ERR_HIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                    \
    } while (0)

#define RC_TRY(expr)                 \
    do {                             \
        int rc_ = (expr);            \
        if (rc_ != DM_OK) return rc_; \
    } while (0)

#define NCCL_TRY(expr)                                                                         \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess)                                                                 \
            return fail(c, DM_ERR_RCCL, "%s: %s", #expr, ncclGetErrorString(r_));              \
    } while (0)

// *_async calls run on the caller's stream verbatim: NULL is HIP's null (legacy default) stream,
// which is also what torch's default stream handle (0) denotes.
hipStream_t pick_stream(Dev&, void* s) { return static_cast<hipStream_t>(s); }

// Every entry point leaves the calling thread's current HIP device as it found it: the library
// switches devices per call, and a caller's own device (torch's, a Go thread's) must not move.
struct DeviceRestore {
    int prev = -1;
    DeviceRestore() {
        if (hipGetDevice(&prev) != hipSuccess) {
            prev = -1;
            (void)hipGetLastError();
        }
    }
    ~DeviceRestore() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceRestore(const DeviceRestore&) = delete;
    DeviceRestore& operator=(const DeviceRestore&) = delete;
};

// The lane's tail: its last call's work ends with this event (begin_call set tail_stream; the
// caller holds the lane's lock).  Then the lane's object buffer is trimmed: a lane keeps at most
// kLaneKeepBytes of it between calls (a larger one goes to the reaper, whose hipFree waits for the
// work still using it), so a context's idle HBM does not scale with its lanes x its largest object.
void record_tail(Dev& d) {
    if (!d.tail_stream) return;
    if (hipSetDevice(d.id) == hipSuccess) (void)hipEventRecord(d.ev_tail, d.tail_stream);
    (void)hipGetLastError();
    d.tail_stream = nullptr;
    if (d.data.cap > d.keep_bytes && d.data.rp) {
        reaper_put(d.data.rp, d.data.dev, d.data.p, false);
        d.data.p = nullptr;
        d.data.cap = 0;
    }
}

// An entry point's hold on ONE lane of its context for the whole call (that lane's scratch,
// streams and staging), and the caller's device restored after.  Calls on different lanes of one
// context run concurrently; a thread holds at most one CallLock.
constexpr bool kReserved = true;   // CallLock on a lane that pick_device / device_of already counted
struct CallLock {
    DeviceRestore dev;
    Dev* d;
    DevSlot* slot;
    std::unique_lock<std::mutex> lk;
    CallLock(dm_ctx* c, int g, bool reserved = false) : d(&c->devs[g]), slot(&c->slots[g]) {
        if (!reserved) slot->load++;
        lk = std::unique_lock<std::mutex>(slot->mu);
        note_call(c, g, 1);
    }
    ~CallLock() {
        record_tail(*d);
        lk.unlock();
        slot->load--;
    }
    CallLock(const CallLock&) = delete;
    CallLock& operator=(const CallLock&) = delete;
};

// Lanes [0, G) of a context, locked in index order (so two of these cannot deadlock): sharded
// calls (G = the GPUs they use: lane 0 of each) and context-wide settings (G = every lane).
struct RangeLock {
    DeviceRestore dev;
    dm_ctx* c;
    int G;
    std::vector<std::unique_lock<std::mutex>> lks;
    // lanes [0, G): lane 0 of the first G GPUs, for a call sharded over them
    RangeLock(dm_ctx* c_, int G_) : RangeLock(c_, G_, true) {}
    // every lane: context-wide settings (not a call: dm_last_call_devices keeps the last call)
    explicit RangeLock(dm_ctx* c_) : RangeLock(c_, (int)c_->devs.size(), false) {}
    RangeLock(dm_ctx* c_, int G_, bool is_call) : c(c_), G(G_) {
        for (int g = 0; g < G; g++) c->slots[g].load++;
        for (int g = 0; g < G; g++) lks.emplace_back(c->slots[g].mu);
        if (is_call) note_call(c, 0, G);
    }
    ~RangeLock() {
        for (int g = 0; g < G; g++) record_tail(c->devs[g]);
        for (auto& l : lks) l.unlock();
        for (int g = 0; g < G; g++) c->slots[g].load--;
    }
    RangeLock(const RangeLock&) = delete;
    RangeLock& operator=(const RangeLock&) = delete;
};

// The lane loads of a context, lane-major (dm_plan::pick_lane's layout); caller holds route_mu.
std::vector<int> lane_loads(dm_ctx* c) {
    std::vector<int> v(c->devs.size());
    for (size_t i = 0; i < v.size(); i++) v[i] = c->slots[i].load.load();
    return v;
}

// Lane choice, counted in the lane's load before return (the caller's CallLock(..., kReserved) or
// stream releases it): dm_plan::pick_lane over the calls running or queued per lane, GPU first
// (least total load, ties round-robin from `start`), then within that GPU the lanes whose last
// call's GPU work has not finished count one more (an async call's kernels outlive its lock, so
// a second async caller goes to an idle lane instead of queueing behind them).  phys >= 0 fixes
// the GPU.  Caller holds route_mu.
int choose_lane(dm_ctx* c, int start, int phys) {
    std::vector<int> v = lane_loads(c);
    int g = dm_plan::pick_lane(v.data(), c->nphys, c->lanes, start, phys);
    if (c->lanes > 1) {
        const int p = g % c->nphys;
        for (int l = 0; l < c->lanes; l++) {
            const int i = l * c->nphys + p;
            if (c->devs[i].ev_tail && hipEventQuery(c->devs[i].ev_tail) == hipErrorNotReady) v[i]++;
        }
        (void)hipGetLastError();
        g = dm_plan::pick_lane(v.data(), c->nphys, c->lanes, start, p);
    }
    c->slots[g].load++;
    return g;
}

int pick_device(dm_ctx* c) {
    std::lock_guard<std::mutex> lk(c->route_mu);
    const int start = c->nphys > 1 ? (int)(c->rr.fetch_add(1) % (uint32_t)c->nphys) : 0;
    return choose_lane(c, start, -1);
}

// Calls already running or queued on the context (routing: a busy context never shards).
int ctx_load(const dm_ctx* c) {
    int s = 0;
    for (size_t g = 0; g < c->devs.size(); g++) s += c->slots[g].load.load();
    return s;
}

void kit_destroy(StreamKit* k) {
    for (hipStream_t s : {k->copy, k->code, k->comp[0], k->comp[1]})
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    for (hipEvent_t e : k->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& b : k->slot) b.release();
    k->tabs.release();
    delete k;
}

// A stream kit of device g (the caller has made g current): an idle one from the pool, else new.
int kit_acquire(dm_ctx* c, int g, StreamKit** out) {
    *out = nullptr;
    DevSlot& sl = c->slots[g];
    {
        std::lock_guard<std::mutex> lk(sl.kit_mu);
        if (!sl.kits.empty()) {
            *out = sl.kits.back();
            sl.kits.pop_back();
            (*out)->tabs_used = 0;
            return DM_OK;
        }
    }
    StreamKit* k = new StreamKit();
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipError_t e = hipStreamCreateWithPriority(&k->copy, hipStreamNonBlocking, hi);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&k->code, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&k->comp[0], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&k->comp[1], hipStreamNonBlocking);
    for (int i = 0; i < StreamKit::kEvents && e == hipSuccess; i++)
        e = hipEventCreateWithFlags(&k->ev[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        kit_destroy(k);
        return fail(c, DM_ERR_HIP, "stream kit: %s", hipGetErrorString(e));
    }
    *out = k;
    return DM_OK;
}

// Back to device g's pool; the caller has synchronised the kit's streams (its own work only).
void kit_release(dm_ctx* c, int g, StreamKit* k) {
    if (!k) return;
    DevSlot& sl = c->slots[g];
    std::lock_guard<std::mutex> lk(sl.kit_mu);
    sl.kits.push_back(k);
}

// `bytes` of the kit's pinned table arena (leaf tables uploaded by later H2D copies).  A full
// arena is replaced, and the old one goes to the reaper: copies still queued may read it.
uint8_t* kit_table(dm_ctx* c, int dev, StreamKit* k, uint64_t bytes) {
    bytes = round_up(std::max<uint64_t>(bytes, 1), 256);
    if (k->tabs_used + bytes > k->tabs.cap) {
        const uint64_t want = std::max<uint64_t>({bytes, 2 * k->tabs.cap, 1ull << 20});
        c->reaper.put(dev, k->tabs);
        if (k->tabs.ensure(want) != hipSuccess) return nullptr;
        k->tabs_used = 0;
    }
    uint8_t* p = k->tabs.u8() + k->tabs_used;
    k->tabs_used += bytes;
    return p;
}

// Grow a pinned buffer to n bytes without waiting on the device: the old one goes to the reaper.
// Both attempts go through host_alloc (under the host allocation lock).
hipError_t pinned_grow(dm_ctx* c, int dev, PinnedBuf& b, uint64_t n) {
    if (n <= b.cap) return hipSuccess;
    c->reaper.put(dev, b);
    hipError_t e = b.ensure(n);
    if (e == hipErrorOutOfMemory) {   // the old buffer may still be queued: free it, retry once
        c->reaper.drain();
        e = b.ensure(n);
    }
    return e;
}

// Lane for a device-memory call (device-resident entry points run where their data lives), counted
// like pick_device: the least-loaded lane of the GPU holding p, or of the first GPU when p is not
// device memory of one of the context's GPUs.
int device_of(dm_ctx* c, const void* p) {
    int phys = 0;
    if (c->nphys > 1 && p) {
        hipPointerAttribute_t attr{};
        if (hipPointerGetAttributes(&attr, p) == hipSuccess)
            for (int i = 0; i < c->nphys; i++)
                if (c->devs[i].id == attr.device) {
                    phys = i;
                    break;
                }
        (void)hipGetLastError();
    }
    std::lock_guard<std::mutex> lk(c->route_mu);
    return choose_lane(c, 0, phys);
}

// Order this call's use of the context scratch after the previous call's (possibly other stream).
int begin_call(dm_ctx* c, Dev& d, hipStream_t s) {
    HIP_TRY(hipSetDevice(d.id));
    // after the lane's previous call: wait for its tail event (recorded when its lock was
    // released), never for the old stream itself, which its caller may have destroyed since.
    // Always, even when s compares equal to the last stream: a caller may have destroyed that
    // stream and created a new one at the same address while the old one's kernels (which use
    // this lane's scratch) still run; the wait is near-free on a completed event.
    if (d.has_last) HIP_TRY(hipStreamWaitEvent(s, d.ev_tail, 0));
    d.has_last = true;
    d.tail_stream = s;
    return DM_OK;
}

bool is_aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Next timing record (3 events) of device d; nullptr when timing is off.
hipEvent_t* timing_record(dm_ctx* c, Dev& d) {
    if (!c->timing) return nullptr;
    const size_t need = 3 * (d.ntimed + 1);
    while (d.tev.size() < need) {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        d.tev.push_back(e);
    }
    return &d.tev[3 * d.ntimed++];
}

// Start a call's table uploads: wait until the previous call's uploads have left the bounce buffer.
int tables_begin(dm_ctx* c, Dev& d, uint64_t bytes) {
    HIP_TRY(hipEventSynchronize(d.ev_htab));
    HIP_TRY(d.htab.ensure(std::max<uint64_t>(round_up(bytes, 256) + 4096, 1ull << 20)));
    d.htab_used = 0;
    return DM_OK;
}

// Stream-ordered upload of a host table through the pinned bounce buffer (host memory may be
// released as soon as this returns).
int upload(dm_ctx* c, Dev& d, hipStream_t s, DevBuf& dst, const void* src, uint64_t bytes) {
    HIP_TRY(dst.ensure(std::max<uint64_t>(bytes, 8)));
    if (bytes == 0) return DM_OK;
    if (d.htab_used + bytes > d.htab.cap) return fail(c, DM_ERR_INVALID, "table bounce buffer overflow");
    uint8_t* h = d.htab.u8() + d.htab_used;
    std::memcpy(h, src, bytes);
    d.htab_used = round_up(d.htab_used + bytes, 256);
    HIP_TRY(hipMemcpyAsync(dst.p, h, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(d.ev_htab, s));
    return DM_OK;
}

// K2 stages: reduce m nodes at `in` for exactly D levels (D >= 1) into dst.
int reduce_stages(dm_ctx* c, Dev& d, hipStream_t s, const uint8_t* in, uint64_t m, uint32_t D, uint8_t* dst) {
    std::vector<uint32_t> ks;
    for (uint32_t r = D; r > 0;) {
        uint32_t k = std::min<uint32_t>(9, r);
        ks.push_back(k);
        r -= k;
    }
    HIP_TRY(d.nodes_a.ensure(std::max<uint64_t>(ceil_div(m, 2), 1) * 32));
    HIP_TRY(d.nodes_b.ensure(std::max<uint64_t>(ceil_div(m, 2), 1) * 32));
    const uint8_t* cur = in;
    for (size_t i = 0; i < ks.size(); i++) {
        uint8_t* out = (i + 1 == ks.size()) ? dst : (cur == d.nodes_a.u8() ? d.nodes_b.u8() : d.nodes_a.u8());
        const uint64_t grid = ceil_div(m, dm::kReduceTile);
        hipLaunchKernelGGL(dm::reduce_kernel, dim3((uint32_t)grid), dim3(dm::kBlock), 0, s, cur, m, ks[i], out);
        HIP_TRY(hipGetLastError());
        m = ceil_shift(m, ks[i]);
        cur = out;
    }
    return DM_OK;
}

// Hash the leaves described by `la` (uniform or table mode) and reduce `levels` levels
// (levels < 0: to the root, >= 1 level).  Nodes go to dst; *nout gets their count.
// Leaf-kernel choice for a uniform-chunk object of n leaves: the more lanes a kernel spends per
// leaf, the shorter each leaf's serial chain, as long as its workgroups fit the chip at once.
// Returns DM_LEAF_WIDE, DM_LEAF_LATENCY, DM_LEAF_PAIR or DM_LEAF_QUAD.
// Measured on MI355X (8 GiB object, profiles/r01/LOGS.md#r01_sweep_k1q4.log): K1Q wins up to 8,192 leaves
// (four 37 KiB-LDS workgroups per CU: 345.6 GiB/s at 8,192 leaves vs 274.7 for K1P), K1L up to
// 16,384 (536 vs 397 for K1P, 223 for K1Q in two rounds of workgroups); past that one lane per
// leaf with >= 2 waves per SIMD wins.  K1P stays selectable (DM_LEAF_PAIR).
int pick_leaf_kernel(const dm_ctx* c, const Dev& d, uint64_t n) {
    static_assert(dm_plan::kQuadLeaves == dm::kQuadLeaves && dm_plan::kLatLeaves == dm::kLatLeaves, "plan shapes");
    return dm_plan::leaf_kind(n, d.cus, c->leaf_mode.load());
}

template <bool TABLE, bool ALIGNED>
void launch_leaves_t(hipStream_t s, const dm::LeafArgs& la, int kind, int cus) {
    const uint64_t n = la.nleaves;
    const dim3 qgrid((uint32_t)ceil_div(n, dm::kQuadLeaves));
    if (kind == DM_LEAF_QUAD && qgrid.x > 2 * (uint64_t)cus) {   // > 2 workgroups per CU: compact ring
        hipLaunchKernelGGL(dm::quad_shape_primer, dim3(4 * (uint32_t)cus), dim3(dm::kLatThreads), dm::kQuadLdsBytes, s, 0);
        hipLaunchKernelGGL((dm::leaf_kernel_quad<TABLE, ALIGNED, true>), qgrid, dim3(dm::kLatThreads), 0, s, la);
    }
    else if (kind == DM_LEAF_QUAD)
        hipLaunchKernelGGL((dm::leaf_kernel_quad<TABLE, ALIGNED, false>), qgrid, dim3(dm::kLatThreads), 0, s, la);
    else if (kind == DM_LEAF_PAIR)
        hipLaunchKernelGGL((dm::leaf_kernel_pair<TABLE, ALIGNED>), dim3((uint32_t)ceil_div(n, dm::kPairLeaves)),
                           dim3(dm::kLatThreads), 0, s, la);
    else if (kind == DM_LEAF_LATENCY)
        hipLaunchKernelGGL((dm::leaf_kernel_lat<TABLE, ALIGNED>), dim3((uint32_t)ceil_div(n, dm::kLatLeaves)),
                           dim3(dm::kLatThreads), 0, s, la);
    else
        hipLaunchKernelGGL((dm::leaf_kernel<TABLE, ALIGNED>), dim3((uint32_t)ceil_div(n, dm::kBlock)), dim3(dm::kBlock),
                           0, s, la);
}

// Launch the chosen leaf kernel (K1 / K1L / K1P / K1Q) over la's leaves on device d.
int launch_leaves(dm_ctx* c, const Dev& d, hipStream_t s, const dm::LeafArgs& la, bool table, bool aligned, int kind) {
    if (table) {
        if (aligned) launch_leaves_t<true, true>(s, la, kind, d.cus);
        else launch_leaves_t<true, false>(s, la, kind, d.cus);
    } else {
        if (aligned) launch_leaves_t<false, true>(s, la, kind, d.cus);
        else launch_leaves_t<false, false>(s, la, kind, d.cus);
    }
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int run_tree(dm_ctx* c, Dev& d, hipStream_t s, dm::LeafArgs la, bool table, bool aligned, int levels,
             uint8_t* dst, uint64_t* nout, uint8_t* leaf_dig) {
    const uint64_t n = la.nleaves;
    const int kind = pick_leaf_kernel(c, d, n);
    const uint32_t D = levels < 0 ? std::max<uint32_t>(1, ceil_log2(n)) : (uint32_t)levels;
    const uint32_t fuse_max = kind == DM_LEAF_QUAD ? dm::kQuadFuseMax
                              : kind == DM_LEAF_PAIR ? dm::kPairFuseMax
                              : kind == DM_LEAF_LATENCY ? dm::kLatFuseMax : dm::kLeafFuseMax;
    const uint32_t L1 = std::min<uint32_t>(fuse_max, D);
    const uint64_t m1 = ceil_shift(n, L1);
    la.byte_off = 0;
    la.byte_end = ~0ull;
    la.state = nullptr;
    la.fuse_levels = L1;
    uint8_t* k1_out = dst;
    if (D > L1) {
        HIP_TRY(d.leaves.ensure(m1 * 32));   // level-L1 nodes
        k1_out = d.leaves.u8();
    }
    if (L1 == 0) {
        la.digests = dst;
        la.level_out = nullptr;
    } else {
        la.digests = leaf_dig;
        la.level_out = k1_out;
    }
    hipEvent_t* tr = timing_record(c, d);
    if (tr) HIP_TRY(hipEventRecord(tr[0], s));
    RC_TRY(launch_leaves(c, d, s, la, table, aligned, kind));
    if (tr) HIP_TRY(hipEventRecord(tr[1], s));
    if (L1 == 0 && leaf_dig != nullptr && leaf_dig != dst)
        HIP_TRY(hipMemcpyAsync(leaf_dig, dst, n * 32, hipMemcpyDeviceToDevice, s));
    if (D > L1) RC_TRY(reduce_stages(c, d, s, k1_out, m1, D - L1, dst));
    if (tr) HIP_TRY(hipEventRecord(tr[2], s));
    *nout = ceil_shift(n, D);
    return DM_OK;
}

dm::LeafArgs uniform_args(const void* dev, uint64_t len, uint64_t chunk) {
    dm::LeafArgs la{};
    const uint64_t n = ceil_div(len, chunk);
    la.base = static_cast<const uint8_t*>(dev);
    la.pitch = chunk;
    la.leaf_len = chunk;
    la.last_len = len - (n - 1) * chunk;
    la.nleaves = n;
    return la;
}

// Finish: reduce n nodes to the root (>= 1 level if min_one or n > 1).
int finish(dm_ctx* c, Dev& d, hipStream_t s, const uint8_t* nodes, uint64_t n, bool min_one, uint8_t* dst) {
    uint32_t D = ceil_log2(n);
    if (D == 0 && min_one) D = 1;
    if (D == 0) {
        HIP_TRY(hipMemcpyAsync(dst, nodes, 32, hipMemcpyDeviceToDevice, s));
        return DM_OK;
    }
    return reduce_stages(c, d, s, nodes, n, D, dst);
}

// Batched per-object trees over leaf digests already in d.leaves-like storage.
int batch_roots_from_leaves(dm_ctx* c, Dev& d, hipStream_t s, const uint8_t* leaves,
                            const std::vector<uint64_t>& first, uint8_t* roots) {
    const uint64_t nobj = first.size() - 1;
    std::vector<uint32_t> small;
    small.reserve(nobj);
    for (uint64_t o = 0; o < nobj; o++)
        if (first[o + 1] - first[o] <= (uint64_t)dm::kReduceTile) small.push_back((uint32_t)o);
    if (!small.empty()) {
        RC_TRY(upload(c, d, s, d.tab_first, first.data(), first.size() * 8));
        RC_TRY(upload(c, d, s, d.tab_ids, small.data(), small.size() * 4));
        hipLaunchKernelGGL(dm::batch_root_kernel, dim3((uint32_t)small.size()), dim3(dm::kBlock), 0, s,
                           leaves, static_cast<const uint64_t*>(d.tab_first.p),
                           static_cast<const uint32_t*>(d.tab_ids.p), roots);
        HIP_TRY(hipGetLastError());
    }
    for (uint64_t o = 0; o < nobj; o++) {
        const uint64_t cnt = first[o + 1] - first[o];
        if (cnt <= (uint64_t)dm::kReduceTile) continue;
        RC_TRY(finish(c, d, s, leaves + 32 * first[o], cnt, true, roots + 32 * o));
    }
    return DM_OK;
}

// Leaf hashing of a batch of objects at device addresses + per-object roots.
int batch_device(dm_ctx* c, Dev& d, hipStream_t s, const void* const* objs, const uint64_t* lens, uint64_t nobj,
                 uint64_t chunk, uint8_t* roots, int kind = -1) {
    std::vector<uint64_t> first(nobj + 1, 0);
    for (uint64_t o = 0; o < nobj; o++) {
        if (lens[o] == 0) return fail(c, DM_ERR_EMPTY, "Empty data (object %llu has no bytes)", (unsigned long long)o);
        first[o + 1] = first[o] + ceil_div(lens[o], chunk);
    }
    const uint64_t T = first[nobj];
    std::vector<uint64_t> addr(T), len(T);
    bool aligned = true;
    for (uint64_t o = 0; o < nobj; o++) {
        const uint64_t n = first[o + 1] - first[o];
        for (uint64_t j = 0; j < n; j++) {
            const uint64_t a = reinterpret_cast<uint64_t>(objs[o]) + j * chunk;
            addr[first[o] + j] = a;
            len[first[o] + j] = (j + 1 < n) ? chunk : lens[o] - j * chunk;
            aligned &= (a & 15) == 0;
        }
    }
    RC_TRY(tables_begin(c, d, T * 16 + (nobj + 1) * 12 + 1024));
    HIP_TRY(d.leaves.ensure(T * 32));
    RC_TRY(upload(c, d, s, d.tab_addr, addr.data(), T * 8));
    RC_TRY(upload(c, d, s, d.tab_len, len.data(), T * 8));
    dm::LeafArgs la{};
    la.addrs = static_cast<const uint64_t*>(d.tab_addr.p);
    la.lens = static_cast<const uint64_t*>(d.tab_len.p);
    la.nleaves = T;
    la.byte_end = ~0ull;
    la.digests = d.leaves.u8();
    hipEvent_t* tr = timing_record(c, d);
    if (tr) HIP_TRY(hipEventRecord(tr[0], s));
    RC_TRY(launch_leaves(c, d, s, la, true, aligned, kind >= 0 ? kind : pick_leaf_kernel(c, d, T)));
    if (tr) HIP_TRY(hipEventRecord(tr[1], s));
    RC_TRY(batch_roots_from_leaves(c, d, s, d.leaves.u8(), first, roots));
    if (tr) HIP_TRY(hipEventRecord(tr[2], s));
    return DM_OK;
}

// Device-visible addresses of host chunks that all lie in page-locked memory (hipHostMalloc,
// hipHostRegister): one runtime query per pinned allocation, not per chunk (12,500 queries cost
// ~30 ms per call).  False if any non-empty chunk is pageable or runs past its allocation.  Empty
// chunks get the first non-empty chunk's address (the kernels never dereference them).
bool pinned_view(const void* const* ptrs, const uint64_t* lens, uint64_t n, std::vector<uint64_t>* dev_addr) {
    uintptr_t lo = 0, hi = 0;
    uint64_t delta = 0;   // device address = host address + delta inside [lo, hi)
    bool ok = true;
    if (dev_addr) dev_addr->assign(n, 0);
    uint64_t any = 0;
    for (uint64_t i = 0; i < n && ok; i++) {
        if (lens[i] == 0) continue;
        const uintptr_t p = reinterpret_cast<uintptr_t>(ptrs[i]);
        if (!(p >= lo && p + lens[i] <= hi)) {
            hipPointerAttribute_t attr{};
            void* start = nullptr;
            void* dp = nullptr;
            ok = hipPointerGetAttributes(&attr, ptrs[i]) == hipSuccess && attr.type == hipMemoryTypeHost &&
                 hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)ptrs[i]) == hipSuccess &&
                 start != nullptr && (!dev_addr || (hipHostGetDevicePointer(&dp, start, 0) == hipSuccess && dp));
            if (!ok) break;
            // Extent of the allocation.  HIP_POINTER_ATTRIBUTE_RANGE_SIZE comes back truncated to
            // 32 bits for pinned allocations of 4 GiB and more (0 for torch's 16 GiB block,
            // measured), so take the larger of it and hipMemPtrGetInfo.  If neither covers the chunk,
            // accept it when its last byte lies in the same allocation (same range start).
            const uintptr_t s0 = reinterpret_cast<uintptr_t>(start);
            size_t size = 0, size2 = 0;
            if (hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)ptrs[i]) != hipSuccess) size = 0;
            if (hipMemPtrGetInfo(start, &size2) == hipSuccess && size2 > size) size = size2;
            uintptr_t end = s0 + size;
            if (p + lens[i] > end) {
                void* s_last = nullptr;
                const void* last = reinterpret_cast<const void*>(p + lens[i] - 1);
                ok = hipPointerGetAttribute(&s_last, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)last) == hipSuccess &&
                     s_last == start;
                end = p + lens[i];
            }
            if (!ok) break;
            lo = s0;
            hi = end;
            delta = dev_addr ? reinterpret_cast<uintptr_t>(dp) - s0 : 0;
        }
        if (dev_addr) {
            (*dev_addr)[i] = p + delta;
            if (!any) any = p + delta;
        }
    }
    (void)hipGetLastError();   // clear the error of an unregistered pointer
    if (ok && dev_addr)
        for (uint64_t i = 0; i < n; i++)
            if (lens[i] == 0) (*dev_addr)[i] = any;
    return ok;
}

// Zero-copy: leaves in pinned host memory are read in place by K1Q over PCIe, without a copy
// to HBM.  K1Q's producer lanes load 8 consecutive 64-byte blocks per leaf, so its reads cross
// PCIe as whole lines.  Measured from torch-pinned memory (profiles/r02/LOGS.md, r02s_zc_*.log),
// zero-copy vs copy: 8 GiB as 256 x 32 MiB 15.81 vs 15.63 GiB/s (the
// chain rate either way, without the 8 GiB device copy), 8,192 x 1 MiB 53.2 vs 52.4 (PCIe),
// batches of 1 MiB objects 51.5 vs 43.8 (4,096), 53.2 vs 46.9 (8,192), 49.4 vs 47.6 (12,500).
// K1L, K1P and K1 reach only ~41 GB/s reading host memory (profiles/r02/LOGS.md), so the
// many-leaf (wide) regime still copies.  Auto mode only (a forced kernel keeps the copy
// paths testable); DEOSS_ZERO_COPY=0 turns it off.
bool zero_copy_regime(const dm_ctx* c, const Dev& d, uint64_t nleaves) {
    static const bool off = [] {
        const char* e = std::getenv("DEOSS_ZERO_COPY");
        return e != nullptr && e[0] == '0';
    }();
    return !off && c->leaf_mode == DM_LEAF_AUTO && nleaves > 0 && pick_leaf_kernel(c, d, nleaves) != DM_LEAF_WIDE;
}

// Copy host chunks to d.data + off[i] (device offsets chosen by the caller, 256-B aligned,
// non-overlapping; bytes up to the next 256-B boundary after a chunk may be overwritten) through
// the pinned ring, or straight from the caller's memory when every chunk is pinned.
int h2d_at(dm_ctx* c, Dev& d, const void* const* ptrs, const uint64_t* lens, uint64_t n,
           const std::vector<uint64_t>& off) {
    // Pinned sources (every chunk in page-locked host memory): async copies straight from the
    // caller's buffers, coalescing runs that are contiguous on both sides with no padding between
    // them (so a copy never reads a host byte outside the caller's chunks).
    const bool all_pinned = pinned_view(ptrs, lens, n, nullptr);
    if (all_pinned) {
        uint64_t i = 0;
        while (i < n) {
            if (lens[i] == 0) { i++; continue; }
            const uint8_t* h0 = static_cast<const uint8_t*>(ptrs[i]);
            uint64_t j = i + 1;
            while (j < n && lens[j] && off[j] == off[j - 1] + lens[j - 1] &&
                   static_cast<const uint8_t*>(ptrs[j]) == static_cast<const uint8_t*>(ptrs[j - 1]) + lens[j - 1])
                j++;
            const uint64_t bytes = off[j - 1] - off[i] + lens[j - 1];
            HIP_TRY(hipMemcpyAsync(d.data.u8() + off[i], h0, bytes, hipMemcpyHostToDevice, d.copy));
            i = j;
        }
        HIP_TRY(hipStreamSynchronize(d.copy));
        return DM_OK;
    }
    HIP_TRY(d.stage[0].ensure(kStageBytes));
    HIP_TRY(d.stage[1].ensure(kStageBytes));
    int slot = 0;
    bool busy[2] = {false, false};
    uint64_t fill = 0, slot_dev_off = 0;
    std::vector<dm_copy::CopyItem> pending;   // this slot's host copies, done together at flush (par_copy)
    auto flush = [&]() -> int {
        if (fill == 0) return DM_OK;
        par_copy(pending);   // while the other slot's H2D is in flight
        pending.clear();
        HIP_TRY(hipMemcpyAsync(d.data.u8() + slot_dev_off, d.stage[slot].p, fill, hipMemcpyHostToDevice, d.copy));
        HIP_TRY(hipEventRecord(d.ev_copy[slot], d.copy));
        busy[slot] = true;
        slot ^= 1;
        if (busy[slot]) HIP_TRY(hipEventSynchronize(d.ev_copy[slot]));
        busy[slot] = false;
        fill = 0;
        return DM_OK;
    };
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t span = round_up(lens[i], kAlign);
        if (lens[i] > kStageBytes) {   // large chunk: direct copy (pageable source, synchronous)
            RC_TRY(flush());
            HIP_TRY(hipMemcpyAsync(d.data.u8() + off[i], ptrs[i], lens[i], hipMemcpyHostToDevice, d.copy));
            continue;
        }
        if (fill != 0 && (off[i] != slot_dev_off + fill || fill + span > kStageBytes)) RC_TRY(flush());
        if (fill == 0) slot_dev_off = off[i];
        if (lens[i]) pending.push_back({d.stage[slot].u8() + fill, ptrs[i], (size_t)lens[i]});
        fill += span;
    }
    RC_TRY(flush());
    HIP_TRY(hipStreamSynchronize(d.copy));
    return DM_OK;
}

// Pack host chunks into device memory (256-B aligned starts) through the pinned ring.
// Returns the device address of each chunk in `addr`.
int pack_chunks(dm_ctx* c, Dev& d, const void* const* ptrs, const uint64_t* lens, uint64_t n,
                std::vector<uint64_t>& addr) {
    std::vector<uint64_t> off(n);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) {
        off[i] = total;
        total = round_up(total + lens[i], kAlign);
    }
    HIP_TRY(d.data.ensure(std::max<uint64_t>(total, kAlign)));
    addr.resize(n);
    for (uint64_t i = 0; i < n; i++) addr[i] = reinterpret_cast<uint64_t>(d.data.u8() + off[i]);
    return h2d_at(c, d, ptrs, lens, n, off);
}

// Stripe schedule of the streamed paths (host buffers, files): W bytes of every leaf per step at
// full width, but the stripes start at W/16 and grow by 1/8 per step.  The first stripe's transfer
// overlaps nothing (the GPU waits for it), and each later one must finish within the previous
// stripe's hashing (transfers run ~1.2x the chain-bound hash rate at 256 x 32 MiB).  Offsets and
// widths are multiples of 64 (whole blocks).  Measured on the files path: 15.45 -> 15.70 GiB/s
// (profiles/r02/LOGS.md#r02x_files.log).
void stripe_schedule(uint64_t W, uint64_t len, std::vector<uint64_t>& so, std::vector<uint64_t>& sw) {
    so.clear();
    sw.clear();
    for (uint64_t off = 0, w = std::max<uint64_t>(64, (W / 16) / 64 * 64); off < len;) {
        so.push_back(off);
        sw.push_back(w);
        off += w;
        w = std::min(W, std::max(w + 64, (w + w / 8) / 64 * 64));
    }
}

// Host object buffer -> HBM, hashing overlapped with the H2D copies.  Leaf digests land in
// d.leaves; the caller reduces them.  Stripes: every leaf advances by W bytes per step, so all
// leaves stay in flight (large-chunk case); when W covers a whole chunk this is one step of
// contiguous copies.
int h2d_and_hash_leaves(dm_ctx* c, Dev& d, const void* host, uint64_t len, uint64_t chunk) {
    const uint64_t n = ceil_div(len, chunk);
    const uint64_t last_len = len - (n - 1) * chunk;
    std::vector<uint64_t> view;
    if (zero_copy_regime(c, d, n) && pinned_view(&host, &len, 1, &view)) {
        HIP_TRY(d.leaves.ensure(n * 32));
        dm::LeafArgs la = uniform_args(reinterpret_cast<const void*>(view[0]), len, chunk);
        la.byte_end = ~0ull;
        la.digests = d.leaves.u8();
        return launch_leaves(c, d, d.stream, la, false, view[0] % 16 == 0 && chunk % 16 == 0, DM_LEAF_QUAD);
    }
    HIP_TRY(d.data.ensure(len));
    HIP_TRY(d.leaves.ensure(n * 32));
    hipPointerAttribute_t attr{};
    bool pinned = false;
    if (hipPointerGetAttributes(&attr, host) == hipSuccess)
        pinned = attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();   // clear the error of an unregistered pointer
    const bool aligned = (chunk % 16) == 0;
    // Many leaves (wide kernel): hashing runs far above the PCIe rate, so copy then hash in one
    // launch.  Fewer, larger leaves (latency-bound hashing): stripes keep every leaf in flight
    // while the next stripe is copied.
    const bool contiguous = pick_leaf_kernel(c, d, n) == DM_LEAF_WIDE || len <= kStripeBudget;
    dm::LeafArgs la{};
    la.pitch = chunk;
    la.leaf_len = chunk;
    la.last_len = last_len;
    la.digests = d.leaves.u8();
    hipStream_t s = d.stream;
    if (contiguous) {
        // one hashing step over all leaves; copies in <= kStageBytes pieces
        HIP_TRY(d.stage[0].ensure(kStageBytes));
        HIP_TRY(d.stage[1].ensure(kStageBytes));
        int slot = 0;
        bool busy[2] = {false, false};
        for (uint64_t o = 0; o < len; o += kStageBytes) {
            const uint64_t sz = std::min(kStageBytes, len - o);
            if (pinned) {
                HIP_TRY(hipMemcpyAsync(d.data.u8() + o, static_cast<const uint8_t*>(host) + o, sz,
                                       hipMemcpyHostToDevice, d.copy));
            } else {
                if (busy[slot]) HIP_TRY(hipEventSynchronize(d.ev_copy[slot]));
                par_copy({{d.stage[slot].p, static_cast<const uint8_t*>(host) + o, (size_t)sz}});
                HIP_TRY(hipMemcpyAsync(d.data.u8() + o, d.stage[slot].p, sz, hipMemcpyHostToDevice, d.copy));
                HIP_TRY(hipEventRecord(d.ev_copy[slot], d.copy));
                busy[slot] = true;
                slot ^= 1;
            }
        }
        HIP_TRY(hipEventRecord(d.ev_copy[0], d.copy));
        HIP_TRY(hipStreamWaitEvent(s, d.ev_copy[0], 0));
        la.base = d.data.u8();
        la.nleaves = n;
        la.byte_end = ~0ull;
        return launch_leaves(c, d, s, la, false, aligned, pick_leaf_kernel(c, d, n));
    }
    // striped: W bytes of every leaf per step (W multiple of 64), state carried in HBM
    const uint64_t W = std::max<uint64_t>(64, (kStripeBudget / n) / 64 * 64);
    std::vector<uint64_t> so, sw;
    stripe_schedule(W, chunk, so, sw);
    const uint64_t nsteps = so.size();
    HIP_TRY(d.nodes_b.ensure(n * 32));   // per-leaf chaining state (8 words)
    uint32_t* state = static_cast<uint32_t*>(d.nodes_b.p);
    HIP_TRY(d.stage[0].ensure(std::min<uint64_t>(W * n, kStripeBudget)));
    HIP_TRY(d.stage[1].ensure(std::min<uint64_t>(W * n, kStripeBudget)));
    bool busy[2] = {false, false};
    int slot = 0;
    hipEvent_t* ev_hashed = d.ev_step;
    for (uint64_t step = 0; step < nsteps; step++) {
        const uint64_t b0 = so[step];
        const uint64_t w = std::min(sw[step], chunk - b0);
        const uint8_t* src = static_cast<const uint8_t*>(host);
        // rows 0..n-2 are full chunks; row n-1 holds last_len bytes
        const uint64_t last_w = last_len > b0 ? std::min(w, last_len - b0) : 0;
        if (pinned) {
            if (n > 1)
                HIP_TRY(hipMemcpy2DAsync(d.data.u8() + b0, chunk, src + b0, chunk, w, n - 1, hipMemcpyHostToDevice, d.copy));
            if (last_w)
                HIP_TRY(hipMemcpyAsync(d.data.u8() + (n - 1) * chunk + b0, src + (n - 1) * chunk + b0, last_w,
                                       hipMemcpyHostToDevice, d.copy));
        } else {
            if (busy[slot]) HIP_TRY(hipEventSynchronize(d.ev_copy[slot]));
            uint8_t* st = d.stage[slot].u8();
            std::vector<dm_copy::CopyItem> rows;
            rows.reserve(n);
            for (uint64_t r = 0; r + 1 < n; r++) rows.push_back({st + r * w, src + r * chunk + b0, (size_t)w});
            if (last_w) rows.push_back({st + (n - 1) * w, src + (n - 1) * chunk + b0, (size_t)last_w});
            par_copy(rows);
            if (n > 1)
                HIP_TRY(hipMemcpy2DAsync(d.data.u8() + b0, chunk, st, w, w, n - 1, hipMemcpyHostToDevice, d.copy));
            if (last_w)
                HIP_TRY(hipMemcpyAsync(d.data.u8() + (n - 1) * chunk + b0, st + (n - 1) * w, last_w,
                                       hipMemcpyHostToDevice, d.copy));
            HIP_TRY(hipEventRecord(d.ev_copy[slot], d.copy));
            busy[slot] = true;
            slot ^= 1;
        }
        HIP_TRY(hipEventRecord(ev_hashed[step & 1], d.copy));
        HIP_TRY(hipStreamWaitEvent(s, ev_hashed[step & 1], 0));
        la.base = d.data.u8() + b0;
        la.nleaves = n;
        la.byte_off = b0;
        la.byte_end = b0 + w;
        la.state = state;
        RC_TRY(launch_leaves(c, d, s, la, false, aligned, pick_leaf_kernel(c, d, n)));
    }
    return DM_OK;
}

// Device-resident single object on device d (caller holds the context lock).
int root_device_impl(dm_ctx* c, Dev& d, hipStream_t s, const void* dev, uint64_t len, uint64_t chunk,
                     uint8_t* dev_root, uint8_t* leaf_out_dev) {
    if (len == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    RC_TRY(begin_call(c, d, s));
    dm::LeafArgs la = uniform_args(dev, len, chunk);
    uint64_t nout = 0;
    const bool aligned = is_aligned16(dev) && chunk % 16 == 0;
    return run_tree(c, d, s, la, false, aligned, -1, dev_root, &nout, leaf_out_dev);
}

int init_device(dm_ctx* c, Dev& d) {
    HIP_TRY(hipSetDevice(d.id));
    for (DevBuf* b : {&d.data, &d.nodes_a, &d.nodes_b, &d.leaves, &d.tab_addr, &d.tab_len, &d.tab_first, &d.tab_ids,
                      &d.root, &d.gather, &d.proof_paths, &d.proof_bits, &d.proof_roots}) {
        b->rp = &c->reaper;   // scratch growth never synchronises the device (Reaper)
        b->dev = d.id;
    }
    HIP_TRY(hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, d.id));
    // A process's ordinary HIP streams share GPU_MAX_HW_QUEUES (4) hardware queues per priority
    // level, assigned least-used at creation, and a kernel or copy waits behind anything queued
    // before it on its queue (profiles/r03/r03l_hwq.log; tools/conc_probe.hip: 4 normal streams run side
    // by side, a 5th waits).  Which queue a lane would get then depends on every stream the process
    // made before (torch's included): measured, two lanes' 0.5 s chains shared one queue after a
    // caller had created 4 streams (profiles/r03/LOGS.md#r03u_lanes.log).  A stream made with a CU mask gets
    // a hardware queue of its own (conc_probe cumask: 8 such streams side by side after 8 ordinary
    // ones), so each lane's compute stream is one, with every CU enabled.  Such streams synchronise
    // with the legacy null stream (the library never uses it; a caller's stream-0 work orders with
    // them).  The copy stream takes a lowest-priority queue: H2D copies never wait behind a chain.
    int prio_least = 0, prio_greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
    {
        std::vector<uint32_t> all_cus((size_t)(d.cus + 31) / 32, 0xffffffffu);
        HIP_TRY(hipExtStreamCreateWithCUMask(&d.stream, (uint32_t)all_cus.size(), all_cus.data()));
    }
    HIP_TRY(hipStreamCreateWithPriority(&d.copy, hipStreamNonBlocking, prio_least));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_tail, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_done, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_copy[0], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_copy[1], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_step[0], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_step[1], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.ev_htab, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(d.ev_htab, d.stream));
    HIP_TRY(d.root.ensure(4096));
    return DM_OK;
}

void destroy_device(Dev& d) {
    if (hipSetDevice(d.id) != hipSuccess) return;
    (void)hipDeviceSynchronize();
    for (DevBuf* b : {&d.data, &d.nodes_a, &d.nodes_b, &d.leaves, &d.tab_addr, &d.tab_len, &d.tab_first, &d.tab_ids,
                      &d.root, &d.gather, &d.proof_paths, &d.proof_bits, &d.proof_roots})
        b->release();
    d.stage[0].release();
    d.stage[1].release();
    d.htab.release();
    for (hipEvent_t e : {d.ev_done, d.ev_copy[0], d.ev_copy[1], d.ev_step[0], d.ev_step[1], d.ev_htab, d.ev_tail})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : d.tev) (void)hipEventDestroy(e);
    if (d.stream) (void)hipStreamDestroy(d.stream);
    if (d.copy) (void)hipStreamDestroy(d.copy);
}

// D2H of the leaf digests + root of a single-device tree whose leaf digests sit in d.leaves.
int reduce_leaves_to_host(dm_ctx* c, Dev& d, uint64_t n, uint8_t* leaf_out, uint8_t root[32]) {
    hipStream_t s = d.stream;
    uint8_t* droot = d.root.u8();
    RC_TRY(finish(c, d, s, d.leaves.u8(), n, true, droot));
    HIP_TRY(hipMemcpyAsync(root, droot, 32, hipMemcpyDeviceToHost, s));
    if (leaf_out) HIP_TRY(hipMemcpyAsync(leaf_out, d.leaves.p, n * 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return DM_OK;
}

// Leaf producer of the multi-device path: fills d.leaves with the digests of leaves [l0, l1)
// (stream-ordered on d.stream), reporting errors into its own context `cc`.
using LeafProducer = std::function<int(dm_ctx* cc, Dev& d, uint64_t l0, uint64_t l1)>;

// RCCL communicators over devices [0, G) of the context, created on first use (the caller holds
// those devices' locks, so no other call is using them).
int comms_for(dm_ctx* c, int G, std::vector<ncclComm_t>** out) {
    std::lock_guard<std::mutex> lk(c->comm_mu);
    auto it = c->comms.find(G);
    if (it == c->comms.end()) {
        std::vector<int> ids(G);
        for (int g = 0; g < G; g++) ids[g] = c->devs[g].id;
        std::vector<ncclComm_t> cm(G);
        if (c->fail_comm_init)
            return fail(c, DM_ERR_RCCL, "ncclCommInitAll over %d GPUs: injected failure (DEOSS_TEST_RCCL_INIT_FAIL=1)", G);
        NCCL_TRY(ncclCommInitAll(cm.data(), G, ids.data()));
        it = c->comms.emplace(G, std::move(cm)).first;
    }
    *out = &it->second;
    return DM_OK;
}

// Multi-device single object over devices [0, G) (the caller holds their locks): the aligned
// partition of dm_plan::plan_shards (blocks of 2^k leaves, contiguous block ranges), each device's
// leaf digests from ONE pass of `produce` (they feed both the k-level subtree reduce and
// leaf_out), one RCCL all-gather of the 32-byte level-k nodes, final levels on device 0.  Odd-node
// duplication only ever touches the global last node, which lives in the last block, so the
// per-device nodes are exactly the global level-k nodes (shard_plan.hpp).
int multi_root(dm_ctx* c, int G, uint64_t n, const LeafProducer& produce, uint8_t* leaf_out, uint8_t root[32]) {
    const dm_plan::Layout P = dm_plan::plan_shards(n, G);
    const uint32_t k = P.k;
    const uint64_t nb = P.nb, maxc = P.max_nodes();
    std::vector<ncclComm_t>* comms = nullptr;
    if (!c->virtual_devs) RC_TRY(comms_for(c, G, &comms));
    // order this call's scratch use after every call still queued on another stream of each device
    for (int g = 0; g < G; g++) RC_TRY(begin_call(c, c->devs[g], c->devs[g].stream));
    std::vector<int> rcs(G, DM_OK);
    std::vector<std::string> errs(G);
    auto work = [&](int g) {
        Dev& d = c->devs[g];
        dm_ctx local;   // private error sink (no devices: helpers given it must not index devs)
        local.leaf_mode = c->leaf_mode.load();
        dm_ctx* cc = &local;
        int rc = DM_OK;
        do {
            if (hipSetDevice(d.id) != hipSuccess) { rc = fail(cc, DM_ERR_HIP, "hipSetDevice(%d)", d.id); break; }
            const uint64_t l0 = P.leaf_lo(g), l1 = P.leaf_hi(g);
            if (d.gather.ensure(std::max<uint64_t>(maxc, 1) * 32 * (G + 1)) != hipSuccess) {
                rc = fail(cc, DM_ERR_NOMEM, "gather slots");
                break;
            }
            if (l1 <= l0) break;
            const uint64_t nl = l1 - l0;
            if ((rc = produce(cc, d, l0, l1)) != DM_OK) break;
            // exactly k levels of this device's blocks (odd levels self-pair inside the last block)
            if (k == 0) {
                if (hipMemcpyAsync(d.gather.p, d.leaves.p, nl * 32, hipMemcpyDeviceToDevice, d.stream) != hipSuccess) {
                    rc = fail(cc, DM_ERR_HIP, "level-0 copy");
                    break;
                }
            } else if ((rc = reduce_stages(cc, d, d.stream, d.leaves.u8(), nl, k, d.gather.u8())) != DM_OK) {
                break;
            }
            if (leaf_out && hipMemcpyAsync(leaf_out + 32 * l0, d.leaves.p, nl * 32, hipMemcpyDeviceToHost, d.stream) != hipSuccess) {
                rc = fail(cc, DM_ERR_HIP, "leaf digests D2H");
                break;
            }
        } while (0);
        rcs[g] = rc;
        errs[g] = local.err;
    };
    if (G == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; g++) th.emplace_back(work, g);
        for (auto& t : th) t.join();
    }
    for (int g = 0; g < G; g++)
        if (rcs[g] != DM_OK) {
            // a file error keeps the Go message shape ("open <path>: ..."): no device prefix
            if (rcs[g] == DM_ERR_IO || rcs[g] == DM_ERR_EMPTY) return fail(c, rcs[g], "%s", errs[g].c_str());
            return fail(c, rcs[g], "device %d: %s", c->devs[g].id, errs[g].c_str());
        }
    // C1: all-gather of fixed-size slots (maxc nodes of 32 B per device) over RCCL
    const size_t slot = maxc * 32;
    const bool timed = c->timing;
    std::chrono::steady_clock::time_point x0;
    if (timed) {   // measured exchange: every device's subtree roots ready first
        for (int g = 0; g < G; g++) {
            HIP_TRY(hipSetDevice(c->devs[g].id));
            HIP_TRY(hipStreamSynchronize(c->devs[g].stream));
        }
        x0 = std::chrono::steady_clock::now();
    }
    if (c->virtual_devs) {   // test hook: every context device is the same GPU (no RCCL), see dm_ctx
        for (int g = 0; g < G; g++) {
            Dev& d = c->devs[g];
            HIP_TRY(hipMemcpyAsync(c->devs[0].gather.u8() + slot + g * slot, d.gather.p, slot, hipMemcpyDeviceToDevice,
                                   d.stream));
        }
        for (int g = 0; g < G; g++) HIP_TRY(hipStreamSynchronize(c->devs[g].stream));
    } else {
        NCCL_TRY(ncclGroupStart());
        for (int g = 0; g < G; g++) {
            Dev& d = c->devs[g];
            const ncclResult_t r = ncclAllGather(d.gather.u8(), d.gather.u8() + slot, slot, ncclUint8, (*comms)[g], d.stream);
            if (r != ncclSuccess) {   // close the group first: an open one would swallow the next call's collectives
                (void)ncclGroupEnd();
                return fail(c, DM_ERR_RCCL, "ncclAllGather on device %d: %s", d.id, ncclGetErrorString(r));
            }
        }
        NCCL_TRY(ncclGroupEnd());
    }
    if (timed) {
        for (int g = 0; g < G; g++) {
            HIP_TRY(hipSetDevice(c->devs[g].id));
            HIP_TRY(hipStreamSynchronize(c->devs[g].stream));
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - x0).count();
        std::lock_guard<std::mutex> lk(c->xmu);
        c->x_n++;
        c->x_sum_us += us;
        c->x_max_us = std::max(c->x_max_us, us);
        c->x_last_G = G;
    }
    Dev& d0 = c->devs[0];
    HIP_TRY(hipSetDevice(d0.id));
    // compact the gathered slots into block order on device 0, in d0.leaves (K2's scratch is
    // nodes_a/b) once device 0's leaf_out copy has left it
    HIP_TRY(hipStreamSynchronize(d0.stream));
    HIP_TRY(d0.leaves.ensure(std::max<uint64_t>(nb, 1) * 32 + 256));
    for (int g = 0; g < G; g++) {
        if (P.nodes(g) == 0) continue;
        HIP_TRY(hipMemcpyAsync(d0.leaves.u8() + 32 * P.node_offset(g), d0.gather.u8() + slot + g * slot,
                               P.nodes(g) * 32, hipMemcpyDeviceToDevice, d0.stream));
    }
    RC_TRY(finish(c, d0, d0.stream, d0.leaves.u8(), nb, k == 0, d0.root.u8()));
    HIP_TRY(hipMemcpyAsync(root, d0.root.p, 32, hipMemcpyDeviceToHost, d0.stream));
    for (int g = 0; g < G; g++) {
        HIP_TRY(hipSetDevice(c->devs[g].id));
        HIP_TRY(hipStreamSynchronize(c->devs[g].stream));
    }
    return DM_OK;
}

// Multi-device host buffer: each device stages its byte range through its own pinned ring (or
// straight from pinned memory) with H2D overlapped with leaf hashing (h2d_and_hash_leaves:
// stripes for few long leaves).
int root_buffer_multi(dm_ctx* c, int G, const void* host, uint64_t len, uint64_t chunk, uint8_t* leaf_out,
                      uint8_t root[32]) {
    const uint64_t n = ceil_div(len, chunk);
    auto produce = [&](dm_ctx* cc, Dev& d, uint64_t l0, uint64_t l1) -> int {
        const uint64_t byte0 = l0 * chunk, byte1 = std::min(len, l1 * chunk);
        return h2d_and_hash_leaves(cc, d, static_cast<const uint8_t*>(host) + byte0, byte1 - byte0, chunk);
    };
    return multi_root(c, G, n, produce, leaf_out, root);
}

// Source kind of host memory for routing: page-locked (crosses PCIe directly) or pageable.
int host_src(const void* p) {
    hipPointerAttribute_t attr{};
    const bool pinned = p && hipPointerGetAttributes(&attr, p) == hipSuccess && attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    return pinned ? DM_SRC_HOST_PINNED : DM_SRC_HOST_PAGEABLE;
}

// Devices a host-memory call uses (dm_plan::route; forced sharding is a test hook).
int route_call(dm_ctx* c, uint64_t n, uint64_t bytes, uint64_t leaf_max, int src, bool by_objects = false) {
    const int G = c->nphys;   // GPUs; a call never shards over lanes of one GPU
    if (c->force_sharded) return n >= 2 * (uint64_t)G ? G : 1;
    if (G <= 1 || (!c->shard_ok && !by_objects)) return 1;
    return dm_plan::route(n, bytes, leaf_max, src, G, c->devs[0].cus, c->leaf_mode.load(), ctx_load(c), by_objects,
                          nullptr, c->route_k);
}

// Whether a call of n leaves routed to G devices takes the multi-device path (with
// DEOSS_FORCE_SHARDED even G = 1 does, when n >= 2 x the context's devices).
bool sharded(const dm_ctx* c, int G, uint64_t n) {
    return G > 1 || (c->force_sharded && n >= 2 * (uint64_t)c->nphys);
}

// Leaf digests of host chunks into d.leaves (stream-ordered on d.stream): read in place from
// pinned memory by K1Q (zero-copy regime) or packed into HBM first.
int chunks_leaves(dm_ctx* c, Dev& d, const void* const* ptrs, const uint64_t* lens, uint64_t n) {
    std::vector<uint64_t> addr;
    const bool zc = zero_copy_regime(c, d, n) && pinned_view(ptrs, lens, n, &addr);
    if (!zc) RC_TRY(pack_chunks(c, d, ptrs, lens, n, addr));
    bool aligned = true;
    for (uint64_t i = 0; i < n && zc; i++) aligned &= addr[i] % 16 == 0;
    RC_TRY(tables_begin(c, d, n * 16 + 1024));
    HIP_TRY(d.leaves.ensure(n * 32));
    RC_TRY(upload(c, d, d.stream, d.tab_addr, addr.data(), n * 8));
    RC_TRY(upload(c, d, d.stream, d.tab_len, lens, n * 8));
    dm::LeafArgs la{};
    la.addrs = static_cast<const uint64_t*>(d.tab_addr.p);
    la.lens = static_cast<const uint64_t*>(d.tab_len.p);
    la.nleaves = n;
    la.byte_end = ~0ull;
    la.digests = d.leaves.u8();
    return launch_leaves(c, d, d.stream, la, true, aligned, zc ? DM_LEAF_QUAD : pick_leaf_kernel(c, d, n));
}

// Host batch of objects on device d: roots (host, nobj x 32).
int batch_host_on(dm_ctx* c, Dev& d, const void* const* objs, const uint64_t* lens, uint64_t nobj, uint64_t chunk,
                  uint8_t* roots) {
    RC_TRY(begin_call(c, d, d.stream));
    uint64_t T = 0;
    for (uint64_t o = 0; o < nobj; o++) T += ceil_div(lens[o], chunk);
    std::vector<uint64_t> addr;
    const bool zc = zero_copy_regime(c, d, T) && pinned_view(objs, lens, nobj, &addr);
    if (!zc) RC_TRY(pack_chunks(c, d, objs, lens, nobj, addr));
    std::vector<const void*> dptr(nobj);
    for (uint64_t o = 0; o < nobj; o++) dptr[o] = reinterpret_cast<const void*>(addr[o]);
    HIP_TRY(d.gather.ensure(nobj * 32));
    RC_TRY(batch_device(c, d, d.stream, dptr.data(), lens, nobj, chunk, d.gather.u8(), zc ? DM_LEAF_QUAD : -1));
    HIP_TRY(hipMemcpyAsync(roots, d.gather.p, nobj * 32, hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    return DM_OK;
}

// Host batch over devices [0, G) (the caller holds their locks): device g takes a contiguous range
// of objects with about 1/G of the leaves; objects never interact, so there is no exchange.
int batch_host_multi(dm_ctx* c, int G, const void* const* objs, const uint64_t* lens, uint64_t nobj, uint64_t chunk,
                     uint8_t* roots) {
    std::vector<uint64_t> first(nobj + 1, 0);
    for (uint64_t o = 0; o < nobj; o++) first[o + 1] = first[o] + ceil_div(lens[o], chunk);
    std::vector<uint64_t> o_lo(G + 1, nobj);
    o_lo[0] = 0;
    for (int g = 1; g < G; g++) {   // first object whose leaves start at or after g/G of the total
        const uint64_t want = first[nobj] * (uint64_t)g / (uint64_t)G;
        o_lo[g] = std::max<uint64_t>(o_lo[g - 1], (uint64_t)(std::lower_bound(first.begin(), first.end() - 1, want) - first.begin()));
    }
    std::vector<int> rcs(G, DM_OK);
    std::vector<std::string> errs(G);
    auto work = [&](int g) {
        dm_ctx local;
        local.leaf_mode = c->leaf_mode.load();
        int rc = DM_OK;
        const uint64_t a = o_lo[g], b = o_lo[g + 1];
        if (b > a) {
            if (hipSetDevice(c->devs[g].id) != hipSuccess) rc = fail(&local, DM_ERR_HIP, "hipSetDevice(%d)", c->devs[g].id);
            else rc = batch_host_on(&local, c->devs[g], objs + a, lens + a, b - a, chunk, roots + 32 * a);
        }
        rcs[g] = rc;
        errs[g] = local.err;
    };
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++) th.emplace_back(work, g);
    for (auto& t : th) t.join();
    for (int g = 0; g < G; g++)
        if (rcs[g] != DM_OK) return fail(c, rcs[g], "device %d: %s", c->devs[g].id, errs[g].c_str());
    return DM_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------
extern "C" {

const char* dm_strerror(int rc) {
    switch (rc) {
        case DM_OK: return "ok";
        case DM_ERR_EMPTY: return "Empty data";
        case DM_ERR_INVALID: return "invalid argument";
        case DM_ERR_HIP: return "HIP runtime error";
        case DM_ERR_RCCL: return "RCCL error";
        case DM_ERR_NOMEM: return "out of memory";
        case DM_ERR_IO: return "I/O error";
        case DM_ERR_NODEV: return "no usable GPU";
        default: return "unknown error";
    }
}

const char* dm_last_error(dm_ctx*) { return t_err.c_str(); }

int dm_device_count(dm_ctx* ctx) { return ctx ? ctx->nphys : 0; }

int dm_lane_count(dm_ctx* ctx) { return ctx ? ctx->lanes : 0; }

int dm_gpu_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int dm_host_alloc(uint64_t bytes, void** out) {
    if (!out || bytes == 0) return bad_arg();
    *out = nullptr;
    DeviceRestore dev;
    const hipError_t e = host_alloc(out, bytes, hipHostMallocPortable);
    if (e != hipSuccess) {
        *out = nullptr;
        return set_err(e == hipErrorOutOfMemory ? DM_ERR_NOMEM : DM_ERR_HIP, "dm_host_alloc: hipHostMalloc failed");
    }
    return DM_OK;
}

void dm_host_free(void* p) { host_release(p); }

}  // extern "C"

namespace {

// Object-buffer bytes every live context of this process may keep idle on each HIP device (lanes
// x keep_bytes per GPU of the context), claimed at dm_create and returned at dm_destroy, so the
// default lane count is sized per GPU, not per context: the Go hashtree context, the
// process context and any other dm_ctx on the same GPU share one budget.
std::mutex g_keep_mu;
std::map<int, uint64_t> g_keep_claimed;
// dm_create / dm_create_lanes hold this from sizing the lanes to claiming them, so two contexts
// created at once never both size themselves against the same unclaimed budget.
std::mutex g_create_mu;

uint64_t keep_claimed(int dev) {
    std::lock_guard<std::mutex> lk(g_keep_mu);
    auto it = g_keep_claimed.find(dev);
    return it == g_keep_claimed.end() ? 0 : it->second;
}

void keep_claim(int dev, int64_t delta) {
    std::lock_guard<std::mutex> lk(g_keep_mu);
    uint64_t& v = g_keep_claimed[dev];
    v = delta < 0 && (uint64_t)(-delta) > v ? 0 : v + delta;
}

// Call lanes per GPU when the caller does not say (dm_create): DEOSS_LANES, else sized from every
// GPU of the context's HBM and claims (the same count on each).  Every lane runs on a hardware
// queue of its own (init_device), so L lanes
// overlap L large calls (measured: 2 lanes 2x, 4 lanes 4x for pageable 2 GiB objects, PCIe-bound
// at 4 for pinned 8 GiB ones; tools/lanes_probe.py, profiles/r03/LOGS.md#r03w_lanes.log).  What a lane
// costs while idle is the object buffer it keeps between calls, at most lane_keep_bytes() (16 GiB),
// so the default is as many lanes (1 to 4) as keep (a) at most half of the free HBM idle and (b),
// together with every other live context's claim on this GPU, at most half of the GPU's HBM:
// 4 for the first two default contexts on an MI355X (288 GB), then 1.
// The object buffer each lane of a context created now keeps between calls: DEOSS_LANE_KEEP_BYTES
// (a test hook; a whole non-negative number of bytes), else kLaneKeepBytes.
uint64_t lane_keep_bytes() {
    const char* kb = std::getenv("DEOSS_LANE_KEEP_BYTES");
    if (!kb || !*kb) return kLaneKeepBytes;
    char* end = nullptr;
    const unsigned long long v = std::strtoull(kb, &end, 10);
    return (end != kb && *end == '\0' && kb[0] != '-') ? (uint64_t)v : kLaneKeepBytes;
}

// Lanes per GPU for a context over HIP devices devs[0 .. ndev) (devs NULL: device 0): the budget
// of every one of its GPUs bounds it (each GPU gets the same count), in units of what each lane
// will actually claim (lane_keep_bytes).
int default_lanes(const int* devs, int ndev) {
    const char* v = std::getenv("DEOSS_LANES");
    if (v && *v) return std::min(std::max(std::atoi(v), 1), kMaxLanes);
    const uint64_t keep = std::max<uint64_t>(lane_keep_bytes(), 1);
    uint64_t lanes = 4;
    const int n = (devs && ndev > 0) ? ndev : 1;
    for (int i = 0; i < n; i++) {
        const int dev = (devs && ndev > 0) ? devs[i] : 0;
        size_t free_b = 0, total_b = 0;
        if (hipSetDevice(dev) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();   // an unusable id: ctx_create rejects it
            continue;
        }
        const uint64_t by_free = (uint64_t)free_b / (2 * keep);
        const uint64_t half = (uint64_t)total_b / 2, claimed = keep_claimed(dev);
        const uint64_t by_budget = claimed >= half ? 0 : (half - claimed) / keep;
        lanes = std::min(lanes, std::max<uint64_t>(std::min(by_free, by_budget), 1));
    }
    return (int)lanes;
}

// An unforced multi-GPU context whose RCCL communicators could not be created keeps working with
// every call whole on one GPU (dm_ctx::shard_ok); said once on stderr, queryable (dm_can_shard).
void no_sharding(dm_ctx* c, const char* why) {
    c->shard_ok = false;
    std::fprintf(stderr, "deoss_merkle: RCCL communicators over %d GPUs unavailable (%s); every call runs whole on "
                 "one GPU\n", c->nphys, why);
}

int ctx_create(dm_ctx** out, const int* devs, int ndev, int lanes) {
    if (!out || lanes < 1 || lanes > kMaxLanes) return bad_arg();
    *out = nullptr;
    DeviceRestore dev;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return set_err(DM_ERR_NODEV, "no usable GPU");
    std::vector<int> ids;
    if (!devs || ndev <= 0) ids.push_back(0);
    else ids.assign(devs, devs + ndev);
    for (size_t i = 0; i < ids.size(); i++) {
        if (ids[i] < 0 || ids[i] >= count) return bad_arg();
        for (size_t j = 0; j < i; j++)
            if (ids[j] == ids[i]) return bad_arg();
    }
    const char* vd = std::getenv("DEOSS_VIRTUAL_DEVICES");   // test hook (dm_ctx::virtual_devs)
    const int nvirt = vd ? std::atoi(vd) : 0;
    if (nvirt > 1) {
        ids.assign((size_t)std::min(nvirt, 64), ids[0]);
        lanes = 1;   // every virtual device stands for a GPU of its own
    }
    dm_ctx* c = new dm_ctx();
    c->nphys = (int)ids.size();
    c->lanes = lanes;
    c->devs.resize(ids.size() * (size_t)lanes);
    c->slots.reset(new DevSlot[c->devs.size()]);
    const uint64_t keep = lane_keep_bytes();
    for (size_t i = 0; i < c->devs.size(); i++) {   // lane-major: lane 0 of every GPU first
        c->devs[i].id = ids[i % ids.size()];
        c->devs[i].keep_bytes = keep;
        int rc = init_device(c, c->devs[i]);
        if (rc != DM_OK) {
            dm_destroy(c);
            return rc;
        }
    }
    for (const Dev& d : c->devs) keep_claim(d.id, (int64_t)d.keep_bytes);   // returned by dm_destroy
    c->keep_claimed = true;
    const char* fs = std::getenv("DEOSS_FORCE_SHARDED");
    c->force_sharded = fs != nullptr && fs[0] == '1';
    c->route_k = dm_plan::route_constants_from_env();
    c->virtual_devs = nvirt > 1;
    const char* tf = std::getenv("DEOSS_TEST_RCCL_INIT_FAIL");
    c->fail_comm_init = tf && tf[0] == '1' && ids.size() > 1 && !c->force_sharded;
    // every device's communicator up front: fail here, not mid-call
    if ((ids.size() > 1 || c->force_sharded) && (!c->virtual_devs || c->fail_comm_init)) {
        std::vector<ncclComm_t>* cm = nullptr;
        const int rc = comms_for(c, (int)ids.size(), &cm);
        if (rc != DM_OK && c->force_sharded) {
            dm_destroy(c);
            return set_err(DM_ERR_RCCL, "ncclCommInitAll failed");
        }
        if (rc != DM_OK) {   // sharding is an optimisation: keep the context, never shard an object
            std::string why;
            {
                std::lock_guard<std::mutex> lk(c->err_mu);
                why.swap(c->err);
            }
            t_err.clear();
            no_sharding(c, why.c_str());
        }
    }
    *out = c;
    return DM_OK;
}

}  // namespace

extern "C" {

int dm_create(dm_ctx** out, const int* devs, int ndev) {
    int first = (devs && ndev > 0) ? devs[0] : 0;
    int count = 0;
    DeviceRestore dr;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return set_err(DM_ERR_NODEV, "no usable GPU");
    if (first < 0 || first >= count) return bad_arg();
    std::lock_guard<std::mutex> lk(g_create_mu);
    return ctx_create(out, devs, ndev, default_lanes(devs, ndev));
}

int dm_create_lanes(dm_ctx** out, const int* devs, int ndev, int lanes) {
    std::lock_guard<std::mutex> lk(g_create_mu);
    return ctx_create(out, devs, ndev, lanes);
}

int dm_can_shard(dm_ctx* ctx) { return ctx && ctx->nphys > 1 && (ctx->shard_ok || ctx->force_sharded) ? 1 : 0; }

int dm_keep_claimed(int hip_device, uint64_t* bytes) {
    if (!bytes || hip_device < 0) return bad_arg();
    *bytes = keep_claimed(hip_device);
    return DM_OK;
}

void dm_destroy(dm_ctx* ctx) {
    if (!ctx) return;
    DeviceRestore dev;
    for (auto& kv : ctx->comms)
        for (auto& cm : kv.second) (void)ncclCommDestroy(cm);
    for (size_t g = 0; g < ctx->devs.size() && ctx->slots; g++) {
        if (hipSetDevice(ctx->devs[g].id) != hipSuccess) continue;
        for (StreamKit* k : ctx->slots[g].kits) kit_destroy(k);
        ctx->slots[g].kits.clear();
    }
    ctx->reaper.finish();
    for (auto& d : ctx->devs) {
        if (ctx->keep_claimed) keep_claim(d.id, -(int64_t)d.keep_bytes);
        destroy_device(d);
    }
    delete ctx;
}

int dm_set_leaf_kernel(dm_ctx* ctx, int mode) {
    if (!ctx || mode < DM_LEAF_AUTO || mode > DM_LEAF_QUAD) return bad_arg();
    RangeLock lk(ctx);   // after every call in flight
    ctx->leaf_mode = mode;
    return DM_OK;
}

int dm_leaf_kernel_for(dm_ctx* ctx, uint64_t nleaves) {
    if (!ctx) return bad_arg();
    return pick_leaf_kernel(ctx, ctx->devs[0], nleaves);
}

int dm_set_timing(dm_ctx* ctx, int enable) {
    if (!ctx) return bad_arg();
    RangeLock lk(ctx);
    ctx->timing = enable != 0;
    for (auto& d : ctx->devs) d.ntimed = 0;
    std::lock_guard<std::mutex> xl(ctx->xmu);
    ctx->x_n = 0;
    ctx->x_sum_us = ctx->x_max_us = 0;
    ctx->x_last_G = 0;
    return DM_OK;
}

int dm_exchange_timing(dm_ctx* ctx, uint64_t* n, double* us_sum, double* us_max, int* last_ndev) {
    if (!ctx) return bad_arg();
    std::lock_guard<std::mutex> xl(ctx->xmu);
    if (n) *n = ctx->x_n;
    if (us_sum) *us_sum = ctx->x_sum_us;
    if (us_max) *us_max = ctx->x_max_us;
    if (last_ndev) *last_ndev = ctx->x_last_G;
    return DM_OK;
}

int dm_last_call_devices(dm_ctx* ctx, int* devs, int* hip_ids, int cap, int* lane) {
    if (!ctx || cap < 0) return bad_arg();
    if (t_call_ctx != ctx->serial) {   // no call of this context on this thread yet
        if (lane) *lane = -1;
        return 0;
    }
    const int n = (int)t_call_devs.size();
    for (int i = 0; i < n && i < cap; i++) {
        if (devs) devs[i] = t_call_devs[i];
        if (hip_ids) hip_ids[i] = ctx->devs[t_call_devs[i]].id;
    }
    if (lane) *lane = t_call_lane;
    return n;
}

int dm_timing_summary(dm_ctx* ctx, uint64_t* ncalls, double* leaf_ms_sum, double* total_ms_sum, double* leaf_ms_max) {
    if (!ctx) return bad_arg();
    RangeLock lk(ctx);
    dm_ctx* c = ctx;
    uint64_t n = 0;
    double a = 0, b = 0, mx = 0;
    for (auto& d : ctx->devs) {
        if (d.ntimed == 0) continue;
        HIP_TRY(hipSetDevice(d.id));
        HIP_TRY(hipEventSynchronize(d.tev[3 * d.ntimed - 1]));
        for (size_t i = 0; i < d.ntimed; i++) {
            float x = 0, y = 0;
            HIP_TRY(hipEventElapsedTime(&x, d.tev[3 * i], d.tev[3 * i + 1]));
            HIP_TRY(hipEventElapsedTime(&y, d.tev[3 * i], d.tev[3 * i + 2]));
            a += x;
            b += y;
            mx = std::max(mx, (double)x);
            n++;
        }
    }
    if (ncalls) *ncalls = n;
    if (leaf_ms_sum) *leaf_ms_sum = a;
    if (total_ms_sum) *total_ms_sum = b;
    if (leaf_ms_max) *leaf_ms_max = mx;
    return DM_OK;
}

int dm_plan_shards(uint64_t nleaves, int ndev, uint32_t* levels, uint64_t* nblocks, uint64_t* leaf_lo,
                   uint64_t* leaf_hi) {
    if (ndev < 1 || !levels || !nblocks) return bad_arg();
    const dm_plan::Layout P = dm_plan::plan_shards(nleaves, ndev);
    *levels = P.k;
    *nblocks = P.nb;
    for (int g = 0; g < ndev; g++) {
        if (leaf_lo) leaf_lo[g] = P.leaf_lo(g);
        if (leaf_hi) leaf_hi[g] = P.leaf_hi(g);
    }
    return DM_OK;
}

int dm_plan_route(uint64_t nleaves, uint64_t bytes, uint64_t leaf_max, int source, int by_objects, int ndev, int cus,
                  int leaf_mode, int busy, double* est_ms) {
    if (ndev < 1 || cus < 1 || source < DM_SRC_DEVICE || source > DM_SRC_FILES || leaf_mode < DM_LEAF_AUTO ||
        leaf_mode > DM_LEAF_QUAD)
        return bad_arg();
    return dm_plan::route(nleaves, bytes, leaf_max, source, ndev, cus, leaf_mode, busy, by_objects != 0, est_ms,
                          dm_plan::route_constants_from_env());
}

int dm_route_constants(dm_ctx* ctx, double* allgather_us, double* host_bytes_per_s) {
    const dm_plan::RouteConstants k = ctx ? ctx->route_k : dm_plan::route_constants_from_env();
    if (allgather_us) *allgather_us = k.allgather_ms * 1e3;
    if (host_bytes_per_s) *host_bytes_per_s = k.host_bytes_per_s;
    return DM_OK;
}

int dm_root_device_async(dm_ctx* ctx, const void* dev, uint64_t len, uint64_t chunk, void* dev_root,
                         void* leaf_out_dev, void* stream) {
    if (!ctx || !dev_root || chunk == 0 || (!dev && len)) return bad_arg();
    const int g = device_of(ctx, dev);
    CallLock lk(ctx, g, kReserved);
    Dev& d = ctx->devs[g];
    return root_device_impl(ctx, d, pick_stream(d, stream), dev, len, chunk, static_cast<uint8_t*>(dev_root),
                            static_cast<uint8_t*>(leaf_out_dev));
}

int dm_root_device(dm_ctx* ctx, const void* dev, uint64_t len, uint64_t chunk, uint8_t root[32]) {
    if (!ctx || !root || chunk == 0 || (!dev && len)) return bad_arg();
    const int g = device_of(ctx, dev);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    Dev& d = c->devs[g];
    RC_TRY(root_device_impl(c, d, d.stream, dev, len, chunk, d.root.u8(), nullptr));
    HIP_TRY(hipMemcpyAsync(root, d.root.p, 32, hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    return DM_OK;
}

int dm_subtree_device_async(dm_ctx* ctx, const void* dev, uint64_t len, uint64_t chunk, uint32_t levels,
                            void* dev_nodes, uint64_t* n_out, void* stream) {
    if (!ctx || !dev_nodes || chunk == 0 || (!dev && len) || levels > 63) return bad_arg();
    const int g = device_of(ctx, dev);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (len == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    dm::LeafArgs la = uniform_args(dev, len, chunk);
    uint64_t nout = 0;
    const bool aligned = is_aligned16(dev) && chunk % 16 == 0;
    RC_TRY(run_tree(c, d, s, la, false, aligned, (int)levels, static_cast<uint8_t*>(dev_nodes), &nout, nullptr));
    if (n_out) *n_out = nout;
    return DM_OK;
}

int dm_finish_device_async(dm_ctx* ctx, const void* dev_nodes, uint64_t n, int min_one_level, void* dev_root,
                           void* stream) {
    if (!ctx || !dev_nodes || !dev_root) return bad_arg();
    const int g = device_of(ctx, dev_nodes);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (n == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    return finish(c, d, s, static_cast<const uint8_t*>(dev_nodes), n, min_one_level != 0,
                  static_cast<uint8_t*>(dev_root));
}

int dm_root_batch_device_async(dm_ctx* ctx, const void* const* dev_objs, const uint64_t* lens, uint64_t nobj,
                               uint64_t chunk, void* dev_roots, void* stream) {
    if (!ctx || chunk == 0 || (nobj && (!dev_objs || !lens || !dev_roots))) return bad_arg();
    const int g = device_of(ctx, dev_roots);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (nobj == 0) return DM_OK;
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    return batch_device(c, d, s, dev_objs, lens, nobj, chunk, static_cast<uint8_t*>(dev_roots));
}

int dm_fill_synthetic_async(dm_ctx* ctx, void* dev, uint64_t off, uint64_t nbytes, uint64_t seed, void* stream) {
    if (!ctx || (!dev && nbytes) || off % 8 || nbytes % 8 || !is_aligned16(dev)) return bad_arg();
    const int g = device_of(ctx, dev);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    if (nbytes == 0) return DM_OK;
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    const uint64_t nwords = nbytes / 8;
    const uint64_t grid = std::min<uint64_t>(ceil_div(nwords, 2 * dm::kBlock), 8192);
    hipLaunchKernelGGL(dm::fill_splitmix_kernel, dim3((uint32_t)grid), dim3(dm::kBlock), 0, s,
                       static_cast<uint64_t*>(dev), off / 8, nwords, seed);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_read_probe_async(dm_ctx* ctx, const void* dev, uint64_t nbytes, void* dev_xor8, void* stream) {
    if (!ctx || !dev_xor8 || (!dev && nbytes) || nbytes % 16 || !is_aligned16(dev) ||
        reinterpret_cast<uintptr_t>(dev_xor8) % 8)
        return bad_arg();
    const int g = device_of(ctx, dev_xor8);
    CallLock lk(ctx, g, kReserved);
    dm_ctx* c = ctx;
    Dev& d = c->devs[g];
    hipStream_t s = pick_stream(d, stream);
    RC_TRY(begin_call(c, d, s));
    HIP_TRY(hipMemsetAsync(dev_xor8, 0, 8, s));
    if (nbytes == 0) return DM_OK;
    const uint64_t n16 = nbytes / 16;
    // 8 workgroups per CU (the measured best, tools/read_peak_ab.hip), at least one load round each
    const uint64_t grid =
        std::max<uint64_t>(1, std::min<uint64_t>(8ull * d.cus, ceil_div(n16, dm::kProbeLoads * dm::kBlock)));
    hipLaunchKernelGGL(dm::read_probe_kernel, dim3((uint32_t)grid), dim3(dm::kBlock), 0, s,
                       static_cast<const uint8_t*>(dev), n16, static_cast<uint64_t*>(dev_xor8));
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_root_buffer(dm_ctx* ctx, const void* host, uint64_t len, uint64_t chunk, uint8_t* leaf_out, uint8_t root[32]) {
    if (!ctx || !root || chunk == 0 || (!host && len)) return bad_arg();
    dm_ctx* c = ctx;
    if (len == 0) {
        DeviceRestore dr;
        return fail(c, DM_ERR_EMPTY, "Empty data");
    }
    const uint64_t n = ceil_div(len, chunk);
    const int G = route_call(c, n, len, std::min(len, chunk), host_src(host));
    if (sharded(c, G, n)) {
        RangeLock lk(c, G);
        return root_buffer_multi(c, G, host, len, chunk, leaf_out, root);
    }
    const int g = pick_device(c);
    CallLock lk(c, g, kReserved);
    Dev& d = c->devs[g];
    RC_TRY(begin_call(c, d, d.stream));
    RC_TRY(h2d_and_hash_leaves(c, d, host, len, chunk));
    return reduce_leaves_to_host(c, d, n, leaf_out, root);
}

int dm_root_chunks(dm_ctx* ctx, const void* const* ptrs, const uint64_t* lens, uint64_t n, uint8_t* leaf_out,
                   uint8_t root[32]) {
    if (!ctx || !root || (n && (!ptrs || !lens))) return bad_arg();
    dm_ctx* c = ctx;
    DeviceRestore dr;
    if (n == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    uint64_t bytes = 0, maxlen = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (lens[i] && !ptrs[i]) return fail(c, DM_ERR_INVALID, "chunk %llu: NULL pointer", (unsigned long long)i);
        bytes += lens[i];
        maxlen = std::max(maxlen, lens[i]);
    }
    const int G = route_call(c, n, bytes, maxlen, host_src(ptrs[0]));
    if (sharded(c, G, n)) {
        RangeLock lk(c, G);
        auto produce = [&](dm_ctx* cc, Dev& d, uint64_t l0, uint64_t l1) -> int {
            return chunks_leaves(cc, d, ptrs + l0, lens + l0, l1 - l0);
        };
        return multi_root(c, G, n, produce, leaf_out, root);
    }
    const int g = pick_device(c);
    CallLock lk(c, g, kReserved);
    Dev& d = c->devs[g];
    RC_TRY(begin_call(c, d, d.stream));
    RC_TRY(chunks_leaves(c, d, ptrs, lens, n));
    return reduce_leaves_to_host(c, d, n, leaf_out, root);
}

int dm_root_batch(dm_ctx* ctx, const void* const* objs, const uint64_t* lens, uint64_t nobj, uint64_t chunk,
                  uint8_t* roots) {
    if (!ctx || chunk == 0 || (nobj && (!objs || !lens || !roots))) return bad_arg();
    dm_ctx* c = ctx;
    DeviceRestore dr;
    if (nobj == 0) return DM_OK;
    uint64_t T = 0, bytes = 0, maxlen = 0;
    for (uint64_t o = 0; o < nobj; o++) {
        if (lens[o] == 0) return fail(c, DM_ERR_EMPTY, "Empty data (object %llu has no bytes)", (unsigned long long)o);
        if (!objs[o]) return fail(c, DM_ERR_INVALID, "object %llu: NULL pointer", (unsigned long long)o);
        T += ceil_div(lens[o], chunk);
        bytes += lens[o];
        maxlen = std::max(maxlen, std::min(lens[o], chunk));
    }
    // objects are independent: several devices take contiguous object ranges, no exchange
    const int G = std::min<uint64_t>(route_call(c, T, bytes, maxlen, host_src(objs[0]), true), nobj);
    if (G > 1) {
        RangeLock lk(c, G);
        return batch_host_multi(c, G, objs, lens, nobj, chunk, roots);
    }
    const int g = pick_device(c);
    CallLock lk(c, g, kReserved);
    return batch_host_on(c, c->devs[g], objs, lens, nobj, chunk, roots);
}

}  // extern "C"

// Streaming (incremental) roots: dm_stream_* (shares the helpers above).
#include "merkle_stream.inl"
#include "files_capi.inl"
#include "rs_capi.inl"
#include "process_capi.inl"
#include "fullproc_capi.inl"
#include "fragment_capi.inl"
#include "process_stream.inl"
#include "tree_capi.inl"
#include "batcher.inl"
