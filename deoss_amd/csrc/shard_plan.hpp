// shard_plan.hpp -- multi-device partition and routing rules (pure host code, no HIP).
//
// Shared by the library (merkle_capi.hip: multi_root, the dm_plan_* exports), the one-process-per-GPU
// path (deoss_amd/sharding.py restates plan_shards; tests/test_dispatch_plan.py checks the two agree)
// and the host tests (tests/cpp/test_shard_plan.cpp, plain and ASan/UBSan, no GPU).
//
// Partition: the n leaves of one object are cut into blocks of S = 2^k leaves;
// device g owns the contiguous block range [nb*g/G, nb*(g+1)/G).  Every block starts at a multiple
// of 2^k, so below level k the parity of the last block's level size equals the global level's:
// merkletree v0.2.0's odd-node duplication only touches the global last node, which lives in the
// last block, and each device's k-level subtree nodes are exactly the global level-k nodes.
//
// Routing: one call either runs whole on one device or is sharded over the first G' devices.  In
// the latency regime every leaf is one serial SHA-256 chain; while a device holds all of an
// object's chains at once (<= 2 K1Q workgroups per CU), sharding cannot shorten the call, it only
// occupies more GPUs.  So a call is sharded only when the cost model below says it finishes
// sooner: the per-device share is past full-speed residency, the object is throughput-bound, or
// the host-side feed (PCIe, page cache) is the bound and more devices bring more links.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>

namespace dm_plan {

// Leaf-kernel codes (= DM_LEAF_* in include/deoss_merkle.h).
enum { kAuto = 0, kWide = 1, kLatency = 2, kPair = 3, kQuad = 4 };
// Where a call's bytes start (= DM_SRC_* in include/deoss_merkle.h).
enum { kSrcDevice = 0, kSrcHostPinned = 1, kSrcHostPageable = 2, kSrcFiles = 3 };

constexpr uint64_t kQuadLeaves = 8;   // leaves per K1Q workgroup
constexpr uint64_t kLatLeaves = 64;   // leaves per K1L workgroup

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline uint64_t ceil_shift(uint64_t n, uint32_t k) { return k >= 64 ? (n ? 1 : 0) : (n + (1ull << k) - 1) >> k; }

// Leaf kernel for a uniform object of n leaves on a device with `cus` CUs (measured crossovers,
// DESIGN.md §4.3): K1Q while ceil(n/8) <= 4 x CUs, K1L while ceil(n/64) <= CUs, K1 beyond.
inline int leaf_kind(uint64_t n, int cus, int mode) {
    if (mode != kAuto) return mode;
    if (ceil_div(n, kQuadLeaves) <= 4 * (uint64_t)cus) return kQuad;
    if (ceil_div(n, kLatLeaves) <= (uint64_t)cus) return kLatency;
    return kWide;
}

struct Layout {
    uint64_t n = 0;      // leaves
    int G = 1;           // devices (ranks)
    uint32_t k = 0;      // levels each device reduces (block = 2^k leaves)
    uint64_t nb = 0;     // blocks = level-k nodes of the global tree
    uint64_t block_lo(int g) const { return nb * (uint64_t)g / (uint64_t)G; }
    uint64_t block_hi(int g) const { return nb * (uint64_t)(g + 1) / (uint64_t)G; }
    uint64_t leaf_lo(int g) const { return std::min(n, k >= 64 ? (block_lo(g) ? n : 0) : block_lo(g) << k); }
    uint64_t leaf_hi(int g) const { return std::min(n, k >= 64 ? (block_hi(g) ? n : 0) : block_hi(g) << k); }
    uint64_t leaves(int g) const { return leaf_hi(g) - leaf_lo(g); }
    uint64_t nodes(int g) const { return block_hi(g) - block_lo(g); }   // level-k nodes device g yields
    uint64_t max_nodes() const {
        uint64_t m = 0;
        for (int g = 0; g < G; g++) m = std::max(m, nodes(g));
        return m;
    }
    uint64_t max_leaves() const {
        uint64_t m = 0;
        for (int g = 0; g < G; g++) m = std::max(m, leaves(g));
        return m;
    }
    // Where device g's nodes go when the gathered slots are compacted into block order.
    uint64_t node_offset(int g) const { return block_lo(g); }
};

// k = the largest block size (fewest gathered nodes) that still keeps every device within 1/8 of
// an even split of the leaves and gives every device at least one block; k = 0 when n < G (some
// devices then get nothing).  Exact splits are found: n = G x 2^j gives k = j, one block each
// (the weak-scaling curve, BASELINE configs[3]: 32,768 leaves over 8 GPUs -> k = 12).  k never
// exceeds ceil(log2 n): one block of 2^k >= n leaves reduced k levels is the root itself, and more
// levels would self-hash it.
inline Layout plan_shards(uint64_t n, int G) {
    Layout L;
    L.n = n;
    L.G = std::max(1, G);
    L.k = 0;
    L.nb = n;
    if (n == 0) return L;
    const uint64_t even = ceil_div(n, (uint64_t)L.G);
    for (uint32_t k = 0; k < 63 && (k == 0 || (1ull << (k - 1)) < n); k++) {
        Layout t = L;
        t.k = k;
        t.nb = ceil_shift(n, k);
        if (t.nb < (uint64_t)L.G) break;
        if (8 * t.max_leaves() <= 9 * even) L = t;
    }
    return L;
}

// ---- cost model of one call (milliseconds), constants measured on one MI355X ----------------
// Per-block time of one leaf chain (8 GiB at 32 MiB chunks, DESIGN.md §4.2 / §6.2 sweep):
// K1Q 490.6 ms / 524,289 blocks (round 3, 4-read step); K1P 9.4 GiB/s; K1L 8.7 GiB/s; K1 5.6 GiB/s.
inline double chain_ns_per_block(int kind) {
    switch (kind) {
        case kQuad: return 936.0;
        case kPair: return 1740.0;
        case kLatency: return 1880.0;
        default: return 2730.0;
    }
}
// Leaf-hashing rate of a full chip (bytes/s; DESIGN.md §6.2 best leaf-kernel GB/s).
inline double chip_bytes_per_s(int kind) {
    switch (kind) {
        case kQuad: return 429e9;
        case kPair: return 320e9;
        case kLatency: return 596e9;
        default: return 1.6e12;
    }
}
// Host-side feed per device (bytes/s): pinned memory crosses PCIe (zero-copy K1Q or H2D,
// ~53-57 GB/s); pageable memory goes through a memcpy into the pinned ring first;
// files are pread from the page cache by 4 threads per device.  Host memory is shared by all
// devices: RouteConstants::host_bytes_per_s caps the sum.
inline double feed_bytes_per_s(int src) {
    switch (src) {
        case kSrcHostPinned: return 55e9;
        case kSrcHostPageable: return 25e9;
        case kSrcFiles: return 25e9;
        default: return 0;
    }
}

// The model's two terms no multi-GPU node has measured yet, as estimates: the all-gather of the
// 32-byte subtree roots over RCCL (0.1 ms) and the host memory bandwidth all devices share (500
// GB/s: a 2-socket DDR5 host, ~1.2 TB/s peak, serving PCIe reads and copies).  The N = 8 bench
// line measures both and prints them as the environment variables that replace these at
// dm_create (route_constants_from_env): DEOSS_ALLGATHER_US (exchange.avg_us) and
// DEOSS_HOST_BYTES_PER_S (in_process.host_feed.all_GBps x 1e9), DESIGN.md §7.
struct RouteConstants {
    double allgather_ms = 0.10;
    double host_bytes_per_s = 500e9;
};

// A positive finite number from environment variable `name`, else `fallback` (unset, empty,
// malformed, negative or zero values are ignored).
inline double env_positive(const char* name, double fallback) {
    const char* v = std::getenv(name);
    if (!v || !*v) return fallback;
    char* end = nullptr;
    const double x = std::strtod(v, &end);
    return (end != v && *end == '\0' && std::isfinite(x) && x > 0) ? x : fallback;
}

inline RouteConstants route_constants_from_env() {
    RouteConstants k;
    k.allgather_ms = env_positive("DEOSS_ALLGATHER_US", k.allgather_ms * 1e3) * 1e-3;
    k.host_bytes_per_s = env_positive("DEOSS_HOST_BYTES_PER_S", k.host_bytes_per_s);
    return k;
}
// Fixed cost of a sharded call: a host thread per device, per-device setup, the gather of the
// 32-byte nodes and the final levels on the first device.  Measured with G virtual devices on one
// GPU (tools/shard_overhead.py, profiles/r03/LOGS.md#shard_overhead.log: +0.093 / 0.230 / 0.463 ms at
// G = 2 / 4 / 8 over one device, i.e. ~0.06 ms per device), plus 0.1 ms for the all-gather of a
// few KiB (RouteConstants::allgather_ms).  dm_exchange_timing measures that gather: 0.19 ms at G = 8 with virtual devices (the
// D2D stand-in, profiles/r04/LOGS.md#r04a_inproc.log); the RCCL gather over xGMI is recorded by the N = 8
// bench line (other_configs.in_process.sharded_object.exchange).  Sharding needs a >= 5 % gain, so
// an error in this sub-millisecond term can only change the choice for calls under ~10 ms.
inline double shard_overhead_ms(int G, double allgather_ms = RouteConstants().allgather_ms) {
    return G > 1 ? allgather_ms + 0.06 * G : 0.0;
}

// Estimated time of one device hashing m leaves (longest leaf_max bytes, `bytes` in total) that
// start at `src`; feed and hashing overlap (stripes / zero-copy), so the larger one bounds it.
inline double device_ms(uint64_t m, uint64_t bytes, uint64_t leaf_max, int src, int cus, int mode) {
    if (m == 0) return 0.0;
    const int kind = leaf_kind(m, cus, mode);
    double chain = (double)ceil_div(leaf_max + 9, 64) * chain_ns_per_block(kind) * 1e-6;
    if (kind == kQuad && ceil_div(m, kQuadLeaves) > 2 * (uint64_t)cus) chain *= 1.10;   // 2 chains per SIMD
    const double hash = std::max(chain, (double)bytes / chip_bytes_per_s(kind) * 1e3);
    const double feed = src == kSrcDevice ? 0.0 : (double)bytes / feed_bytes_per_s(src) * 1e3;
    return std::max(hash, feed);
}

// Devices a call should use: 1 = the whole call on one device; G' > 1 = sharded over G' devices.
// by_objects: a batch of independent objects, split by objects (about n/G' leaves each) instead of
// one tree's aligned blocks (plan_shards, within 1/8 of even).  busy = calls already running or
// queued on the context: a loaded context gains more from routing whole calls to idle devices than
// from splitting one, so it never shards.  est_ms (nullable, G entries): the model's time for 1..G.
// k: the all-gather and host-bandwidth terms (estimates, or measured values from the environment).
inline int route(uint64_t n, uint64_t bytes, uint64_t leaf_max, int src, int G, int cus, int mode, int busy,
                 bool by_objects = false, double* est_ms = nullptr, const RouteConstants& k = RouteConstants()) {
    int best = 1;
    double best_ms = 0;
    for (int g = 1; g <= std::max(1, G); g++) {
        const uint64_t m = by_objects ? ceil_div(n, (uint64_t)g) : plan_shards(n, g).max_leaves();
        const uint64_t b = n ? (uint64_t)((double)bytes * (double)m / (double)n) : 0;
        double t = device_ms(m, b, leaf_max, src, cus, mode);
        if (src != kSrcDevice) t = std::max(t, (double)bytes / k.host_bytes_per_s * 1e3);
        t += shard_overhead_ms(g, k.allgather_ms);
        if (est_ms) est_ms[g - 1] = t;
        if (g == 1) best_ms = t;
        else if (src != kSrcDevice && busy == 0 && n >= 2 && t < 0.95 * best_ms) {   // >= 5 % sooner
            best = g;
            best_ms = t;
        }
    }
    return best;
}

// Coalescing executor (dm_batcher): how long a free worker slot holds a burst open, counted from
// the arrival of the oldest queued request.  base_us is the caller's linger.  When other slots are
// already running batches, a burst that starts now would otherwise be cut into one small batch per
// free slot, and whatever arrives after the last slot is taken waits a whole chain (chain_us, the
// longest queued request's leaf chain).  So the wait grows with the share of busy slots: the last
// free slot of 4 holds the burst open for 9/256 of a chain (17 ms of a 32 MiB segment's 490 ms),
// an idle executor launches after base_us, and a queue whose oldest request has waited that long
// already (a freed slot under steady load) launches at once.
inline double batch_linger_us(double base_us, double chain_us, int busy, int slots) {
    if (busy <= 0 || slots <= 0) return base_us;
    const double f = (double)std::min(busy, slots) / (double)slots;
    return base_us + chain_us * f * f / 16.0;
}

// Call lanes (dm_ctx): loads[l * nphys + p] = calls running or queued on lane l of GPU p (plus
// open streams).  A call that can run anywhere goes to the GPU whose lanes carry the least load
// (GPUs scanned from `start`, the first minimum wins, so ties rotate with `start`), then to that
// GPU's least-loaded lane (the lowest lane on ties, so an idle GPU's lane 0 takes single calls).
// phys >= 0 fixes the GPU (device-memory calls, rs coders).  Returns the lane's index into loads.
inline int pick_lane(const int* loads, int nphys, int lanes, int start, int phys = -1) {
    int p = phys;
    if (p < 0) {
        p = 0;
        int best = -1;
        for (int i = 0; i < nphys; i++) {
            const int q = (start + i) % nphys;
            int x = 0;
            for (int l = 0; l < lanes; l++) x += loads[l * nphys + q];
            if (best < 0 || x < best) {
                best = x;
                p = q;
            }
        }
    }
    int g = p, best = loads[p];
    for (int l = 1; l < lanes; l++)
        if (loads[l * nphys + p] < best) {
            best = loads[l * nphys + p];
            g = l * nphys + p;
        }
    return g;
}

}  // namespace dm_plan
