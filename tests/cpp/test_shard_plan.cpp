// Host test of the multi-device partition (deoss_amd/csrc/shard_plan.hpp): no GPU, built plain and
// with ASan/UBSan by tests/test_dispatch_plan.py.
//
// For G = 1..8 devices and n = 1..600 leaves (plus large n):
//  1. the partition equals deoss_amd.sharding.plan_shards (the one-process-per-GPU rule), read from
//     the table file given as argv[1] ("G n k nb lo_0 hi_0 ... lo_{G-1} hi_{G-1}" per line);
//  2. the ranges cover [0, n) in order, every range starts on a 2^k boundary, the nodes per device
//     and their compaction offsets tile [0, nb);
//  3. composing the tree the way multi_root does -- each device reduces its leaves exactly k levels,
//     the nodes are compacted in block order and reduced to the root (>= 1 level only when k = 0) --
//     gives the same root as the oracle's single tree over all n leaves (merkletree v0.2.0 rule).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../deoss_amd/csrc/shard_plan.hpp"

extern "C" {
void or_sha256(const void* data, uint64_t len, uint8_t out[32]);
uint64_t or_reduce(const uint8_t* digests, uint64_t n, int levels, uint8_t* out);
}

static int failures = 0;
#define CHECK(cond, ...)                                      \
    do {                                                      \
        if (!(cond)) {                                        \
            if (failures++ < 20) {                            \
                std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
                std::fprintf(stderr, __VA_ARGS__);            \
                std::fprintf(stderr, "\n");                   \
            }                                                 \
        }                                                     \
    } while (0)

static std::vector<uint8_t> leaf_digests(uint64_t n) {
    std::vector<uint8_t> d(32 * n);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = i * 0x9e3779b97f4a7c15ull + n;
        or_sha256(&x, sizeof x, d.data() + 32 * i);
    }
    return d;
}

// Root of the sharded composition (multi_root's order of operations on the CPU).
static std::vector<uint8_t> sharded_root(const dm_plan::Layout& P, const std::vector<uint8_t>& leaves) {
    std::vector<uint8_t> nodes(32 * P.nb + 32);
    for (int g = 0; g < P.G; g++) {
        const uint64_t nl = P.leaves(g);
        if (nl == 0) continue;
        std::vector<uint8_t> out(32 * nl + 32);
        const uint64_t cnt = P.k == 0 ? (std::memcpy(out.data(), leaves.data() + 32 * P.leaf_lo(g), 32 * nl), nl)
                                      : or_reduce(leaves.data() + 32 * P.leaf_lo(g), nl, (int)P.k, out.data());
        CHECK(cnt == P.nodes(g), "G=%d n=%llu g=%d: %llu nodes, plan says %llu", P.G, (unsigned long long)P.n, g,
              (unsigned long long)cnt, (unsigned long long)P.nodes(g));
        if (cnt != P.nodes(g)) return {};
        std::memcpy(nodes.data() + 32 * P.node_offset(g), out.data(), 32 * cnt);
    }
    std::vector<uint8_t> root(32 * P.nb + 32);
    if (P.k > 0 && P.nb == 1) std::memcpy(root.data(), nodes.data(), 32);   // the block is the whole tree
    else or_reduce(nodes.data(), P.nb, -1, root.data());
    root.resize(32);
    return root;
}

static void check_case(int G, uint64_t n, bool compose) {
    const dm_plan::Layout P = dm_plan::plan_shards(n, G);
    CHECK(P.nb == dm_plan::ceil_shift(n, P.k), "G=%d n=%llu: nb", G, (unsigned long long)n);
    uint64_t next = 0, node_next = 0;
    for (int g = 0; g < G; g++) {
        CHECK(P.leaf_lo(g) == next, "G=%d n=%llu g=%d: gap", G, (unsigned long long)n, g);
        CHECK(P.leaf_lo(g) % (1ull << P.k) == 0 || P.leaf_lo(g) == n, "G=%d n=%llu g=%d: unaligned start", G,
              (unsigned long long)n, g);
        CHECK(P.node_offset(g) == node_next, "G=%d n=%llu g=%d: node offset", G, (unsigned long long)n, g);
        next = P.leaf_hi(g);
        node_next += P.nodes(g);
    }
    CHECK(next == n && node_next == P.nb, "G=%d n=%llu: cover", G, (unsigned long long)n);
    if (n >= (uint64_t)G) {   // balance: within 1/8 of an even split
        const uint64_t even = dm_plan::ceil_div(n, (uint64_t)G);
        CHECK(8 * P.max_leaves() <= 9 * even, "G=%d n=%llu: imbalance %llu vs %llu", G, (unsigned long long)n,
              (unsigned long long)P.max_leaves(), (unsigned long long)even);
        for (int g = 0; g < G; g++) CHECK(P.nodes(g) >= 1, "G=%d n=%llu g=%d: no block", G, (unsigned long long)n, g);
    }
    if (compose) {
        const std::vector<uint8_t> leaves = leaf_digests(n);
        std::vector<uint8_t> want(32 * n + 32);
        or_reduce(leaves.data(), n, -1, want.data());
        const std::vector<uint8_t> got = sharded_root(P, leaves);
        CHECK(got.size() == 32 && std::memcmp(got.data(), want.data(), 32) == 0, "G=%d n=%llu k=%u: root differs", G,
              (unsigned long long)n, P.k);
    }
}

int main(int argc, char** argv) {
    // 1. the table from deoss_amd.sharding.plan_shards
    uint64_t rows = 0;
    if (argc > 1) {
        std::ifstream f(argv[1]);
        CHECK(f.good(), "cannot open %s", argv[1]);
        std::string line;
        while (std::getline(f, line)) {
            std::istringstream is(line);
            int G;
            uint64_t n, k, nb;
            if (!(is >> G >> n >> k >> nb)) continue;
            const dm_plan::Layout P = dm_plan::plan_shards(n, G);
            CHECK(P.k == k && P.nb == nb, "G=%d n=%llu: C++ k=%u nb=%llu, Python k=%llu nb=%llu", G,
                  (unsigned long long)n, P.k, (unsigned long long)P.nb, (unsigned long long)k, (unsigned long long)nb);
            for (int g = 0; g < G; g++) {
                uint64_t lo, hi;
                is >> lo >> hi;
                CHECK(P.leaf_lo(g) == lo && P.leaf_hi(g) == hi, "G=%d n=%llu g=%d: C++ [%llu,%llu) Python [%llu,%llu)",
                      G, (unsigned long long)n, g, (unsigned long long)P.leaf_lo(g), (unsigned long long)P.leaf_hi(g),
                      (unsigned long long)lo, (unsigned long long)hi);
            }
            rows++;
        }
        CHECK(rows >= 8 * 600, "table has %llu rows", (unsigned long long)rows);
    }
    // 2 + 3. invariants and the composed root
    for (int G = 1; G <= 8; G++)
        for (uint64_t n = 1; n <= 600; n++) check_case(G, n, true);
    for (int G = 1; G <= 8; G++)
        for (uint64_t n : {1023ull, 1024ull, 1025ull, 4096ull, 32768ull, 100000ull, (1ull << 18) + 3})
            check_case(G, n, n <= 4096);
    // the configured layouts (BASELINE configs[3]: 1 TiB at 32 MiB over 8 GPUs; weak scaling 256 per GPU)
    CHECK(dm_plan::plan_shards(32768, 8).k == 12 && dm_plan::plan_shards(32768, 8).nb == 8, "configs[3] layout");
    CHECK(dm_plan::plan_shards(2048, 8).k == 8 && dm_plan::plan_shards(2048, 8).nb == 8, "weak-scaling layout");
    // 4. call lanes (dm_plan::pick_lane): loads are lane-major, loads[l * nphys + p]
    {
        const int idle[16] = {};
        CHECK(dm_plan::pick_lane(idle, 8, 2, 0) == 0 && dm_plan::pick_lane(idle, 8, 2, 5) == 5, "idle: lane 0 of start");
        CHECK(dm_plan::pick_lane(idle, 1, 4, 0) == 0, "one GPU idle: lane 0");
        const int one[4] = {1, 0, 0, 0};                  // 1 GPU, 4 lanes, lane 0 busy
        CHECK(dm_plan::pick_lane(one, 1, 4, 0) == 1, "lane 1 when lane 0 is busy");
        const int two[4] = {1, 1, 0, 0};
        CHECK(dm_plan::pick_lane(two, 1, 4, 0) == 2, "lowest idle lane");
        const int full[2] = {3, 2};                       // 1 GPU, 2 lanes, both busy: the lighter one
        CHECK(dm_plan::pick_lane(full, 1, 2, 0) == 1, "least-loaded lane");
        // 2 GPUs x 2 lanes: GPU 0 carries 1 (lane 0), GPU 1 carries 2 -> GPU 0's idle lane 1
        const int g2[4] = {1, 1, 0, 1};                   // lane 0: GPU0=1, GPU1=1; lane 1: GPU0=0, GPU1=1
        CHECK(dm_plan::pick_lane(g2, 2, 2, 0) == 2 && dm_plan::pick_lane(g2, 2, 2, 1) == 2, "least-loaded GPU, then lane");
        // 8 concurrent calls on 8 idle GPUs with rotating starts land on 8 different GPUs (lane 0)
        int loads[16] = {};
        for (int i = 0; i < 8; i++) loads[dm_plan::pick_lane(loads, 8, 2, i)]++;
        bool spread = true;
        for (int p = 0; p < 8; p++) spread &= loads[p] == 1 && loads[8 + p] == 0;
        CHECK(spread, "8 calls over 8 GPUs");
        for (int i = 0; i < 8; i++) loads[dm_plan::pick_lane(loads, 8, 2, i)]++;   // the next 8: every lane 1
        for (int p = 0; p < 8; p++) spread &= loads[8 + p] == 1;
        CHECK(spread, "16 calls over 16 lanes");
        CHECK(dm_plan::pick_lane(loads, 8, 2, 3, 6) == 6, "fixed GPU: its lane 0 on ties");
    }
    {   // batcher linger: the caller's base while no slot is busy, growing with the busy share
        const double chain = 490e3;                           // one 32 MiB segment chain, us
        CHECK(dm_plan::batch_linger_us(2000, chain, 0, 4) == 2000, "idle executor: base linger");
        CHECK(dm_plan::batch_linger_us(0, chain, 0, 4) == 0, "idle executor, no base: at once");
        double prev = 2000;
        for (int busy = 1; busy <= 4; busy++) {
            const double w = dm_plan::batch_linger_us(2000, chain, busy, 4);
            CHECK(w > prev, "busy %d: linger grows", busy);
            prev = w;
        }
        const double last = dm_plan::batch_linger_us(0, chain, 3, 4);  // the last free slot of 4
        CHECK(last > 15e3 && last < 20e3, "last free slot of 4: %.0f us (9/256 of a chain)", last);
        CHECK(dm_plan::batch_linger_us(0, chain, 1, 32) < 50, "1 busy slot of 32: negligible");
        CHECK(dm_plan::batch_linger_us(0, chain, 9, 4) == dm_plan::batch_linger_us(0, chain, 4, 4), "busy capped");
    }
    if (failures) {
        std::fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    std::printf("shard plan OK: %llu table rows, G = 1..8 x n = 1..600 composed\n", (unsigned long long)rows);
    return 0;
}
