// Host test of dm_batch::Queue (deoss_amd/csrc/batch_queue.hpp), the coalescing executor's queue,
// with fake workers in place of the GPU passes.  Built and run plain, with ASan/UBSan and with
// TSan by tests/test_batch_queue.py (no GPU).  Checks:
//  - every request is run exactly once and gets its own batch's result; budgets hold;
//  - an idle queue launches a lone request after the base linger, not later;
//  - a burst that starts while other slots are busy is held open (busy-scaled linger), so a burst
//    trickling in over a few ms is not cut into one batch per free slot;
//  - a queue whose oldest request has already waited launches at once;
//  - a queue that holds a full batch by the byte budget (leaves to spare) launches at once;
//  - stop() drains what is queued, then refuses new requests.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "batch_queue.hpp"

using clk = std::chrono::steady_clock;
static int fails = 0;
#define EXPECT(c, ...)                                                   \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #c); \
            std::fprintf(stderr, __VA_ARGS__);                           \
            std::fprintf(stderr, "\n");                                  \
            fails++;                                                     \
        }                                                                \
    } while (0)

struct TReq : dm_batch::Req {
    int id = 0;
    std::atomic<int> runs{0};
};

// workers: each batch "runs" for run_us, then returns rc = sum of ids (checked by the callers)
struct Pool {
    dm_batch::Queue& q;
    std::vector<std::thread> th;
    std::atomic<uint64_t> max_leaves_seen{0}, max_bytes_seen{0};
    Pool(dm_batch::Queue& q_, int n, int run_us) : q(q_) {
        for (int i = 0; i < n; i++)
            th.emplace_back([this, run_us] {
                std::vector<dm_batch::Req*> b;
                while (q.take(b)) {
                    uint64_t leaves = 0, bytes = 0;
                    int sum = 0;
                    for (dm_batch::Req* r : b) {
                        auto* t = static_cast<TReq*>(r);
                        t->runs++;
                        leaves += r->leaves;
                        bytes += r->bytes;
                        sum += t->id;
                    }
                    if (b.size() > 1) {
                        uint64_t m = max_leaves_seen.load();
                        while (leaves > m && !max_leaves_seen.compare_exchange_weak(m, leaves)) {}
                        m = max_bytes_seen.load();
                        while (bytes > m && !max_bytes_seen.compare_exchange_weak(m, bytes)) {}
                    }
                    std::this_thread::sleep_for(std::chrono::microseconds(run_us));
                    q.finish(b, sum, "");
                }
            });
    }
    void join() {
        q.stop();
        for (auto& t : th) t.join();
    }
};

static double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

// many callers, random sizes: exactly-once, own result among its batch's, budgets
static void test_exactly_once() {
    dm_batch::Queue q(4, 64, 1 << 20, 200, 936.0);
    Pool pool(q, 4, 300);
    const int N = 600;
    std::vector<TReq> reqs(N);
    std::vector<std::thread> callers;
    std::atomic<int> bad{0};
    for (int t = 0; t < 12; t++)
        callers.emplace_back([&, t] {
            std::mt19937 rng(t);
            for (int i = t; i < N; i += 12) {
                TReq& r = reqs[i];
                r.id = i;
                r.leaves = 1 + rng() % 13;
                r.bytes = (1 + rng() % 8) << 14;
                r.chain_bytes = 64 << 10;
                if (!q.submit(r) || !r.done || r.rc < i) bad++;
                if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 500));
            }
        });
    for (auto& c : callers) c.join();
    pool.join();
    EXPECT(bad == 0, "%d callers saw a wrong result", bad.load());
    for (int i = 0; i < N; i++) EXPECT(reqs[i].runs == 1, "request %d ran %d times", i, reqs[i].runs.load());
    EXPECT(pool.max_leaves_seen <= 64, "leaf budget exceeded: %llu", (unsigned long long)pool.max_leaves_seen.load());
    EXPECT(pool.max_bytes_seen <= (1u << 20), "byte budget exceeded");
    const dm_batch::Stats st = q.stats();
    EXPECT(st.requests == (uint64_t)N && st.batches >= 1 && st.batches < (uint64_t)N, "stats %llu %llu",
           (unsigned long long)st.requests, (unsigned long long)st.batches);
}

// idle queue: a lone request launches after the base linger (2 ms), well before any chain term
static void test_idle_launch() {
    dm_batch::Queue q(4, 4096, 1ull << 34, 2000, 936.0);
    Pool pool(q, 4, 100);
    TReq r;
    r.id = 7;
    r.leaves = 13;
    r.bytes = 1;
    r.chain_bytes = 32 << 20;   // a 490 ms chain: the idle queue must not wait on it
    const auto t0 = clk::now();
    EXPECT(q.submit(r) && r.rc == 7, "lone request");
    const double ms = ms_since(t0);
    EXPECT(ms >= 1.9 && ms < 60, "lone request took %.2f ms (base linger 2 ms)", ms);
    pool.join();
}

// slots busy: a burst trickling in over ~6 ms (one request per 0.25 ms) must not be cut into one
// batch per free slot -- with a 32 MiB chain estimate the free slots hold 1.9 / 7.7 / 17 ms
static void test_burst_while_busy() {
    const int slots = 4;
    dm_batch::Queue q(slots, 4096, 1ull << 40, 0, 936.0);
    Pool pool(q, slots, 120000);            // a batch "runs" 120 ms
    TReq first;                             // occupies one slot
    first.id = 1;
    first.leaves = 13;
    first.chain_bytes = 32 << 20;
    std::thread t1([&] { q.submit(first); });
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    const int n = 24;
    std::vector<TReq> burst(n);
    std::vector<clk::time_point> sent(n);
    std::vector<std::thread> th;
    // threads exist before the burst starts (thread creation under TSan on a loaded host takes
    // milliseconds); each submits at start + i x 0.25 ms
    std::atomic<bool> go{false};
    clk::time_point start;
    for (int i = 0; i < n; i++) {
        burst[i].id = 100 + i;
        burst[i].leaves = 13;
        burst[i].chain_bytes = 32 << 20;
        th.emplace_back([&, i] {
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            std::this_thread::sleep_until(start + std::chrono::microseconds(250 * i));
            sent[i] = clk::now();
            q.submit(burst[i]);
        });
    }
    start = clk::now();
    go.store(true, std::memory_order_release);
    for (auto& t : th) t.join();
    t1.join();
    const dm_batch::Stats st = q.stats();
    const double spread_ms =
        std::chrono::duration<double, std::milli>(*std::max_element(sent.begin(), sent.end()) - start).count();
    if (spread_ms > 8.0) {   // the host could not deliver the burst in its ~6 ms: the premise did not hold
        std::printf("note: burst arrived over %.1f ms (planned 6): batch-count check skipped\n", spread_ms);
    } else {
        // 1 batch for `first`, and the burst in at most 3 more (it never waits a whole 120 ms batch)
        EXPECT(st.batches <= 4, "burst of %d cut into %llu batches (arrived over %.1f ms)", n,
               (unsigned long long)st.batches - 1, spread_ms);
    }
    pool.join();
}

// a queue whose oldest request has already waited past the linger launches as soon as a slot
// frees (the linger counts from the arrival, not from when a slot became free)
static void test_old_queue_launches_at_once() {
    dm_batch::Queue q(1, 4096, 1ull << 40, 40000, 936.0);   // one slot, 40 ms base linger
    Pool pool(q, 1, 150000);                                // a batch "runs" 150 ms
    TReq a, b;
    a.id = 1;
    b.id = 2;
    a.leaves = b.leaves = 1;
    a.chain_bytes = b.chain_bytes = 64;
    std::thread ta([&] { q.submit(a); });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));   // a: 40 ms linger, then running
    clk::time_point tb;
    std::thread tbt([&] {
        tb = clk::now();
        q.submit(b);
    });
    ta.join();
    tbt.join();
    // b is queued ~10 ms into a's 150 ms run and has waited ~140 ms > 40 ms when the slot frees:
    // done ~290 ms after it was queued; a linger restarted at the free slot would make it ~330
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - tb).count();
    EXPECT(ms < 315, "b took %.1f ms", ms);
    pool.join();
}

// the byte budget ends the linger too: one slot busy, a 100 ms base linger, and four
// 1 MiB requests that fill the 4 MiB byte budget with 4 of 4096 leaves: the free slot launches
// them at once instead of holding the burst open
static void test_byte_budget_ends_linger() {
    dm_batch::Queue q(2, 4096, 4ull << 20, 100000, 936.0);
    Pool pool(q, 2, 100000);                // a batch "runs" 100 ms
    TReq first;
    first.id = 1;
    first.leaves = 1;
    first.bytes = 1;
    first.chain_bytes = 32 << 20;
    std::thread t1([&] { q.submit(first); });
    std::this_thread::sleep_for(std::chrono::milliseconds(120));  // first: 100 ms linger, then running
    std::vector<TReq> full(4);
    std::vector<std::thread> th;
    const auto t0 = clk::now();
    for (int i = 0; i < 4; i++) {
        full[i].id = 10 + i;
        full[i].leaves = 1;
        full[i].bytes = 1 << 20;
        full[i].chain_bytes = 32 << 20;
        th.emplace_back([&, i] { q.submit(full[i]); });
    }
    for (auto& t : th) t.join();
    const double ms = ms_since(t0);
    t1.join();
    // launched at once: ~100 ms of "run"; a linger of 100 ms + the busy-scaled chain term would make
    // it >= 200 ms (the margin is wide so a loaded host under ASan does not flip it)
    EXPECT(ms < 160, "a byte-full batch took %.1f ms", ms);
    const dm_batch::Stats st = q.stats();
    EXPECT(st.batches == 2, "expected 2 batches, got %llu", (unsigned long long)st.batches);
    pool.join();
}

static void test_stop_drains() {
    dm_batch::Queue q(2, 4096, 1ull << 40, 0, 936.0);
    std::vector<TReq> reqs(16);
    std::vector<std::thread> th;
    for (int i = 0; i < 16; i++) {
        reqs[i].id = i;
        reqs[i].leaves = 1;
        th.emplace_back([&, i] { q.submit(reqs[i]); });
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));   // queued, no worker yet
    Pool pool(q, 2, 100);
    q.stop();
    for (auto& t : th) t.join();
    for (int i = 0; i < 16; i++) EXPECT(reqs[i].done && reqs[i].runs == 1, "request %d not drained", i);
    TReq late;
    EXPECT(!q.submit(late), "submit after stop accepted");
    pool.join();
}

int main() {
    test_exactly_once();
    test_idle_launch();
    test_burst_while_busy();
    test_old_queue_launches_at_once();
    test_byte_budget_ends_linger();
    test_stop_drains();
    if (fails) {
        std::fprintf(stderr, "%d failure(s)\n", fails);
        return 1;
    }
    std::printf("batch queue PASS\n");
    return 0;
}
