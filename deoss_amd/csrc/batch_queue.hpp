// batch_queue.hpp -- the coalescing executor's request queue (pure host C++, no HIP: batcher.inl
// runs its GPU passes on top of it; tests/cpp/test_batch_queue.cpp drives it with fake workers,
// plain, ASan/UBSan and TSan).
//
// Callers block in submit() until a worker has run their request.  Workers (one per slot) block
// in take(), which returns the next batch: everything queued, oldest first, up to the leaf and
// byte budgets, after holding a burst open for dm_plan::batch_linger_us from the oldest request's
// arrival.  That wait is re-evaluated whenever a slot finishes (the busy count changes), and it
// ends at once when the queue holds a full batch by either budget (leaves or bytes) or on stop().  finish() hands a batch's result back to
// its callers.  After stop(), take() drains what is queued and then returns false; submit()
// refuses new requests.
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "shard_plan.hpp"

namespace dm_batch {

struct Req {
    uint64_t leaves = 0;       // leaves this request adds to a batch (the leaf budget)
    uint64_t bytes = 0;        // bytes it adds (the byte budget)
    uint64_t chain_bytes = 0;  // its longest leaf (the linger's chain estimate)
    int rc = 0;
    std::string err;
    bool done = false;
    std::chrono::steady_clock::time_point arrived{};
};

struct Stats {
    uint64_t requests = 0, batches = 0, max_batch = 0;
};

class Queue {
  public:
    // chain_ns_per_block: one 64-byte block of one leaf chain (dm_plan::chain_ns_per_block)
    Queue(int nslots, uint64_t max_leaves, uint64_t max_bytes, double linger_us, double chain_ns_per_block)
        : nslots_(std::max(1, nslots)), max_leaves_(max_leaves), max_bytes_(max_bytes), linger_us_(linger_us),
          chain_ns_(chain_ns_per_block) {}
    Queue(const Queue&) = delete;
    Queue& operator=(const Queue&) = delete;

    // Blocks until a worker has finished r; false (r untouched) when the queue is stopping.
    bool submit(Req& r) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (stop_) return false;
            r.arrived = std::chrono::steady_clock::now();
            q_.push_back(&r);
            q_leaves_ += r.leaves;
            q_bytes_ += r.bytes;
            st_.requests++;
        }
        cv_work_.notify_all();   // idle slots start; a lingering one re-checks the budget
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return r.done; });
        return true;
    }

    // Worker side: the next batch into `batch` (cleared first); false once stopped and drained.
    bool take(std::vector<Req*>& batch) {
        batch.clear();
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_work_.wait(lk, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return false;   // stop requested and nothing left to drain
            while (!stop_ && !q_.empty() && !full()) {
                double chain_us = 0;
                if (busy_ > 0) {
                    uint64_t longest = 0;
                    for (const Req* r : q_) longest = std::max(longest, r->chain_bytes);
                    chain_us = (double)dm_plan::ceil_div(longest + 9, 64) * chain_ns_ * 1e-3;
                }
                const double w = dm_plan::batch_linger_us(linger_us_, chain_us, busy_, nslots_);
                const auto until = q_.front()->arrived + std::chrono::microseconds((int64_t)w);
                if (std::chrono::steady_clock::now() >= until) break;
                const int busy0 = busy_;
                cv_work_.wait_until(lk, until, [&] {
                    return stop_ || q_.empty() || full() || busy_ != busy0;
                });
            }
            if (!q_.empty()) break;   // else another slot took them meanwhile
        }
        uint64_t leaves = 0, bytes = 0;
        while (!q_.empty()) {
            Req* r = q_.front();
            if (!batch.empty() && (leaves + r->leaves > max_leaves_ || bytes + r->bytes > max_bytes_)) break;
            batch.push_back(r);
            leaves += r->leaves;
            bytes += r->bytes;
            q_leaves_ -= r->leaves;
            q_bytes_ -= r->bytes;
            q_.pop_front();
        }
        busy_++;
        st_.batches++;
        st_.max_batch = std::max<uint64_t>(st_.max_batch, batch.size());
        if (!q_.empty()) cv_work_.notify_one();   // another slot can start on the rest
        return true;
    }

    // Worker side: the batch's result to its callers.
    void finish(const std::vector<Req*>& batch, int rc, const std::string& err) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            busy_--;
            for (Req* r : batch) {
                r->rc = rc;
                r->err = err;
                r->done = true;
            }
        }
        cv_done_.notify_all();
        cv_work_.notify_all();   // a lingering slot re-evaluates with one busy slot fewer
    }

    void stop() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_work_.notify_all();
    }

    Stats stats() {
        std::lock_guard<std::mutex> lk(mu_);
        return st_;
    }

  private:
    // a whole batch's worth is queued (either budget reached): the linger ends, the batch launches
    bool full() const { return q_leaves_ >= max_leaves_ || q_bytes_ >= max_bytes_; }

    const int nslots_;
    const uint64_t max_leaves_, max_bytes_;
    const double linger_us_, chain_ns_;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::deque<Req*> q_;
    uint64_t q_leaves_ = 0;   // leaves queued
    uint64_t q_bytes_ = 0;    // bytes queued
    int busy_ = 0;            // slots running a batch
    bool stop_ = false;
    Stats st_;
};

}  // namespace dm_batch
