// copy_pool.hpp -- host copies into the pinned staging ring, spread over a few threads (pure host
// C++, no HIP: merkle_capi.hip uses it; tests/cpp/test_copy_pool.cpp runs it under ASan and TSan).
//
// One thread's memcpy from pageable memory into pinned memory runs well below PCIe (the ring's H2D
// side), so a pageable source was copy-bound (1 MiB requests through the batcher: ~13 GiB/s).  One
// process-wide pool (DEOSS_COPY_THREADS helpers, default 7; 0 = the caller alone) serves every
// lane: a call splits its copies into pieces of at most kCopyPiece and copies them together with
// the helpers, pulling pieces from a shared index, so concurrent calls share the helpers and the
// caller always makes progress itself.  run() returns once every piece has been copied.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace dm_copy {

constexpr size_t kCopyPiece = 4ull << 20;

struct CopyItem {
    void* dst;
    const void* src;
    size_t n;
};

class CopyPool {
  public:
    static CopyPool& get() {
        static CopyPool pool(default_threads());
        return pool;
    }
    static size_t default_threads() {
        const char* v = std::getenv("DEOSS_COPY_THREADS");
        return v && *v ? (size_t)std::max(0, std::atoi(v)) : 7;
    }
    explicit CopyPool(size_t nthreads) : nthreads_(nthreads) {
        for (size_t t = 0; t < nthreads_; t++) th_.emplace_back([this] { helper(); });
    }
    CopyPool(const CopyPool&) = delete;
    CopyPool& operator=(const CopyPool&) = delete;
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(const std::vector<CopyItem>& items) {
        auto job = std::make_shared<Job>();
        for (const CopyItem& it : items)
            for (size_t o = 0; o < it.n; o += kCopyPiece)
                job->pieces.push_back({static_cast<uint8_t*>(it.dst) + o, static_cast<const uint8_t*>(it.src) + o,
                                       std::min(kCopyPiece, it.n - o)});
        if (job->pieces.empty()) return;
        const size_t helpers = std::min(nthreads_, job->pieces.size() - 1);
        if (helpers) {
            {
                std::lock_guard<std::mutex> lk(mu_);
                for (size_t h = 0; h < helpers; h++) q_.push_back(job);
            }
            if (helpers == 1) cv_.notify_one();
            else cv_.notify_all();
        }
        work(*job);
        std::unique_lock<std::mutex> lk(job->mu);
        job->cv.wait(lk, [&] { return job->done == job->pieces.size(); });
    }
    size_t threads() const { return nthreads_; }

  private:
    struct Job {
        std::vector<CopyItem> pieces;
        std::atomic<size_t> next{0};
        size_t done = 0;   // guarded by mu
        std::mutex mu;
        std::condition_variable cv;
    };
    static void work(Job& j) {
        size_t mine = 0;
        for (size_t i; (i = j.next.fetch_add(1)) < j.pieces.size(); mine++) {
            const CopyItem& p = j.pieces[i];
            std::memcpy(p.dst, p.src, p.n);
        }
        if (mine) {
            std::lock_guard<std::mutex> lk(j.mu);
            j.done += mine;
            if (j.done == j.pieces.size()) j.cv.notify_all();
        }
    }
    void helper() {
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                j = q_.front();
                q_.pop_front();
            }
            work(*j);
        }
    }
    size_t nthreads_ = 0;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Job>> q_;
    std::vector<std::thread> th_;
    bool stop_ = false;
};

}  // namespace dm_copy
