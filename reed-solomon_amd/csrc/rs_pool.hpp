// rs_pool.hpp -- persistent host thread pool for the drop-in per-call API (gather of caller-owned
// symbol_t buffers into pinned staging and scatter back, rs_api.cpp). The reference API hands over
// non-contiguous, individually allocated symbols (reference src/memory/seq.c:17-46), so every call
// moves k + r separate buffers through host memory; one thread cannot saturate that.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rsamd {

class HostPool {
   public:
    explicit HostPool(int workers) {
        for (int w = 0; w < workers; ++w) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return int(th_.size()) + 1; }
    // fn(i) for every i in [0, n), on the workers and the calling thread; returns when all are done.
    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 0) return;
        if (th_.empty() || n == 1) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            busy_ = int(th_.size());
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return busy_ == 0; });
        fn_ = nullptr;
    }

   private:
    void work() {
        for (int i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
            std::lock_guard<std::mutex> lk(mu_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int n_ = 0, busy_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace rsamd
