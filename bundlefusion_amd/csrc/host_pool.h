// host_pool.h — a few persistent host threads for the frame loop's per-submap host loops over every
// frame so far (the trajectory product of Recon::apply and the queue's MatrixToPose conversions: at
// 5 000 frames ~0.3 ms each, once per submap, on the frame thread that also issues the GPU work).
// parallel_for splits [0, n) into contiguous chunks, runs one on the calling thread and waits for the
// rest; the loop bodies are independent per element, so results do not depend on the split.
// bf_set_host_threads (default 4) sets the thread count including the caller before the pool's first use;
// 1 runs everything inline.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bf {

class HostPool {
public:
    static HostPool& get() {
        static HostPool* p = new HostPool(requested());  // leaked on purpose: no join ordering at process exit
        return *p;
    }
    // threads for the pool, counting the caller (bf_set_host_threads); read once, at the pool's first use
    static std::atomic<int>& requested() {
        static std::atomic<int> n{4};
        return n;
    }
    int threads() const { return (int)workers_.size() + 1; }

    // fn(begin, end) over [0, n); serial below minPerThread elements per thread
    void parallel_for(size_t n, const std::function<void(size_t, size_t)>& fn, size_t minPerThread = 256) {
        const size_t t = std::min<size_t>((size_t)threads(), std::max<size_t>(1, n / std::max<size_t>(1, minPerThread)));
        if (t <= 1) {
            if (n) fn(0, n);
            return;
        }
        std::unique_lock<std::mutex> serial(run_);  // one parallel_for at a time (frame and bundling threads)
        const size_t chunk = (n + t - 1) / t;
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            chunk_ = chunk;
            parts_ = t - 1;
            pending_.store((int)(t - 1), std::memory_order_relaxed);
            gen_++;
        }
        cv_.notify_all();
        fn(0, std::min(n, chunk));  // part 0 on the caller
        std::unique_lock<std::mutex> lk(mu_);
        doneCv_.wait(lk, [this] { return pending_.load(std::memory_order_acquire) == 0; });
        fn_ = nullptr;
    }

private:
    explicit HostPool(const std::atomic<int>& req) {
        const int n = std::max(1, req.load());
        for (int i = 1; i < n; i++) workers_.emplace_back([this, i] { loop((size_t)i); });
        for (auto& w : workers_) w.detach();
    }
    void loop(size_t part) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t, size_t)>* fn;
            size_t b, e;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (part > parts_) continue;  // fewer parts than threads this time
                fn = fn_;
                b = std::min(n_, part * chunk_);
                e = std::min(n_, b + chunk_);
            }
            if (b < e) (*fn)(b, e);
            if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                doneCv_.notify_one();
            }
        }
    }
    std::vector<std::thread> workers_;
    std::mutex run_, mu_;
    std::condition_variable cv_, doneCv_;
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t n_ = 0, chunk_ = 0, parts_ = 0;
    uint64_t gen_ = 0;
    std::atomic<int> pending_{0};
};

}  // namespace bf
