// Host side of the boundary's bulk copies: a push of 10^8 events is GBs of columns going to HBM, a poll of 4*10^7
// records GBs coming back. One thread copies ~10 GB/s; the host link and the pinned DMA take several times that,
// so these loops split a copy over SDG_HOST_THREADS threads (default 8) and, for pageable sources, double-buffer
// through pinned chunks so the host copy of chunk i+1 overlaps the DMA of chunk i.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace sdg {

inline int host_threads() {
    static const int t = [] {
        const char* s = getenv("SDG_HOST_THREADS");
        int v = s ? atoi(s) : 8;
        const int hw = (int)std::thread::hardware_concurrency();
        if (hw > 0) v = std::min(v, hw);
        return std::max(1, std::min(v, 64));
    }();
    return t;
}

// A persistent pool of host_threads() - 1 workers (the caller is the last one): a multi-GB push calls par_range
// once per 32 MB bounce chunk and a poll once per column, so starting threads per call would put hundreds of thread
// launches into the boundary timings. One job at a time (callers serialise on call_mu); a call from inside a job, or
// from a process forked after the pool started, runs serially / gets a fresh pool.
class HostPool {
   public:
    static HostPool& get() {
        static std::mutex mu;
        static HostPool* p = nullptr;
        std::lock_guard<std::mutex> g(mu);
        if (!p || p->pid_ != getpid()) p = new HostPool(host_threads() - 1);  // (a forked child: the old one's
        return *p;                                                             //  workers did not survive the fork)
    }
    int workers() const { return (int)th_.size(); }
    static bool in_job() { return in_job_flag(); }
    // job(i) for i in [0, n): the workers and the caller take indices until none are left
    void run(int n, const std::function<void(int)>& job) {
        std::lock_guard<std::mutex> g(call_mu_);
        {
            std::lock_guard<std::mutex> l(mu_);
            job_ = &job;
            n_ = n;
            next_ = 0;
            done_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> l(mu_);
        done_cv_.wait(l, [&] { return done_ == n_; });
        job_ = nullptr;
    }

   private:
    explicit HostPool(int nw) : pid_(getpid()) {
        for (int i = 0; i < nw; ++i) {
            th_.emplace_back([this] { loop(); });
            th_.back().detach();  // (process exit ends them; the pool itself is never destroyed)
        }
    }
    static bool& in_job_flag() {
        static thread_local bool f = false;
        return f;
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return gen_ != seen; });
                seen = gen_;
            }
            work();
        }
    }
    void work() {  // take indices of the current job until none are left
        in_job_flag() = true;
        for (;;) {
            int i;
            const std::function<void(int)>* job;
            {
                std::lock_guard<std::mutex> l(mu_);
                if (!job_ || next_ >= n_) break;
                i = next_++;
                job = job_;
            }
            (*job)(i);
            std::lock_guard<std::mutex> l(mu_);
            if (++done_ == n_) done_cv_.notify_all();
        }
        in_job_flag() = false;
    }
    pid_t pid_;
    std::vector<std::thread> th_;
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* job_ = nullptr;
    int n_ = 0, next_ = 0, done_ = 0;
    uint64_t gen_ = 0;
};

// f(lo, hi) over [0, n) in at most host_threads() contiguous pieces of at least `grain` items (f must not throw)
template <class F>
void par_range(int64_t n, int64_t grain, F&& f) {
    if (n <= 0) return;
    const int64_t T = std::min<int64_t>(host_threads(), (n + grain - 1) / std::max<int64_t>(grain, 1));
    if (T <= 1 || HostPool::in_job()) {
        f((int64_t)0, n);
        return;
    }
    const int64_t per = (n + T - 1) / T;
    const std::function<void(int)> job = [&](int t) {
        const int64_t lo = (int64_t)t * per, hi = std::min(n, lo + per);
        if (lo < hi) f(lo, hi);
    };
    HostPool::get().run((int)T, job);
}

inline void par_memcpy(void* dst, const void* src, size_t bytes) {
    par_range((int64_t)bytes, (int64_t)4 << 20, [&](int64_t lo, int64_t hi) {
        memcpy((uint8_t*)dst + lo, (const uint8_t*)src + lo, (size_t)(hi - lo));
    });
}

// std::vector allocator that leaves new elements uninitialised: result columns are written in full right after
// they grow, and value-initialising GBs first would double the host traffic of a poll
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
template <class T>
using HostVec = std::vector<T, NoInitAlloc<T>>;

}  // namespace sdg
