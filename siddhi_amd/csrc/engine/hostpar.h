// Host side of the boundary's bulk copies: a push of 10^8 events is GBs of columns going to HBM, a poll of 4*10^7
// records GBs coming back. One thread copies ~10 GB/s; the host link and the pinned DMA take several times that,
// so these loops split a copy over SDG_HOST_THREADS threads (default 8) and, for pageable sources, double-buffer
// through pinned chunks so the host copy of chunk i+1 overlaps the DMA of chunk i.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
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

// f(lo, hi) over [0, n) in at most host_threads() contiguous pieces of at least `grain` items (f must not throw)
template <class F>
void par_range(int64_t n, int64_t grain, F&& f) {
    if (n <= 0) return;
    int64_t T = std::min<int64_t>(host_threads(), (n + grain - 1) / std::max<int64_t>(grain, 1));
    if (T <= 1) {
        f((int64_t)0, n);
        return;
    }
    const int64_t per = (n + T - 1) / T;
    std::vector<std::thread> th;
    th.reserve((size_t)T);
    for (int64_t t = 1; t < T; ++t) {
        const int64_t lo = t * per, hi = std::min(n, lo + per);
        if (lo < hi) th.emplace_back([&f, lo, hi] { f(lo, hi); });
    }
    f((int64_t)0, std::min(n, per));
    for (auto& x : th) x.join();
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
