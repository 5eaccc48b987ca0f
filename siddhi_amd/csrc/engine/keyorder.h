// The order in which a partition delivers an event of a stream that has no partition key.
//
// Reference: PartitionStreamReceiver.send(ComplexEvent) (core/partition/PartitionStreamReceiver.java:274-283) sends
// such an event to every key of PartitionRuntimeImpl.getPartitionKeys() (core/partition/PartitionRuntimeImpl.java:
// 404-407) = new HashSet<>(partitionKeys.keySet()), where partitionKeys is the ConcurrentHashMap<String, Long> that
// initPartition (:346-366) fills with every key a keyed stream of the partition has delivered. The keys' results are
// therefore delivered in that HashSet's iteration order, which this class reproduces (JDK 8, one thread):
//   * the map: 16 bins at the first key; a new key goes to the TAIL of bin spread(h) & (n - 1); once the count
//     reaches 0.75 n the table doubles, and a bin split keeps its `lastRun` tail in order at the head of its side and
//     prepends every node before it (their order reverses); a put that walks 8 nodes of a bin on a table < 64
//     presizes (doubling until tableSizeFor(3n + 1) <= 0.75 n') instead of building a tree bin;
//   * the copy: a HashMap of tableSizeFor(max((int)(size / .75f) + 1, 16)) bins filled in the map's order (tail
//     appends, order-kept doubling when a bin of a table < 64 reaches 9 keys), iterated bin by bin.
// Tree bins (a put that walks >= 8 nodes of a map bin on a table >= 64, or a set bin reaching 9 keys at capacity
// >= 64: rare at these load factors short of colliding hashes) are not modelled: they are detected (tree_bins())
// and the engine refuses the broadcast, as the oracle does, instead of delivering a possibly wrong order. Keys are the engine's dense key ids; h is the Java String.hashCode of the key's
// toString after HashMap.hash spreading (java_spread_hash).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace sdg {

class PartitionKeyOrder {
   public:
    // partitionKeys.put(key, time) of initPartition, for EVERY event a keyed stream delivers to key k: a new key is
    // linked in; an existing one only matters when putVal walks 8 nodes of its bin (treeifyBin on a small table)
    void add(uint32_t k, int32_t h) {
        h &= 0x7fffffff;
        if (k < live_.size() && live_[k]) {
            if (bins_.size() < 64) {
                const std::vector<E>& b = bins_[(uint32_t)h & (bins_.size() - 1)];
                if (b.size() >= 8) {
                    size_t p = 0;
                    while (p < b.size() && b[p].k != k) ++p;
                    if (p + 1 >= 8) presize();
                }
            } else {  // putVal's binCount >= TREEIFY_THRESHOLD on a table >= 64: treeifyBin builds a tree bin
                const std::vector<E>& b = bins_[(uint32_t)h & (bins_.size() - 1)];
                if (b.size() >= 8) {
                    size_t p = 0;
                    while (p < b.size() && b[p].k != k) ++p;
                    if (p + 1 >= 8) tree_ = true;
                }
            }
            return;
        }
        if (k >= live_.size()) live_.resize(std::max<size_t>(k + 1, live_.size() * 2), 0);
        live_[k] = 1;
        if (bins_.empty()) {
            bins_.assign(16, {});
            size_ctl_ = 12;
        }
        std::vector<E>& b = bins_[(uint32_t)h & (bins_.size() - 1)];
        const size_t before = b.size();
        b.push_back(E{k, h});
        if (before >= 8) {
            if (bins_.size() < 64) presize();
            else tree_ = true;
        }
        if (++count_ >= size_ctl_) grow();
        dirty_ = true;
        ++ver_;
    }
    int64_t size() const { return count_; }
    // changes whenever order() may change (a new key, a resize)
    uint64_t version() const { return ver_; }
    // a tree bin was (or would be) built in the map or its HashSet copy: order() is not the JDK's order then
    bool tree_bins() const { return tree_; }
    // the keys in getPartitionKeys() order (valid until the next add)
    const std::vector<uint32_t>& order() {
        if (!dirty_) return order_;
        dirty_ = false;
        order_.clear();
        std::vector<int32_t> hs;
        for (const auto& b : bins_)
            for (const E& x : b) {
                order_.push_back(x.k);
                hs.push_back(x.h);
            }
        // the HashSet's capacity: HashMap(c) then add() in the map's order; an add that makes a bin 9 long calls
        // treeifyBin, which on a table < 64 doubles it ONCE (order-keeping split) and on a larger one builds a tree
        // bin. The next add into a bin still >= 9 long triggers again.
        int64_t cap = pow2_at_least(std::max<int64_t>((int64_t)((float)count_ / 0.75f) + 1, 16));
        {
            std::vector<uint32_t> cnt((size_t)cap, 0);
            for (size_t i = 0; i < hs.size(); ++i) {
                if (++cnt[(uint32_t)hs[i] & (cap - 1)] < 9) continue;
                if (cap >= 64) {
                    tree_ = true;
                    continue;
                }
                cap *= 2;
                cnt.assign((size_t)cap, 0);
                for (size_t j = 0; j <= i; ++j) ++cnt[(uint32_t)hs[j] & (cap - 1)];
            }
        }
        if (cap != (int64_t)bins_.size()) {  // bins of the map are not the set's bins: stable regroup
            std::vector<uint32_t> idx(order_.size());
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = (uint32_t)i;
            std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
                return ((uint32_t)hs[a] & (cap - 1)) < ((uint32_t)hs[b] & (cap - 1));
            });
            std::vector<uint32_t> o(order_.size());
            for (size_t i = 0; i < idx.size(); ++i) o[i] = order_[idx[i]];
            order_.swap(o);
        }
        return order_;
    }
    // snapshot: bin count, then every bin's keys and hashes (count and sizeCtl follow from them)
    template <class W>
    void save(W& w) const {
        w.template put<uint64_t>(bins_.size());
        w.template put<int64_t>(size_ctl_);
        for (const auto& b : bins_) {
            w.template put<uint32_t>((uint32_t)b.size());
            for (const E& x : b) {
                w.template put<uint32_t>(x.k);
                w.template put<int32_t>(x.h);
            }
        }
    }
    template <class R>
    void load(R& r) {
        *this = PartitionKeyOrder();
        const uint64_t nb = r.template get<uint64_t>();
        size_ctl_ = r.template get<int64_t>();
        if (nb > (1ull << 31) || (nb & (nb - 1))) throw_corrupt();
        bins_.resize(nb);
        for (auto& b : bins_) {
            const uint32_t m = r.template get<uint32_t>();
            for (uint32_t i = 0; i < m; ++i) {
                E x;
                x.k = r.template get<uint32_t>();
                x.h = r.template get<int32_t>();
                b.push_back(x);
                if (nb >= 64 && b.size() >= 9) tree_ = true;  // the 9th put walked 8 nodes: a tree bin
                if (x.k >= live_.size()) live_.resize((size_t)x.k + 1, 0);
                live_[x.k] = 1;
                ++count_;
            }
        }
        dirty_ = true;
        ++ver_;
    }

   private:
    struct E {
        uint32_t k;
        int32_t h;
    };
    std::vector<std::vector<E>> bins_;
    std::vector<uint8_t> live_;
    int64_t count_ = 0, size_ctl_ = 0;
    std::vector<uint32_t> order_;
    bool dirty_ = true;
    uint64_t ver_ = 0;
    bool tree_ = false;
    static int64_t pow2_at_least(int64_t c) {
        int64_t n = 1;
        while (n < c) n <<= 1;
        return n;
    }
    static void throw_corrupt();
    void presize() {  // treeifyBin on a table < 64: tryPresize(n << 1)
        const int64_t c = pow2_at_least(3 * (int64_t)bins_.size() + 1);
        while (c > size_ctl_) grow();
        dirty_ = true;
        ++ver_;
    }
    void grow() {  // ConcurrentHashMap.transfer
        const size_t n = bins_.size();
        std::vector<std::vector<E>> nb(2 * n);
        for (size_t i = 0; i < n; ++i) {
            const std::vector<E>& f = bins_[i];
            if (f.empty()) continue;
            // lastRun: the start of the longest tail that goes to one side
            size_t last = f.size() - 1;
            const bool side_last = (f[last].h & (int32_t)n) != 0;
            while (last > 0 && ((f[last - 1].h & (int32_t)n) != 0) == side_last) --last;
            std::vector<E>& lo = nb[i];
            std::vector<E>& hi = nb[i + n];
            for (size_t p = last; p-- > 0;) ((f[p].h & (int32_t)n) ? hi : lo).push_back(f[p]);  // prepended: reversed
            std::vector<E>& run = side_last ? hi : lo;
            run.insert(run.end(), f.begin() + (long)last, f.end());
        }
        bins_.swap(nb);
        size_ctl_ = (int64_t)(2 * n) - (int64_t)(n >> 1);
    }
};

}  // namespace sdg
