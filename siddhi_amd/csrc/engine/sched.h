// Host side of the absent-state timers: the reference's playback / wall-clock Scheduler across all partition keys.
//
// Reference (paths under modules/siddhi-core/src/main/java/io/siddhi/core/):
//   util/Scheduler.java:71-103   TimeChangeListener.onTimeChange: every clock advance collects, over ALL keys'
//                                SchedulerStates (HashMap iteration order of PartitionStateHolder.states), the
//                                states whose queue head is due into a TreeMultimap<Long, SchedulerState>. Because
//                                SchedulerState.compareTo() always returns 0 (:360-366), only the FIRST state per
//                                distinct head time is kept; each kept state fires (sendTimerEvents :171-209) in
//                                ascending time order. The others wait for a later clock advance.
//   util/Scheduler.java:113-127  notifyAt: computeIfAbsent(partition key) + FIFO append
//   util/snapshot/state/PartitionStateHolder.java:43-70, PartitionSyncStateHolder.java:47-87: states with an empty
//                                queue are removed when returned; a removed key re-enters the map on its next notify
//   util/timestamp/TimestampGeneratorImpl.java:105-122: every event with ts >= clock advances the clock (playback)
// JDK 8 java.util.HashMap (the map's iteration order): computeIfAbsent resizes first when size > threshold, then
// links a new key at the HEAD of its bin; resize splits each bin preserving relative order. Hence iteration order
// is (bucket = spread(String.hashCode) & (capacity - 1), then most recently inserted first) -- an order this class
// keeps as a sort key instead of walking the map. Tree bins (8+ keys in one bucket of a table >= 64) are not
// modelled (the oracle does not model them either).
//
// The device runs each key's NFA (nfa.h) firing every due timer at the first clock advance that reaches it, and
// logs, per key and in order, every fire, every pop and every notify time pushed. simulate() then replays the
// global scheduler once over all keys, position by position, with each key's queue taken from those logs:
//   - a fire the scheduler makes where the key's run made it: consistent;
//   - a fire the collapse delays to a later position: still the key's result if no event of that key lies in
//     between and the fire's outcome does not depend on the later clock (LOG_FIRE_END carries the largest clock
//     it holds for) -- only its position in the delivery order changes;
//   - anything else: the key diverged. From there the simulation runs that key itself on the host (KeyRun, the
//     same nfa.h code from the key's batch-start state, with the scheduler's fire order), in lockstep.
// So one pass yields the reference's sequential execution: every key's history is either its own device run
// (shown consistent with the global order) or a host replay in that order.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include <functional>

#include "keyrun.h"
#include "nfa.h"
#include "plan.h"

namespace sdg {

// clock of one batch: every pushed event (all streams, in push order) and every advance_time point is a position
struct BatchClock {
    int64_t G = 0;
    int64_t clock0 = 0;                // currentTime() before position 0
    std::vector<int64_t> clk;          // [G] currentTime() after position g's clock update
    std::vector<uint8_t> adv;          // [G] position g runs the TimeChangeListeners (onTimeChange / live fire)
    std::vector<uint32_t> nadv;        // [G + 1] first advancing position >= g (G: none)
};

// Float.toString / Double.toString (shortest round-trip digits, Java layout): the partition key of a real value
std::string java_real_string(double x, bool is_float);
// Java String.hashCode of a UTF-8 string (as UTF-16 code units), then HashMap.hash() spreading
int32_t java_spread_hash(const std::string& s);

// a batch's rows by key (the sorted view): key k's rows are [seg_b[k], seg_e[k]), row p at batch position
// pos_off + (orig ? orig[p] : p) (ascending within a key)
struct KeyRows {
    const uint32_t* seg_b = nullptr;
    const uint32_t* seg_e = nullptr;
    int64_t K = 0;
    const uint32_t* orig = nullptr;
    int64_t pos_off = 0;
    int64_t n = 0;
    int64_t pos(int64_t p) const { return pos_off + (orig ? (int64_t)orig[p] : p); }
};

class SchedSim {
   public:
    struct Slot {
        uint32_t g;     // position of the fire in the reference's order
        uint32_t rank;  // order among the fires of that position
    };
    // (position in the key's run, scheduler, key) -> the fire's slot: open addressing, linear probing
    class RankMap {
       public:
        void reserve(size_t n) {
            size_t c = 16;
            while (c < 2 * n) c <<= 1;
            e_.assign(c, E{EMPTY, Slot{0, 0}});
            n_ = 0;
            has_empty_key_ = false;
        }
        void put(uint64_t k, Slot v) {
            if (k == EMPTY) {
                has_empty_key_ = true;
                empty_val_ = v;
                return;
            }
            if (2 * (n_ + 1) > e_.size()) grow();
            E& x = e_[at(k)];
            if (x.k == EMPTY) {
                x.k = k;
                ++n_;
            }
            x.v = v;
        }
        const Slot* find(uint64_t k) const {
            if (k == EMPTY) return has_empty_key_ ? &empty_val_ : nullptr;
            if (e_.empty()) return nullptr;
            const E& x = e_[at(k)];
            return x.k == k ? &x.v : nullptr;
        }
        void clear() { reserve(0); }
        bool empty() const { return n_ == 0 && !has_empty_key_; }

       private:
        static constexpr uint64_t EMPTY = ~0ull;
        struct E {  // key and value side by side: one cache line per probe
            uint64_t k;
            Slot v;
        };
        std::vector<E> e_;
        size_t n_ = 0;
        bool has_empty_key_ = false;
        Slot empty_val_{0, 0};
        size_t at(uint64_t k) const {  // the key's slot or the empty slot where it would go
            const size_t m = e_.size() - 1;
            size_t i = (size_t)((k ^ (k >> 29)) * 0xBF58476D1CE4E5B9ull >> 17) & m;
            while (e_[i].k != EMPTY && e_[i].k != k) i = (i + 1) & m;
            return i;
        }
        void grow() {
            std::vector<E> o;
            o.swap(e_);
            e_.assign(std::max<size_t>(16, 2 * o.size()), E{EMPTY, Slot{0, 0}});
            for (const E& x : o)
                if (x.k != EMPTY) e_[at(x.k)] = x;
        }
    };
    // one change the pass made to the scheduler model on behalf of a key (confirm() compares them)
    enum : uint8_t { OP_NOTIFY = 0, OP_POP = 1, OP_PURGE = 2, OP_FIRE = 3 };
    struct Op {
        uint32_t g;      // position (OP_FIRE and the fire's pops / pushes: the scheduler's fire position)
        uint8_t kind;
        uint8_t sched;
        int64_t t;       // OP_NOTIFY: notify time; OP_FIRE: the clock; else 0
        bool operator==(const Op& o) const { return g == o.g && kind == o.kind && sched == o.sched && t == o.t; }
    };
    struct Result {
        std::vector<uint32_t> taken;                         // keys run on the host (their device run is void)
        // optimistic pass: keys whose device run the scheduler reordered (and their fire lists in its order)
        std::vector<uint32_t> reordered, fire_off;
        std::vector<nfa::TimerFire> fires;
        std::vector<uint32_t> fire_rank;                     // [fires] each fire's rank among its position's fires
        // optimistic pass: per reordered key (trace_off like fire_off), the model changes the pass made for it:
        // its device run's event pushes, each scheduler fire (OP_FIRE) and the fire's records it applied
        std::vector<Op> trace;
        std::vector<uint32_t> trace_off;
        int64_t n_shifted_kept = 0;                          // shifted fires of keys not reordered
        RankMap rank;                                        // (position in the key's run, scheduler, key) -> slot
        int64_t n_fires = 0, n_shifted = 0;
    };
    void setup(int n_sched, bool partitioned, bool live) {
        n_sched_ = n_sched;
        partitioned_ = partitioned;
        live_ = live;
        cur_.sc.assign(n_sched, SchedState{});
    }
    bool active() const { return n_sched_ > 0; }
    // keys with queued timers (the runs a timer-only batch must include)
    void queued_keys(std::vector<uint32_t>& out) const;
    // one pass over the batch; logs sorted by (key, kseq). take_over(key) returns a started KeyRun for the key
    // (batch-start state, its rows); the caller owns it. Works on a copy of the committed state (commit()).
    // optimistic: never take over -- a key the scheduler reorders keeps its device records where they apply (as if
    // its events and fires commuted) and is listed in out.reordered with its fire list, to be rerun on the device
    // in that order before the exact (non-optimistic) pass. The optimistic pass only saves host replays; the
    // exact pass alone decides the result.
    void simulate(const BatchClock& bc, const std::vector<nfa::SchedLog>& logs, const std::vector<int32_t>& key_hash,
                  const KeyRows& rows, const std::function<KeyRun*(uint32_t)>& take_over, Result& out,
                  bool optimistic = false);
    // after the optimistic pass `res` and the device rerun of res.reordered (logs: the merged logs, by key): true
    // when every rerun key's new log makes exactly the model changes the optimistic pass made for it (same event
    // pushes, same fires at the same positions and clocks, same records inside each fire). The exact pass would
    // then retrace the optimistic one -- same model, every fire consistent, no host replay -- so its result is
    // res with the rerun keys' fires ranked at their own (now the scheduler's) positions, which confirm() writes.
    // false: run the exact pass.
    bool confirm(const std::vector<nfa::SchedLog>& logs, Result& res) const;
    void commit() { std::swap(cur_, work_); }  // work_ is rebuilt from cur_ by the next simulate()
    // snapshot / restore of the committed scheduler states (sdg_snapshot): every key's queue and HashMap entry
    void save(std::vector<uint8_t>& out) const;
    const uint8_t* load(const uint8_t* p, const uint8_t* end);  // returns the end of what it read (throws on a bad blob)
    static uint64_t rank_key(uint32_t g, int sch, uint32_t key) {
        return ((uint64_t)g << 32) ^ ((uint64_t)sch << 27) ^ (uint64_t)key * 0x9E3779B97F4A7C15ull;
    }

   private:
    // one key's SchedulerState in one scheduler: its FIFO of notify times (inline up to QI, else in a spill deque),
    // its HashMap entry (hash, insertion stamp) and creation order. Flat, indexed by dense key id.
    static constexpr int QI = 3;
    struct KS {
        int64_t a[QI];
        int32_t spill = -1;    // State::spill index while the queue holds more than QI times
        uint32_t n = 0;        // queued times
        uint32_t ver = 0;      // bumped whenever the head changes (due-heap entries of older versions are stale)
        int32_t hash = 0;
        uint64_t stamp = 0;    // insertion order into the map (iteration: newest first within a bucket)
        uint64_t cseq = 0;     // creation order (live-mode tie break)
        bool in_map = false;
    };
    // ordering key among states whose heads are equal: playback = map iteration order, live = creation order
    struct OKey {
        uint64_t a, b;
        uint32_t key;
        bool operator<(const OKey& o) const { return a != o.a ? a < o.a : (b != o.b ? b < o.b : key < o.key); }
    };
    struct DueE {
        OKey k;
        uint32_t ver;
        bool operator>(const DueE& o) const { return o.k < k; }
    };
    // one head time's states: a min-heap by OKey (lazy deletion), its keys computed for the table capacity `cap`.
    // A HashMap resize changes every state's bucket, so a heap is re-keyed when it is next used (heap_fix), not
    // every heap at every resize
    struct Heap {
        std::vector<DueE> h;
        uint64_t cap = 0;
    };
    struct SchedState {
        std::vector<KS> ks;                                 // [dense key id]
        std::map<int64_t, Heap> due;                        // head time -> min-heap of states (lazy deletion)
        uint64_t cap = 0, threshold = 0, size = 0, stamp = 0;
        size_t kend = 0;                                    // keys [0, kend) have ever entered the map (resize scans them)
        std::vector<uint32_t> bin;                          // keys per bucket (treeifyBin on a small table resizes)
    };
    struct State {
        std::vector<SchedState> sc;
        std::vector<std::deque<int64_t>> spill;             // long queues
        std::vector<int32_t> spill_free;
        uint64_t cseq = 0;
    };
    int n_sched_ = 0;
    bool partitioned_ = false, live_ = false;
    State cur_, work_;
    const std::vector<int32_t>* hash_ = nullptr;

    OKey okey(const SchedState& S, const KS& k, uint32_t key) const;
    KS& ks(SchedState& S, uint32_t key) {
        if (key >= S.ks.size()) S.ks.resize(std::max<size_t>(key + 1, S.ks.size() + S.ks.size() / 2));
        return S.ks[key];
    }
    int64_t qfront(const KS& k) const { return k.spill < 0 ? k.a[0] : work_.spill[k.spill].front(); }
    void qpush(KS& k, int64_t t);
    void qpop(KS& k);
    bool stale(const SchedState& S, const DueE& e) const { return S.ks[e.k.key].ver != e.ver; }
    // the earliest due time with a live entry (cleans stale heap tops); false when nothing is due
    bool due_front(SchedState& S, int64_t& t, OKey& k);
    void due_add(SchedState& S, uint32_t key, KS& k);
    void heap_fix(SchedState& S, Heap& H) const;  // re-key a heap built for an older capacity (drops stale entries)
    void due_del(KS& k) { ++k.ver; }
    void resize(SchedState& S);
    void notify(int sch, uint32_t key, int64_t t);  // Scheduler.notifyAt
    void pop(int sch, uint32_t key);
    void remove_if_empty(int sch, uint32_t key);
    void purge(uint32_t key);
    bool queued(int sch, uint32_t key) const {
        const SchedState& S = work_.sc[sch];
        return key < S.ks.size() && S.ks[key].n > 0;
    }
    int64_t head(int sch, uint32_t key) const { return qfront(work_.sc[sch].ks[key]); }
};

}  // namespace sdg
