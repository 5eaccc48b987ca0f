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

#include <deque>
#include <map>
#include <set>
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
// orig ? orig[p] : pos_off + p (ascending within a key)
struct KeyRows {
    const uint32_t* seg_b = nullptr;
    const uint32_t* seg_e = nullptr;
    int64_t K = 0;
    const uint32_t* orig = nullptr;
    int64_t pos_off = 0;
    int64_t n = 0;
    int64_t pos(int64_t p) const { return orig ? (int64_t)orig[p] : pos_off + p; }
};

class SchedSim {
   public:
    struct Slot {
        uint32_t g;     // position of the fire in the reference's order
        uint32_t rank;  // order among the fires of that position
    };
    struct Result {
        std::vector<uint32_t> taken;                         // keys run on the host (their device run is void)
        // optimistic pass: keys whose device run the scheduler reordered (and their fire lists in its order)
        std::vector<uint32_t> reordered, fire_off;
        std::vector<nfa::TimerFire> fires;
        std::unordered_map<uint64_t, Slot> rank;             // (position in the key's run, scheduler, key) -> slot
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
    void commit() { cur_ = work_; }
    static uint64_t rank_key(uint32_t g, int sch, uint32_t key) {
        return ((uint64_t)g << 32) ^ ((uint64_t)sch << 27) ^ (uint64_t)key * 0x9E3779B97F4A7C15ull;
    }

   private:
    struct KS {
        std::deque<int64_t> q;
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
    struct SchedState {
        std::unordered_map<uint32_t, KS> ks;
        std::map<int64_t, std::set<OKey>> due;     // head time -> states with that head
        uint64_t cap = 0, threshold = 0, size = 0, stamp = 0;
        std::vector<uint32_t> bin;                 // keys per bucket (treeifyBin on a small table resizes)
    };
    struct State {
        std::vector<SchedState> sc;
        uint64_t cseq = 0;
        int64_t live_now = 0;
    };
    int n_sched_ = 0;
    bool partitioned_ = false, live_ = false;
    State cur_, work_;
    const std::vector<int32_t>* hash_ = nullptr;

    OKey okey(const SchedState& S, const KS& k, uint32_t key) const;
    void due_add(SchedState& S, uint32_t key, const KS& k);
    void due_del(SchedState& S, uint32_t key, const KS& k);
    void resize(SchedState& S);
    void notify(int sch, uint32_t key, int64_t t);  // Scheduler.notifyAt
    void pop(int sch, uint32_t key);
    void remove_if_empty(int sch, uint32_t key);
};

}  // namespace sdg
