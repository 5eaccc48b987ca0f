// Generic keyed NFA: the per-partition-key state machine of the reference's state processors, executed by
// one GPU lane per key over that key's events (time order) with the partial-match state in a bounded arena in
// HBM that persists across batches. Semantics follow (paths under modules/siddhi-core/src/main/java/io/siddhi/core/):
//   StreamPreStateProcessor.java      init :178-194, addState :214-227, addEveryState :230-247,
//                                     resetState :288-305, updateState :308-323, expireEvents :326-361,
//                                     processAndReturn :364-403, isExpired :118-129
//   StreamPostStateProcessor.java     process :64-83
//   CountPreStateProcessor.java       processAndReturn :53-95, addState :97-125, startStateReset :168-181,
//                                     updateState :183-193;  CountPostStateProcessor.java :39-89
//   LogicalPreStateProcessor.java     :43-178;  LogicalPostStateProcessor.java :59-87
//   AbsentStreamPreStateProcessor     addState :80-103, addEveryState :105-124, resetState :126-148,
//     .java                           process (TIMER) :151-227, sendEvent :238-254, processAndReturn :257-274,
//                                     partitionCreated :291-308;  AbsentStreamPostStateProcessor.java :36-56
//   AbsentLogicalPreStateProcessor    addState :77-97, addEveryState :99-118, process (TIMER) :121-209,
//     .java                           sendEvent :230-250, processAndReturn :262-319, partitionCreated :331-351,
//                                     partnerCanProceed :353-388;  AbsentLogicalPostStateProcessor.java :37-49
//   Scheduler.java                    notifyAt :113-127 (per-key FIFO of notify times), sendTimerEvents :171-209
//   receivers                         state/receiver/*.java (stabilizeStates), MultiProcessStreamReceiver.java
// Object identity is kept: StateEvents and StreamEvent nodes are arena objects referenced by index, so clones
// share StreamEvent chains exactly as StateEventCloner does (count-state aliasing, CountPatternTestCase :53-111).
// Memory is reclaimed by a mark-sweep pass over the lists at event boundaries; running out of arena space sets
// the key's overflow flag (reported as SDG_ERR_CAPACITY, never a silent drop).
//
// Timers (absent states). Each absent processor has a Scheduler; a key's notify times for it are a FIFO in the
// arena. Which key fires at which batch position is decided by the reference's global scheduler (all keys, one
// TreeMultimap per clock advance, Scheduler.java:71-103). A key run either derives its fires itself ("ideal"
// mode: a due head fires at the first clock advance that reaches it -- exact for a single key, and for keys whose
// due times never coincide with another key's) or replays an explicit fire list computed by the host scheduler
// simulation (sched.h) from the fire/notify log every run writes. The engine iterates the two to a fixpoint.
#pragma once
#include <stdint.h>

#include "eval.h"
#include "plan.h"

#define SDG_HD __host__ __device__ __forceinline__

namespace sdg {
namespace nfa {

enum : uint8_t { T_CURRENT = 0, T_EXPIRED = 1 };
constexpr int16_t NIL = -1;

struct Layout {
    int32_t ns, nn, nr, lcap, n_states, n_cols, n_sched, qcap;
    int64_t off_ps, off_pend, off_newe, off_ret, off_tq, off_tqt, off_se, off_nd, off_rc, bytes;
    int32_t se_bytes, rc_bytes;
};

struct KHead {
    int32_t flags;       // bit0 overflow, bit1 key initialised, bit2 (KH_HOST) the host runs the key (spilled)
    int32_t se_free, nd_free, rc_free;
    int32_t se_used, nd_used, rc_used;
    uint32_t kseq;       // scheduler log records written by this key in the current run
    int32_t screate;     // scheduler states created by this key (creation order, live-mode tie break)
    int32_t pad;
};
constexpr int32_t KH_HOST = 4;

// IX: the arena's object index type -- int16_t on the device (compact arenas, <= 4096 partials per key), int32_t
// for the keys the host takes over when they outgrow that (spilled keys, engine.cpp)
template <class IX>
struct PStateT {
    uint8_t changed, initialized, success, start_reset, active, started, returned, pad;
    int64_t last_sched;    // AbsentStreamPreState.lastScheduledTime
    IX pn, nw;
    IX pad2[2];
    int64_t last_arrival;  // AbsentLogicalPreStateProcessor.LogicalStreamPreState.lastArrivalTime
};
using PState = PStateT<int16_t>;

// one scheduler's notify-time FIFO of one key (Scheduler.SchedulerState.toNotifyQueue)
template <class IX>
struct TQT {
    int64_t earliest;  // first batch position at which the current head may fire (ideal mode)
    int32_t created;   // KHead::screate when this scheduler state was (re)created
    IX h, n;
};
using TQ = TQT<int16_t>;

// scheduler log (device -> host scheduler simulation): every fire a key run performs and every notify time it
// pushes, in the key's order (kseq)
// LOG_PURGE: @purge destroyed the key's states before the event at g (its SchedulerStates leave every scheduler)
enum : uint8_t { LOG_PUSH = 0, LOG_FIRE = 1, LOG_POP = 2, LOG_FIRE_END = 3, LOG_PURGE = 4 };
constexpr uint8_t ORIGIN_EVENT = 0xFF;
struct SchedLog {
    uint32_t key;
    uint32_t kseq;
    uint32_t g;       // batch position: the event being processed, or where the fire happened
    uint8_t type;     // LOG_PUSH / LOG_FIRE / LOG_POP (a fire dequeued t) / LOG_FIRE_END (t: the largest clock the
                      // fire would have behaved identically with -- the scheduler may run it later)
    uint8_t sched;    // PUSH: scheduler the time went to; FIRE / POP: scheduler that fired
    uint8_t origin;   // PUSH: ORIGIN_EVENT (processing the event at g, incl. partitionCreated) or the scheduler
                      //       whose fire at g pushed it
    uint8_t pad;
    int64_t t;        // PUSH: notify time; FIRE: the clock the fire ran with
};
// explicit fire (host -> device): scheduler `sched` of this key fires at position g with currentTime() = clock
struct TimerFire {
    uint32_t g;
    int32_t sched;
    int64_t clock;
};
// per-run timer inputs
struct TimerIn {
    int64_t G;                    // batch positions: every pushed event (all streams) + advance_time points
    const int64_t* clk;           // [G] currentTime() at position g (after its clock advance)
    const uint32_t* nadv;         // [G + 1] first clock-advance position >= g (G: none)
    int64_t clock0;               // currentTime() before position 0
    int32_t live;                 // wall-clock mode: fires in (time, creation) order, the fire's clock = its time
    SchedLog* log;                // nullptr: no scheduler in this query
    unsigned long long* log_count;
    int64_t log_cap;
};

// @purge of the key's partition (PartitionRuntimeImpl.java:368-401, modelled as in the oracle): before an event
// whose clock reading exceeds the key's last activity by idle.period (from the partition's first initPartition +
// interval on), the key's states are destroyed and initPartition runs again
struct PurgeIn {
    const int64_t* clk;           // [G] currentTime() at position g; nullptr: no purge
    int64_t from;                 // first clock reading a purge pass can see
    int64_t idle;                 // idle.period (ms)
    int64_t last;                 // the key's currentTime at its last event (INT64_MIN: none yet); updated by the run
};

template <class IX>
struct SET {
    IX free_next;
    uint8_t type, mark;
    int32_t pad;
    int64_t ts;
    // IX slot[n_states] follows
};

template <class IX>
struct NodeT {
    IX rec, next, free_next;
    uint8_t mark, pad;
};

template <class IX>
struct RecT {
    uint32_t nullmask;
    uint8_t mark, pad;
    IX free_next;
    int64_t ts;
    // int64_t vals[n_cols] follows
};

template <class IX = int16_t>
inline Layout make_layout(int n_states, int n_cols, int ns, int n_sched = 0) {
    using SE = SET<IX>;
    using Node = NodeT<IX>;
    using Rec = RecT<IX>;
    using PState = PStateT<IX>;
    using TQ = TQT<IX>;
    constexpr int W = (int)sizeof(IX);
    Layout L;
    L.ns = ns;
    L.nn = ns * 4;
    L.nr = ns * 2;
    L.lcap = ns;
    L.n_states = n_states;
    L.n_cols = n_cols;
    L.n_sched = n_sched;
    L.qcap = n_sched ? ns : 0;
    L.se_bytes = (int32_t)((sizeof(SE) + W * n_states + 7) & ~7);
    L.rc_bytes = (int32_t)(sizeof(Rec) + 8 * n_cols);
    int64_t o = sizeof(KHead);
    L.off_ps = o;
    o += (int64_t)sizeof(PState) * n_states;
    L.off_pend = o;
    o += (int64_t)W * L.lcap * n_states;
    L.off_newe = o;
    o += (int64_t)W * L.lcap * n_states;
    L.off_ret = o;  // StateEvents one processAndReturn call returns (emitted after its loop)
    o += (int64_t)W * L.lcap;
    o = (o + 7) & ~7;
    L.off_tq = o;
    o += (int64_t)sizeof(TQ) * n_sched;
    L.off_tqt = o;
    o += (int64_t)8 * L.qcap * n_sched;
    L.off_se = o;
    o += (int64_t)L.se_bytes * L.ns;
    L.off_nd = o;
    o += (int64_t)sizeof(Node) * L.nn;
    o = (o + 7) & ~7;
    L.off_rc = o;
    o += (int64_t)L.rc_bytes * L.nr;
    L.bytes = (o + 127) & ~127;
    return L;
}

template <bool TM, class IX = int16_t>
struct CtxT;

// bytecode accessor over a StateEvent (StateEvent.getStreamEvent(int[]) + attribute)
template <bool TM, class IX = int16_t>
struct SEAccT {
    CtxT<TM, IX>* c;
    IX se;
    SDG_HD void load(int slot, int col, int chain, uint8_t kind, int64_t* v, bool* null);
    SDG_HD bool slot_empty(int slot, int chain);
    SDG_HD void agg(int, int64_t* v, bool* n) { *v = 0; *n = true; }  // aggregators: the post pass only
};

// TM: the query has absent states (timer code compiled in); without them the kernel keeps its registers for
// the plain processors
template <bool TM, class IX>
struct CtxT {
    using SE = SET<IX>;
    using Node = NodeT<IX>;
    using Rec = RecT<IX>;
    using PState = PStateT<IX>;
    using TQ = TQT<IX>;
    const Plan* P;
    const Instr* code;
    const int64_t* consts;
    Layout L;
    uint8_t* base;  // this key's arena
    int64_t* stk;
    int stride;
    // output sink (device buffers)
    int64_t* emit_ts;
    int64_t* emit_vals;
    uint32_t* emit_nulls;
    int64_t* emit_seq;
    int64_t* emit_sub;
    uint32_t* emit_key;
    uint8_t* emit_round;  // scheduler round of the run (nullptr: not recorded)
    uint8_t round;
    unsigned long long* emit_count;
    int64_t emit_cap;
    int* flags;
    uint32_t key;
    uint8_t* emit_flags = nullptr;  // [emit_cap] per record: 1 = the key was purged since its previous record (the
                                    // selector's aggregator states restart before it); nullptr: not recorded
    bool purge_pending = false;     // purged, no record emitted since
    int64_t seq_base;   // sequence number of batch position 0
    int64_t cur_seq;
    int64_t cur_sub;
    // timers
    TimerIn T;
    PurgeIn purge{};
    const TimerFire* fires;  // explicit fire list of this key (used when nfires >= 0; -1: ideal mode)
    int32_t nfires, fi;
    int64_t clock;           // currentTime()
    int64_t clk_hi;          // during a fire: the largest clock that gives the same result (see LOG_FIRE_END)
    int64_t pos;             // batch position being processed (-1: before position 0)
    int32_t fsched;          // scheduler whose fire is running (-1: event processing)

    // ---- arena access ------------------------------------------------------------------------------------
    SDG_HD KHead& head() { return *(KHead*)base; }
    SDG_HD PState& ps(int p) { return ((PState*)(base + L.off_ps))[p]; }
    SDG_HD IX* pend(int p) { return (IX*)(base + L.off_pend) + (int64_t)p * L.lcap; }
    SDG_HD IX* newe(int p) { return (IX*)(base + L.off_newe) + (int64_t)p * L.lcap; }
    SDG_HD SE& se(int i) { return *(SE*)(base + L.off_se + (int64_t)i * L.se_bytes); }
    SDG_HD IX* slots(int i) { return (IX*)((uint8_t*)&se(i) + sizeof(SE)); }
    SDG_HD Node& nd(int i) { return ((Node*)(base + L.off_nd))[i]; }
    SDG_HD Rec& rc(int i) { return *(Rec*)(base + L.off_rc + (int64_t)i * L.rc_bytes); }
    SDG_HD TQ& tq(int s) { return ((TQ*)(base + L.off_tq))[s]; }
    SDG_HD int64_t* tqt(int s) { return (int64_t*)(base + L.off_tqt) + (int64_t)s * L.qcap; }
    SDG_HD int64_t* vals(int i) { return (int64_t*)((uint8_t*)&rc(i) + sizeof(Rec)); }
    SDG_HD bool ovf() { return head().flags & 1; }
    SDG_HD void set_ovf() { head().flags |= 1; }

    SDG_HD void arena_init() {
        KHead& h = head();
        h.flags = 0;
        h.se_used = h.nd_used = h.rc_used = 0;
        for (int i = 0; i < L.ns; ++i) se(i).free_next = (IX)(i + 1 < L.ns ? i + 1 : NIL);
        for (int i = 0; i < L.nn; ++i) nd(i).free_next = (IX)(i + 1 < L.nn ? i + 1 : NIL);
        for (int i = 0; i < L.nr; ++i) rc(i).free_next = (IX)(i + 1 < L.nr ? i + 1 : NIL);
        h.se_free = 0;
        h.nd_free = 0;
        h.rc_free = 0;
        h.kseq = 0;
        h.screate = 0;
        for (int p = 0; p < L.n_states; ++p) {
            PState& s = ps(p);
            s.changed = s.initialized = s.success = s.start_reset = s.started = s.returned = 0;
            s.active = 1;
            s.last_sched = 0;
            s.last_arrival = 0;
            s.pn = s.nw = 0;
        }
        for (int q = 0; q < L.n_sched; ++q) {
            tq(q).h = tq(q).n = 0;
            tq(q).created = 0;
            tq(q).earliest = 0;
        }
    }

    SDG_HD IX se_alloc() {
        KHead& h = head();
        if (h.se_free == NIL) { set_ovf(); return NIL; }
        IX i = (IX)h.se_free;
        h.se_free = se(i).free_next;
        h.se_used++;
        SE& s = se(i);
        s.type = T_CURRENT;
        s.ts = -1;
        IX* sl = slots(i);
        for (int k = 0; k < L.n_states; ++k) sl[k] = NIL;
        return i;
    }
    SDG_HD IX nd_alloc(IX rec) {
        KHead& h = head();
        if (h.nd_free == NIL) { set_ovf(); return NIL; }
        IX i = (IX)h.nd_free;
        h.nd_free = nd(i).free_next;
        h.nd_used++;
        nd(i).rec = rec;
        nd(i).next = NIL;
        return i;
    }
    SDG_HD IX rc_alloc() {
        KHead& h = head();
        if (h.rc_free == NIL) { set_ovf(); return NIL; }
        IX i = (IX)h.rc_free;
        h.rc_free = rc(i).free_next;
        h.rc_used++;
        return i;
    }

    // mark-sweep over every list (the only roots between events)
    SDG_HD void gc() {
        for (int i = 0; i < L.ns; ++i) se(i).mark = 0;
        for (int i = 0; i < L.nn; ++i) nd(i).mark = 0;
        for (int i = 0; i < L.nr; ++i) rc(i).mark = 0;
        for (int p = 0; p < L.n_states; ++p) {
            for (int l = 0; l < 2; ++l) {
                IX* lst = l ? newe(p) : pend(p);
                int n = l ? ps(p).nw : ps(p).pn;
                for (int j = 0; j < n; ++j) {
                    IX s = lst[j];
                    if (se(s).mark) continue;
                    se(s).mark = 1;
                    IX* sl = slots(s);
                    for (int k = 0; k < L.n_states; ++k)
                        for (IX x = sl[k]; x != NIL && !nd(x).mark; x = nd(x).next) {
                            nd(x).mark = 1;
                            rc(nd(x).rec).mark = 1;
                        }
                }
            }
        }
        KHead& h = head();
        h.se_free = h.nd_free = h.rc_free = NIL;
        h.se_used = h.nd_used = h.rc_used = 0;
        for (int i = L.ns - 1; i >= 0; --i) {
            if (se(i).mark) { h.se_used++; continue; }
            se(i).free_next = (IX)h.se_free;
            h.se_free = i;
        }
        for (int i = L.nn - 1; i >= 0; --i) {
            if (nd(i).mark) { h.nd_used++; continue; }
            nd(i).free_next = (IX)h.nd_free;
            h.nd_free = i;
        }
        for (int i = L.nr - 1; i >= 0; --i) {
            if (rc(i).mark) { h.rc_used++; continue; }
            rc(i).free_next = (IX)h.rc_free;
            h.rc_free = i;
        }
    }

    // ---- StateEvent helpers ------------------------------------------------------------------------------
    SDG_HD IX clone(IX o) {  // StateEventCloner.copyStateEvent: slots shared
        IX n = se_alloc();
        if (n == NIL) return NIL;
        SE& a = se(n);
        SE& b = se(o);
        a.type = b.type;
        a.ts = b.ts;
        IX* sa = slots(n);
        IX* sb = slots(o);
        for (int k = 0; k < L.n_states; ++k) sa[k] = sb[k];
        return n;
    }
    SDG_HD IX chain_at(IX s, int pos, int idx) {  // StateEvent.getStreamEvent(int[])
        IX e = slots(s)[pos];
        if (e == NIL) return NIL;
        if (idx >= 0) {
            for (int i = 1; i <= idx; ++i) {
                e = nd(e).next;
                if (e == NIL) return NIL;
            }
            return e;
        }
        if (idx == -1) {
            while (nd(e).next != NIL) e = nd(e).next;
            return e;
        }
        if (idx == -2) {
            if (nd(e).next == NIL) return NIL;
            while (nd(nd(e).next).next != NIL) e = nd(e).next;
            return e;
        }
        int len = 0;
        for (IX x = e; x != NIL; x = nd(x).next) ++len;
        int k = len + idx;
        if (k < 0) return NIL;
        for (int i = 0; i < k; ++i) e = nd(e).next;
        return e;
    }
    SDG_HD void add_event(IX s, int pos, IX node) {
        IX a = slots(s)[pos];
        if (a == NIL) { slots(s)[pos] = node; return; }
        while (nd(a).next != NIL) a = nd(a).next;
        nd(a).next = node;
    }
    SDG_HD void remove_last_event(IX s, int pos) {
        IX a = slots(s)[pos];
        if (a == NIL) return;
        while (nd(a).next != NIL) {
            if (nd(nd(a).next).next == NIL) { nd(a).next = NIL; return; }
            a = nd(a).next;
        }
        slots(s)[pos] = NIL;
    }

    // ---- scheduler ---------------------------------------------------------------------------------------
    SDG_HD bool is_absent(int p) const {  // instanceof AbsentPreStateProcessor
        return TM && (P->st[p].kind == PK_ABSENT || (P->st[p].kind == PK_LOGICAL && P->st[p].absent));
    }
    // one slot of a shared output counter. On the GPU the lanes of the wave that reach this point together (the
    // exec mask: every lane emitting at this call site now) share ONE atomic -- a per-record atomic on one counter
    // serialises in L2 at ~10^8/s, which was most of nfa_k's time on match-heavy queries (C3: 10^7 matches per
    // flush). On the host (tests/native, KeyRun replays) a plain increment.
    SDG_HD static unsigned long long reserve(unsigned long long* counter) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint64_t m = __ballot(1);
        const int leader = __ffsll((unsigned long long)m) - 1;
        const int lane = __lane_id();
        unsigned long long base = 0;
        if (lane == leader) base = atomicAdd(counter, (unsigned long long)__popcll(m));
        base = __shfl(base, leader);
        const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        return base + (unsigned long long)__popcll(m & below);
#else
        return __atomic_fetch_add(counter, 1ull, __ATOMIC_RELAXED);
#endif
    }
    SDG_HD void log_rec(uint8_t type, int sch, uint8_t origin, int64_t t) {
        if (!TM || !T.log) return;
        const unsigned long long i = reserve(T.log_count);
        const uint32_t kseq = head().kseq++;
        if ((int64_t)i >= T.log_cap) {  // counted: the host grows the log and reruns
            __atomic_fetch_or(flags + 5, 1, __ATOMIC_RELAXED);
            return;
        }
        SchedLog& r = T.log[i];
        r.key = key;
        r.kseq = kseq;
        r.g = (uint32_t)pos;
        r.type = type;
        r.sched = (uint8_t)sch;
        r.origin = origin;
        r.pad = 0;
        r.t = t;
    }
    // Scheduler.notifyAt :113-127 for this key (SchedulerState created on demand: computeIfAbsent)
    SDG_HD void notify_at(int sch, int64_t t) {
        if (!TM) return;
        TQ& q = tq(sch);
        if (q.n >= L.qcap) { set_ovf(); return; }
        if (q.n == 0) {
            q.created = ++head().screate;
            q.h = 0;
            // a head pushed by a fire can still fire at this position in a scheduler whose TimeChangeListener
            // runs later (playback) / in the same live advance; one pushed while processing an event, only at
            // the next clock advance
            q.earliest = (fsched >= 0 && (T.live || sch > fsched)) ? pos : pos + 1;
        }
        tqt(sch)[(q.h + q.n) % L.qcap] = t;
        q.n++;
        log_rec(LOG_PUSH, sch, fsched >= 0 ? (uint8_t)fsched : ORIGIN_EVENT, t);
    }
    SDG_HD int64_t tq_pop(int sch) {
        TQ& q = tq(sch);
        const int64_t t = tqt(sch)[q.h];
        q.h = (IX)((q.h + 1) % L.qcap);
        q.n--;
        return t;
    }
    // StreamEventFactory.newInstance(): timestamp -1, every attribute null
    SDG_HD IX empty_node() {
        IX r = rc_alloc();
        if (r == NIL) return NIL;
        rc(r).ts = -1;
        rc(r).nullmask = 0xFFFFFFFFu;
        for (int c = 0; c < L.n_cols; ++c) vals(r)[c] = 0;
        return nd_alloc(r);
    }
    // an AbsentStreamPreState that is empty and not initialised is destroyed when its holder returns it
    // (PartitionStateHolder.returnState): its lastScheduledTime restarts from 0. Only that field of a destroyed
    // state is ever read again (start states are initialised, so never destroyed), so it is the one reset here,
    // at the end of each event / fire (every getState/returnState scope of the reference has ended by then)
    // Any other state its holder would destroy (canDestroy: both lists empty, not initialised, no lastArrivalTime)
    // restarts from its defaults too. Its flags are rewritten before they are read (SuccessCondition), read only
    // by updateState of start states, which are initialised (StartStateReset), or set once per key
    // (partitionCreated: Started), so this changes no result -- it keeps snapshots (sdg_snapshot_states) equal to
    // the reference's maps. Run at the end of each event.
    SDG_HD void destroyed_gc() {
        for (int p = 0; p < L.n_states; ++p) {
            PState& s = ps(p);
            if (s.pn || s.nw || s.initialized || s.last_arrival) continue;
            s.success = s.start_reset = s.started = 0;
        }
    }
    SDG_HD void absent_gc() {
        if (!TM) return;
        for (int i = 0; i < P->n_sched; ++i) {
            const int p = P->sched_state[i];
            const StateRow& r = P->st[p];
            if ((TM && r.kind == PK_ABSENT) && !r.is_start && ps(p).pn == 0 && ps(p).nw == 0) ps(p).last_sched = 0;
        }
    }

    // ---- list helpers ------------------------------------------------------------------------------------
    SDG_HD void push(IX* lst, IX& n, IX v) {
        if (n >= L.lcap) { set_ovf(); return; }
        lst[n++] = v;
    }
    SDG_HD static void erase(IX* lst, IX& n, int j) {
        for (int i = j; i + 1 < n; ++i) lst[i] = lst[i + 1];
        --n;
    }
    SDG_HD void pend_push_newe(int p) {  // newAndEvery.sort(eventTimeComparator) + pending.addAll + clear
        PState& s = ps(p);
        IX* nw = newe(p);
        for (int i = 1; i < s.nw; ++i) {  // stable insertion sort; ts == -1 sorts last
            IX v = nw[i];
            int64_t tv = se(v).ts;
            int j = i - 1;
            while (j >= 0) {
                int64_t tj = se(nw[j]).ts;
                bool gt = (tv == -1) ? false : (tj == -1 ? true : tj > tv);
                if (!gt) break;
                nw[j + 1] = nw[j];
                --j;
            }
            nw[j + 1] = v;
        }
        IX* pd = pend(p);
        for (int i = 0; i < s.nw; ++i) push(pd, s.pn, nw[i]);
        s.nw = 0;
    }

    // ---- filters / selector ------------------------------------------------------------------------------
    SDG_HD bool filter(int p, IX s) {
        const StateRow& r = P->st[p];
        const FastPred& f = P->fast[p];
        SEAccT<TM, IX> acc{this, s};
        if (f.kind == FP_TRUE) return true;
        if (f.kind != FP_NONE) return fast_pass(f, acc);
        return pass(code, r.filter, consts, acc, stk, stride);
    }

    SDG_HD void emit(IX s) {  // QuerySelector.processNoGroupBy for one StateEvent (insert current events)
        // (timer emissions: cur_seq = the position of the fire, cur_sub negative -- before that event's own)
        if (se(s).type != T_CURRENT) return;
        unsigned long long slot = reserve(emit_count);
        if ((int64_t)slot >= emit_cap) {
            __atomic_fetch_or(flags, 1, __ATOMIC_RELAXED);
            return;
        }
        emit_ts[slot] = se(s).ts;
        if (emit_flags) emit_flags[slot] = purge_pending ? 1 : 0;
        purge_pending = false;
        emit_seq[slot] = cur_seq;
        emit_sub[slot] = cur_sub++;
        emit_key[slot] = key;
        if (emit_round) emit_round[slot] = round;
        uint32_t nm = 0;
        SEAccT<TM, IX> acc{this, s};
        for (int j = 0; j < P->n_out; ++j) {
            int64_t v;
            bool nl;
            run(code, P->out_prog[j], consts, acc, stk, stride, &v, &nl);
            emit_vals[(int64_t)j * emit_cap + slot] = v;
            if (nl) nm |= 1u << j;
        }
        emit_nulls[slot] = nm;
    }

    // ---- pre-state processors ----------------------------------------------------------------------------
    SDG_HD bool is_expired(IX s, int64_t now) {
        if (!P->has_within) return false;
        for (int i = 0; i < P->n_states; ++i) {
            if (!P->st[i].is_start) continue;
            IX e = slots(s)[i];
            if (e != NIL) {
                int64_t d = rc(nd(e).rec).ts - now;
                if (d < 0) d = -d;
                if (d > P->within_ms) return true;
            }
        }
        return false;
    }

    SDG_HD void add_state(int p, IX s) {
        // iterative: a count state with min 0 forwards at once (CountPreStateProcessor.addState :97-125 ->
        // CountPostStateProcessor.processMinCountReached), which may reach another such state. The every clone of
        // each level is pushed before the forward chain continues: the chain only touches lists of later states,
        // the clone the (earlier) every-group start, so the order of the two does not change any list.
        for (int level = 0; level <= MAX_STATES; ++level) {
            const StateRow& r = P->st[p];
            PState& st = ps(p);
            if (r.kind == PK_LOGICAL) {  // LogicalPreStateProcessor.addState :43-62
                if ((TM && r.absent) && !st.active) return;  // AbsentLogicalPreStateProcessor.addState :77-97
                int q = r.partner;
                if (r.is_start || r.seq) {
                    if (st.nw == 0) push(newe(p), st.nw, s);
                    if (ps(q).nw == 0) push(newe(q), ps(q).nw, s);
                } else {
                    push(newe(p), st.nw, s);
                    push(newe(q), ps(q).nw, s);
                }
                if ((TM && r.absent) && !r.is_start && r.waiting_ms != -1) {
                    notify_at(r.sched, se(s).ts + r.waiting_ms);
                    const StateRow& pr = P->st[q];
                    if (pr.kind == PK_LOGICAL && (TM && pr.absent)) notify_at(pr.sched, se(s).ts + pr.waiting_ms);
                }
                return;
            }
            if ((TM && r.kind == PK_ABSENT)) {  // AbsentStreamPreStateProcessor.addState :80-103
                if (!st.active) return;
                if (r.seq) st.nw = 0;
                push(newe(p), st.nw, s);
                if (!r.is_start) {
                    st.last_sched = se(s).ts + r.waiting_ms;
                    notify_at(r.sched, st.last_sched);
                }
                return;
            }
            if (r.seq) {
                if (st.nw == 0) push(newe(p), st.nw, s);
            } else {
                push(newe(p), st.nw, s);
            }
            if (!(r.kind == PK_COUNT && r.min_count == 0 && slots(s)[p] == NIL)) return;
            if (r.selector_after) {
                ps(p).changed = 1;
                ps(p).returned = 1;
            }
            if (r.next_every >= 0) add_every_state(r.next_every, s);
            if (r.next < 0) return;
            p = r.next;
        }
        set_ovf();
    }

    SDG_HD void add_every_state(int p, IX s) {
        const StateRow& r = P->st[p];
        IX c = clone(s);
        if (c == NIL) return;
        se(c).type = T_CURRENT;
        if (r.kind == PK_LOGICAL && (TM && r.absent)) {  // AbsentLogicalPreStateProcessor.addEveryState :99-118
            if (slots(c)[p] != NIL) se(c).ts = rc(nd(slots(c)[p]).rec).ts;  // the last arrived event's time
            slots(c)[p] = NIL;
            slots(c)[r.partner] = NIL;
            push(newe(p), ps(p).nw, c);
            push(newe(r.partner), ps(r.partner).nw, c);
            return;
        }
        for (int i = p; i < L.n_states; ++i) slots(c)[i] = NIL;
        push(newe(p), ps(p).nw, c);
        if (r.kind == PK_LOGICAL) {  // :65-84
            slots(c)[r.partner] = NIL;
            push(newe(r.partner), ps(r.partner).nw, c);
        }
        if ((TM && r.kind == PK_ABSENT)) {  // AbsentStreamPreStateProcessor.addEveryState :105-124
            ps(p).last_sched = se(s).ts + r.waiting_ms;
            notify_at(r.sched, ps(p).last_sched);
        }
    }

    SDG_HD void init(int p) {  // StreamPreStateProcessor.init :178-194
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        if (r.is_start && (!st.initialized || r.next_every >= 0 || (r.seq && r.next >= 0 && is_absent(r.next)))) {
            IX s = se_alloc();
            if (s == NIL) return;
            add_state(p, s);
            st.initialized = 1;
        }
    }

    SDG_HD void reset_state(int p) {
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        if (r.kind == PK_LOGICAL) {  // :87-125
            int q = r.partner;
            if (r.logical_or || st.pn == ps(q).pn) {
                st.pn = 0;
                ps(q).pn = 0;
                if (r.is_start && st.nw == 0) {
                    if (r.seq && r.next_every < 0 && r.next >= 0 && ps(r.next).pn != 0) return;
                    init(p);
                }
            }
            return;
        }
        if ((TM && r.kind == PK_ABSENT)) {  // AbsentStreamPreStateProcessor.resetState :126-148
            st.pn = 0;
            if (r.is_start) {
                if (r.seq && r.next_every < 0 && r.next >= 0 && ps(r.next).pn != 0) return;
                init(p);
            }
            return;
        }
        st.pn = 0;  // :288-305
        if (r.is_start && st.nw == 0) {
            if (r.seq && r.next_every < 0 && r.next >= 0 && ps(r.next).pn != 0) return;
            init(p);
        }
    }

    SDG_HD void update_state(int p) {
        const StateRow& r = P->st[p];
        if (r.kind == PK_COUNT && ps(p).start_reset) {  // CountPreStateProcessor.updateState :183-193
            ps(p).start_reset = 0;
            init(p);
        }
        pend_push_newe(p);
        if (r.kind == PK_LOGICAL) pend_push_newe(r.partner);
    }

    SDG_HD void expire_events(int p, int64_t now) {  // :326-361
        PState& st = ps(p);
        IX expired = NIL;
        IX* pd = pend(p);
        while (st.pn > 0 && is_expired(pd[0], now)) {
            IX s = pd[0];
            erase(pd, st.pn, 0);
            if (se(s).type != T_EXPIRED) { se(s).type = T_EXPIRED; expired = s; }
        }
        IX* nw = newe(p);
        for (int j = 0; j < st.nw;) {
            IX s = nw[j];
            if (is_expired(s, now)) {
                erase(nw, st.nw, j);
                if (se(s).type != T_EXPIRED) { se(s).type = T_EXPIRED; expired = s; }
            } else {
                ++j;
            }
        }
        int we = P->st[p].within_every;
        if (expired != NIL && we >= 0) {
            add_every_state(we, expired);
            update_state(we);
        }
    }

    SDG_HD void start_state_reset(int p) {  // CountPreStateProcessor.startStateReset :168-181
        ps(p).start_reset = 1;
        // the reference then calls countPostStateProcessor.thisStatePreProcessor.startStateReset() -- itself --
        // whenever its own post has a callback: unbounded recursion (StackOverflowError); reported as an error
        if (P->st[p].callback >= 0) set_ovf();
    }

    // ---- post-state processors ---------------------------------------------------------------------------
    SDG_HD void post_stream(int p, IX s) {  // StreamPostStateProcessor.process :64-83
        const StateRow& r = P->st[p];
        ps(p).changed = 1;
        se(s).ts = rc(nd(slots(s)[p]).rec).ts;
        if (r.selector_after) ps(p).returned = 1;
        if (r.next >= 0) add_state(r.next, s);
        if (r.next_every >= 0) add_every_state(r.next_every, s);
        if (r.callback >= 0) start_state_reset(r.callback);
    }
    SDG_HD void count_min_reached(int p, IX s) {  // CountPostStateProcessor.processMinCountReached
        const StateRow& r = P->st[p];
        if (r.selector_after) {
            ps(p).changed = 1;
            ps(p).returned = 1;
        }
        if (r.next >= 0) add_state(r.next, s);
        if (r.next_every >= 0) add_every_state(r.next_every, s);
    }
    SDG_HD void post_count(int p, IX s) {  // CountPostStateProcessor.process :39-79
        const StateRow& r = P->st[p];
        IX e = slots(s)[p];
        int n = 1;
        while (nd(e).next != NIL) { ++n; e = nd(e).next; }
        ps(p).success = 1;
        se(s).ts = rc(nd(e).rec).ts;
        if (n >= r.min_count) {
            if (r.seq) {
                if (r.next >= 0) add_state(r.next, s);
                if (n != r.max_count) add_state(p, s);
            } else if (n == r.min_count) {
                count_min_reached(p, s);
            }
            if (n == r.max_count) ps(p).changed = 1;
        }
    }
    SDG_HD bool partner_can_proceed(int q, IX s) {  // AbsentLogicalPreStateProcessor.partnerCanProceed :353-388
        const StateRow& r = P->st[q];
        PState& st = ps(q);
        if (r.seq && r.next_every < 0 && st.last_arrival > 0) return false;
        if (r.waiting_ms == -1) {
            if (r.next_every < 0) return slots(s)[q] == NIL;  // not received by the absent processor
            if (st.last_arrival > 0) {                          // every
                st.last_arrival = 0;
                init(q);
                return false;
            }
            return true;
        }
        return slots(s)[q] != NIL;
    }
    SDG_HD void post_absent(int p, IX s) {  // AbsentStreamPostStateProcessor.process :36-56
        const StateRow& r = P->st[p];
        ps(p).changed = 1;
        const int64_t ts = rc(nd(slots(s)[p]).rec).ts;
        se(s).ts = ts;
        ps(p).returned = 1;
        if (r.is_start && r.next_every == p) add_every_state(p, s);
        ps(p).last_sched = ts + r.waiting_ms;  // updateLastArrivalTime :68-78
        notify_at(r.sched, ps(p).last_sched);
    }
    SDG_HD void post_logical(int p, IX s) {  // LogicalPostStateProcessor.process :59-87
        const StateRow& r = P->st[p];
        if ((TM && r.absent)) {  // AbsentLogicalPostStateProcessor.process :37-49
            ps(p).changed = 1;
            ps(p).returned = 1;
            ps(p).last_arrival = rc(nd(slots(s)[p]).rec).ts;  // updateLastArrivalTime
            return;
        }
        if (!r.logical_or) {
            const StateRow& pr = P->st[r.partner];
            const bool proceed = (pr.kind == PK_LOGICAL && (TM && pr.absent)) ? partner_can_proceed(r.partner, s)
                                                                       : slots(s)[r.partner] != NIL;
            if (proceed) post_stream(p, s);
            else ps(p).changed = 1;
        } else {
            post_stream(p, s);
            if (P->st[r.partner].selector_after && r.last == r.partner) ps(r.partner).returned = 1;
        }
    }
    SDG_HD void post(int p, IX s) {
        switch (P->st[p].kind) {
            case PK_COUNT: post_count(p, s); break;
            case PK_LOGICAL: post_logical(p, s); break;
            case PK_ABSENT:
                if (TM) post_absent(p, s);
                break;
            default: post_stream(p, s); break;
        }
    }

    // process(StateEvent): filters then post
    SDG_HD void process_se(int p, IX s) {
        ps(p).changed = 0;
        if (filter(p, s)) post(p, s);
    }

    // processAndReturn; the receiver hands the returned StateEvents to the selector after the loop
    // (StateMultiProcessStreamReceiver.processAndClear :47-68), so they are collected first
    // AbsentLogicalPreStateProcessor.processAndReturn :262-319: a matching event removes the absence candidate; it
    // never returns a match itself
    SDG_HD void alogic_process_and_return(int p, IX rec) {
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        if (!st.active) return;
        IX* pd = pend(p);
        for (int j = 0; j < st.pn;) {
            if (ovf()) return;
            const IX s = pd[j];
            if (r.logical_or && slots(s)[r.partner] != NIL) {
                erase(pd, st.pn, j);
                continue;
            }
            const IX cur = slots(s)[p];
            const IX n = nd_alloc(rec);
            if (n == NIL) return;
            slots(s)[p] = n;
            process_se(p, s);
            if (r.waiting_ms != -1 || (r.seq && !r.logical_or && r.next_every >= 0)) slots(s)[p] = cur;
            bool removed = false;
            if (ps(r.last).returned) {  // passed the filter: no longer an absence candidate
                ps(r.last).returned = 0;
                erase(pd, st.pn, j);
                removed = true;
                if (r.seq) {  // partner's pending list .remove(stateEvent): first occurrence
                    PState& qs = ps(r.partner);
                    IX* qp = pend(r.partner);
                    for (int i = 0; i < qs.pn; ++i)
                        if (qp[i] == s) { erase(qp, qs.pn, i); break; }
                }
            }
            if (!st.changed) {
                slots(s)[p] = cur;
                if (r.seq) {
                    if (removed) { set_ovf(); return; }  // the reference would throw (iterator.remove twice)
                    erase(pd, st.pn, j);
                    removed = true;
                }
            }
            if (!removed) ++j;
        }
    }

    SDG_HD void process_and_return(int p, IX rec, bool selector) {
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        if (r.kind == PK_LOGICAL && (TM && r.absent)) {
            alogic_process_and_return(p, rec);
            return;
        }
        // AbsentStreamPreStateProcessor.processAndReturn :257-274: inactive -> nothing; otherwise the stream loop,
        // whose returned events are discarded (an arriving event only cancels absence candidates)
        if ((TM && r.kind == PK_ABSENT)) {
            if (!st.active) return;
            selector = false;
        }
        IX* pd = pend(p);
        const int last = r.last;
        IX* ret = (IX*)(base + L.off_ret);
        int nret = 0;
        for (int j = 0; j < st.pn;) {
            if (ovf()) return;
            IX s = pd[j];
            if (r.kind == PK_COUNT) {  // :60-66
                if ((p + 1 < L.n_states && slots(s)[p + 1] != NIL) || (p + 2 < L.n_states && slots(s)[p + 2] != NIL)) {
                    erase(pd, st.pn, j);
                    continue;
                }
                IX n = nd_alloc(rec);
                if (n == NIL) return;
                add_event(s, p, n);
                st.success = 0;
            } else if (r.kind == PK_LOGICAL) {
                if (r.logical_or && slots(s)[r.partner] != NIL) {
                    erase(pd, st.pn, j);
                    continue;
                }
                IX n = nd_alloc(rec);
                if (n == NIL) return;
                slots(s)[p] = n;
            } else {
                IX n = nd_alloc(rec);
                if (n == NIL) return;
                slots(s)[p] = n;
            }
            process_se(p, s);
            if (ps(last).returned) {
                ps(last).returned = 0;
                if (nret < L.lcap) ret[nret++] = s;
                else { set_ovf(); return; }
            }
            bool erased = false;
            if (st.changed) {
                erase(pd, st.pn, j);
                erased = true;
            }
            if (r.kind == PK_COUNT) {
                if (!st.success) {
                    remove_last_event(s, p);
                    if (r.seq) {
                        if (erased) { set_ovf(); return; }  // the reference would throw (iterator.remove twice)
                        erase(pd, st.pn, j);
                        erased = true;
                    }
                }
            } else if (!st.changed) {
                slots(s)[p] = NIL;
                if (r.seq) {  // SEQUENCE: no state change -> dropped (removeOnNoStateChange; false for absent)
                    if (r.kind != PK_ABSENT) {
                        erase(pd, st.pn, j);
                        erased = true;
                    }
                    if (r.kind != PK_LOGICAL && P->st[p].callback >= 0) start_state_reset(P->st[p].callback);
                }
            }
            if (!erased) ++j;
        }
        // processAndReturn's getState / returnState scope ends here: a state its holder can destroy now is dropped
        // (PartitionStateHolder.returnState), its flags with it -- a later addState in this event starts afresh
        if (!st.pn && !st.nw && !st.initialized && !st.last_arrival) st.success = st.start_reset = st.started = 0;
        if (selector)
            for (int i = 0; i < nret; ++i) emit(ret[i]);
    }

    // ---- timers ------------------------------------------------------------------------------------------
    // AbsentStreamPreStateProcessor.sendEvent :238-254
    SDG_HD void absent_send(int p, IX s) {
        const StateRow& r = P->st[p];
        if (r.selector_after) emit(s);
        if (r.next >= 0) add_state(r.next, s);
        if (r.next_every >= 0) add_every_state(r.next_every, s);
        else if (r.is_start) ps(p).active = 0;
        if (r.callback >= 0) start_state_reset(r.callback);
    }
    // AbsentStreamPreStateProcessor.process(ComplexEventChunk) :151-227 for one TIMER event at time `now`
    SDG_HD void absent_timer(int p, int64_t now) {
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        if (!st.active) return;
        bool initialize = r.is_start && st.nw == 0 && st.pn == 0;
        if (initialize && r.seq && r.next_every < 0 && st.last_sched > 0) initialize = false;
        if (initialize) {
            const IX s = se_alloc();
            if (s == NIL) return;
            add_state(p, s);
        } else if (r.seq && st.nw != 0) {
            reset_state(p);
        }
        update_state(p);
        IX* pd = pend(p);
        IX* ret = (IX*)(base + L.off_ret);
        int nret = 0;
        for (int j = 0; j < st.pn;) {
            const IX s = pd[j];
            if (is_expired(s, now)) {
                erase(pd, st.pn, j);
                if (r.within_every >= 0 && r.next_every != p) {
                    if (r.next_every < 0) { set_ovf(); return; }  // the reference: NullPointerException
                    add_every_state(r.next_every, s);
                }
                continue;
            }
            const int64_t ts = se(s).ts;
            if ((ts == -1 && now >= st.last_sched) || (ts != -1 && now >= ts + r.waiting_ms)) {
                erase(pd, st.pn, j);
                se(s).ts = now;
                if (nret >= L.lcap) { set_ovf(); return; }
                ret[nret++] = s;
                continue;
            }
            ++j;
        }
        if (r.within_every >= 0) update_state(r.within_every);
        const bool not_processed = nret == 0;
        for (int i = 0; i < nret && !ovf(); ++i) absent_send(p, ret[i]);
        if (clock > r.waiting_ms + now) {
            st.last_sched = clock + r.waiting_ms;
            clk_hi = clock;  // the result depends on the clock itself
        } else if (r.waiting_ms + now < clk_hi) {
            clk_hi = r.waiting_ms + now;  // any clock up to waiting + now takes the same branch
        }
        if (not_processed && st.last_sched < now) {
            st.last_sched = now + r.waiting_ms;
            notify_at(r.sched, st.last_sched);
        }
    }
    // AbsentLogicalPreStateProcessor.sendEvent :230-250
    SDG_HD void alogic_send(int p, IX s) {
        const StateRow& r = P->st[p];
        if (r.selector_after) emit(s);
        if (r.next >= 0) add_state(r.next, s);
        if (r.next_every >= 0) {
            add_every_state(r.next_every, s);
        } else if (r.is_start) {
            ps(p).active = 0;
            if (r.logical_or && is_absent(r.partner)) ps(r.partner).active = 0;
        }
        if (r.callback >= 0) start_state_reset(r.callback);
    }
    // AbsentLogicalPreStateProcessor.process(ComplexEventChunk) :121-209 for one TIMER event at time `now`
    SDG_HD void alogic_timer(int p, int64_t now) {
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        if (!st.active) return;
        bool not_processed = true;
        if (now >= st.last_arrival + r.waiting_ms) {
            if (r.is_start && r.seq && st.nw == 0 && st.pn == 0) {
                const IX s = se_alloc();
                if (s == NIL) return;
                add_state(p, s);
            } else if (r.seq && st.nw != 0) {
                reset_state(p);
            }
            update_state(p);
            IX expired = NIL;
            IX* pd = pend(p);
            IX* ret = (IX*)(base + L.off_ret);
            int nret = 0;
            for (int j = 0; j < st.pn;) {
                const IX s = pd[j];
                if (is_expired(s, now)) {  // within
                    expired = s;
                    erase(pd, st.pn, j);
                    continue;
                }
                const IX own = slots(s)[p];
                const bool passed = own == NIL ? now >= se(s).ts + r.waiting_ms
                                               : now >= rc(nd(own).rec).ts + r.waiting_ms;  // waitingTimePassed
                if (passed) {
                    erase(pd, st.pn, j);
                    const bool partner_in = slots(s)[r.partner] != NIL;
                    if (r.logical_or && !partner_in) {  // OR partner not received
                        const IX n = empty_node();
                        if (n == NIL) return;
                        add_event(s, p, n);
                        if (nret >= L.lcap) { set_ovf(); return; }
                        ret[nret++] = s;
                    } else if (!r.logical_or && partner_in) {  // AND partner received
                        if (nret >= L.lcap) { set_ovf(); return; }
                        ret[nret++] = s;
                    } else if (!r.logical_or) {  // AND partner not received: let it proceed
                        const IX n = empty_node();
                        if (n == NIL) return;
                        add_event(s, p, n);
                    }
                    continue;
                }
                ++j;
            }
            if (expired != NIL && r.within_every >= 0) {
                add_every_state(r.within_every, expired);
                update_state(r.within_every);
            }
            not_processed = nret == 0;
            for (int i = 0; i < nret && !ovf(); ++i) {
                se(ret[i]).ts = now;
                alogic_send(p, ret[i]);
            }
            st.last_arrival = 0;
        }
        if (r.next_every >= 0 || (not_processed && r.is_start)) {  // schedule again
            if (st.last_arrival == 0) clk_hi = clock;  // the next break is clock + waiting
            const int64_t nb = st.last_arrival == 0 ? clock + r.waiting_ms : st.last_arrival + r.waiting_ms;
            notify_at(r.sched, nb);
        }
    }
    // Scheduler.sendTimerEvents :171-209 for this key: every queued time <= c, in FIFO order, each one TIMER event
    // through the EntryValve into the absent processor
    SDG_HD void maybe_gc() {
        const KHead& h = head();
        if (4 * h.se_used > 3 * L.ns || 4 * h.nd_used > 3 * L.nn || 4 * h.rc_used > 3 * L.nr) gc();
    }
    SDG_HD void fire(int sch, int64_t g, int64_t c) {
        maybe_gc();  // between fires nothing but the lists holds StateEvents
        pos = g;
        fsched = sch;
        clock = c;
        cur_seq = seq_base + g;
        cur_sub = INT64_MIN | ((int64_t)sch << 48);  // before the event at g; the host ranks fires across keys
        log_rec(LOG_FIRE, sch, 0, c);
        clk_hi = INT64_MAX;
        const int p = P->sched_state[sch];
        TQ& q = tq(sch);
        while (q.n > 0 && tqt(sch)[q.h] <= c && !ovf()) {
            const int64_t t = tq_pop(sch);
            log_rec(LOG_POP, sch, 0, t);
            if (!TM) break;
            if (P->st[p].kind == PK_ABSENT) absent_timer(p, t);
            else alogic_timer(p, t);
            absent_gc();  // each TIMER event is its own getState / returnState scope (process() :150-227)
        }
        // at a later clock the same fire would also pop the next queued time: the outcome holds below it only
        if (q.n > 0 && tqt(sch)[q.h] - 1 < clk_hi) clk_hi = tqt(sch)[q.h] - 1;
        log_rec(LOG_FIRE_END, sch, 0, clk_hi);
        fsched = -1;
        absent_gc();
    }
    // first position >= lo whose clock reaches t and that advances the clock (G: none in this batch)
    SDG_HD int64_t due_at(int64_t t, int64_t lo) {
        int64_t a = 0, b = T.G;  // lower_bound(clk, t)
        while (a < b) {
            const int64_t m = (a + b) >> 1;
            if (T.clk[m] < t) a = m + 1;
            else b = m;
        }
        const int64_t x = a > lo ? a : lo;
        return x >= T.G ? T.G : (int64_t)T.nadv[x];
    }
    // every fire of this key at positions <= limit, in the reference's order
    SDG_HD void fire_until(int64_t limit) {
        if (!TM || P->n_sched == 0) return;
        if (nfires >= 0) {  // explicit list (host scheduler simulation)
            while (fi < nfires && (int64_t)fires[fi].g <= limit && !ovf()) {
                const TimerFire f = fires[fi++];
                fire(f.sched, f.g, f.clock);
            }
            return;
        }
        while (!ovf()) {  // ideal: each due head at the first clock advance that reaches it
            int64_t bg = T.G;
            int bs = -1;
            int64_t bt = 0;
            int32_t bc = 0;
            for (int i = 0; i < P->n_sched; ++i) {
                const TQ& q = tq(i);
                if (q.n == 0) continue;
                const int64_t h = tqt(i)[q.h];
                const int64_t g = due_at(h, q.earliest);
                // playback: schedulers in listener order at one position; live: (time, creation) across them
                const bool better = g < bg || (g == bg && bs >= 0 && T.live && (h < bt || (h == bt && q.created < bc)));
                if (better) { bg = g; bs = i; bt = h; bc = q.created; }
            }
            if (bs < 0 || bg > limit || bg >= T.G) return;
            int64_t c = T.clk[bg];
            if (T.live) {  // liveNow = max(liveNow before this advance, the due time)
                const int64_t before = bg > 0 ? T.clk[bg - 1] : T.clock0;
                c = bt > before ? bt : before;
            }
            fire(bs, bg, c);
        }
    }

    // ---- receiver ----------------------------------------------------------------------------------------
    SDG_HD void init_key() {  // StateStreamRuntime.initPartition: init, then partitionCreated of the startups
        for (int i = 0; i < P->n_init; ++i) init(P->init_seq[i]);
        for (int i = 0; i < (TM ? P->n_startup : 0); ++i) {
            const int p = P->startup_seq[i];
            const StateRow& r = P->st[p];
            PState& st = ps(p);
            if (st.started) continue;  // AbsentStreamPreStateProcessor :291-308 / AbsentLogical... :331-351
            st.started = 1;
            if (r.is_start && r.waiting_ms != -1 && st.active) {
                if ((TM && r.kind == PK_ABSENT)) {
                    st.last_sched = clock + r.waiting_ms;
                    notify_at(r.sched, st.last_sched);
                } else {
                    notify_at(r.sched, clock + r.waiting_ms);
                }
            }
        }
        absent_gc();
    }

    SDG_HD void on_event(int qs, IX rec, int64_t ts) {
        const RecvRow& rv = P->recv[qs];
        // stabilizeStates (state/receiver/*ProcessStreamReceiver.java)
        for (int i = 0; i < P->n_expire; ++i) expire_events(P->expire_seq[i], ts);
        if (P->seq) {
            for (int i = 0; i < P->n_reset; ++i) reset_state(P->reset_seq[i]);
            for (int i = 0; i < P->n_update; ++i) update_state(P->update_seq[i]);
        } else if (rv.multi) {
            for (int i = 0; i < rv.n; ++i) update_state(rv.procs[i]);
        } else if (rv.n > 0) {
            update_state(rv.procs[0]);
        }
        for (int j = 0; j < rv.n; ++j) {
            if (ovf()) return;
            process_and_return(rv.procs[rv.order[j]], rec, rv.selector);
        }
    }
};

// ---- idle keys: the reference's state destruction (StreamPreState.canDestroy :443-448 via
// PartitionStateHolder.returnState :51-70) ------------------------------------------------------------------------
// The reference destroys a key's processor state once it is empty and not initialised: every non-start processor
// whose lists drained. Only the start processors' states (initialised, holding their seed StateEvents) stay. A key
// in that condition -- non-start processors empty, start processors holding nothing but fresh seeds (no event in any
// slot, timestamp -1, each referenced once) -- needs no partial-match arena: it is kept as an idle record (the start
// processors' flags and seed counts), and its arena slot goes back to the pool. At the key's next event the arena
// is rebuilt from the record (non-start processors fresh, as the reference re-creates them; seeds are
// interchangeable). Queries with absent states (timer queues) or @purge keep their arenas.
constexpr int IDLE_PER_STATE = 12;  // 8 PState flag bytes, int16 pending / newAndEvery seed counts
SDG_HD int idle_bytes(int n_states) { return (4 + IDLE_PER_STATE * n_states + 15) & ~15; }

template <bool TM, class IX>
SDG_HD bool to_idle(CtxT<TM, IX>& c, uint8_t* rec) {
    if (c.ovf()) return false;
    KHead& h = c.head();
    if (!(h.flags & 2)) return false;
    c.gc();
    if (h.nd_used || h.rc_used) return false;
    int entries = 0;
    for (int p = 0; p < c.L.n_states; ++p) {
        const auto& st = c.ps(p);
        if (st.last_sched || st.last_arrival) return false;
        if (!c.P->st[p].is_start && (st.pn || st.nw)) return false;
        for (int l = 0; l < 2; ++l) {
            const IX* lst = l ? c.newe(p) : c.pend(p);
            const int n = l ? st.nw : st.pn;
            for (int j = 0; j < n; ++j) {
                const auto& e = c.se(lst[j]);
                if (e.type != T_CURRENT || e.ts != -1) return false;
                const IX* sl = c.slots(lst[j]);
                for (int k = 0; k < c.L.n_states; ++k)
                    if (sl[k] != NIL) return false;
            }
            entries += n;
        }
    }
    if (entries != h.se_used) return false;  // no seed shared between lists (logical partners)
    *(int32_t*)rec = h.flags;
    for (int p = 0; p < c.L.n_states; ++p) {
        uint8_t* r = rec + 4 + IDLE_PER_STATE * p;
        const auto& st = c.ps(p);
        const uint8_t* f = &st.changed;  // the 8 flag bytes: changed .. pad
        for (int b = 0; b < 8; ++b) r[b] = f[b];
        *(int16_t*)(r + 8) = (int16_t)st.pn;  // (reclaiming device queries only: int16 counts)
        *(int16_t*)(r + 10) = (int16_t)st.nw;
    }
    return true;
}

template <bool TM, class IX>
SDG_HD void from_idle(CtxT<TM, IX>& c, const uint8_t* rec) {
    c.arena_init();
    c.head().flags = *(const int32_t*)rec;
    for (int p = 0; p < c.L.n_states; ++p) {
        const uint8_t* r = rec + 4 + IDLE_PER_STATE * p;
        const int16_t pn = *(const int16_t*)(r + 8), nw = *(const int16_t*)(r + 10);
        if (!c.P->st[p].is_start) continue;  // destroyed: fresh (arena_init)
        auto& st = c.ps(p);
        uint8_t* f = &st.changed;
        for (int b = 0; b < 8; ++b) f[b] = r[b];
        for (int l = 0; l < 2; ++l) {
            const int n = l ? nw : pn;
            for (int j = 0; j < n; ++j) {
                const IX s = c.se_alloc();
                if (s == NIL) return;
                if (l) c.push(c.newe(p), st.nw, s);
                else c.push(c.pend(p), st.pn, s);
            }
        }
    }
}

// one key's committed arena into a larger layout (more partial-match slots, same states / columns / schedulers),
// possibly of a wider index type (SIX: the source's -- a key the host takes over moves from int16 to int32 indices):
// header, processor states, the lists (re-strided), timer queues (unrolled to start at 0) and every pool object at
// its index; the free lists are then rebuilt by a mark-sweep in the new layout (the lists are the only roots
// between batches), which also frees the new slots
template <class SIX = int16_t, bool TM, class IX>
SDG_HD void migrate_key(CtxT<TM, IX>& d, const uint8_t* src, const Layout& Ls) {
    const Layout& Ld = d.L;
    uint8_t* dst = d.base;
    for (int64_t i = 0; i < Ld.bytes; ++i) dst[i] = 0;
    const KHead* sh = (const KHead*)src;
    if (!(sh->flags & 2)) return;  // never initialised: stays zero (= fresh)
    d.head() = *sh;
    for (int p = 0; p < Ld.n_states; ++p) {
        const PStateT<SIX>& sp0 = ((const PStateT<SIX>*)(src + Ls.off_ps))[p];
        auto& dp = d.ps(p);
        dp.changed = sp0.changed;
        dp.initialized = sp0.initialized;
        dp.success = sp0.success;
        dp.start_reset = sp0.start_reset;
        dp.active = sp0.active;
        dp.started = sp0.started;
        dp.returned = sp0.returned;
        dp.last_sched = sp0.last_sched;
        dp.last_arrival = sp0.last_arrival;
        dp.pn = sp0.pn;
        dp.nw = sp0.nw;
        const SIX* sp = (const SIX*)(src + Ls.off_pend) + (int64_t)p * Ls.lcap;
        const SIX* sn = (const SIX*)(src + Ls.off_newe) + (int64_t)p * Ls.lcap;
        for (int j = 0; j < dp.pn; ++j) d.pend(p)[j] = sp[j];
        for (int j = 0; j < dp.nw; ++j) d.newe(p)[j] = sn[j];
    }
    for (int q = 0; q < Ld.n_sched; ++q) {
        const TQT<SIX>& t = ((const TQT<SIX>*)(src + Ls.off_tq))[q];
        const int64_t* st = (const int64_t*)(src + Ls.off_tqt) + (int64_t)q * Ls.qcap;
        for (int j = 0; j < t.n; ++j) d.tqt(q)[j] = st[(t.h + j) % Ls.qcap];
        auto& dt = d.tq(q);
        dt.earliest = t.earliest;
        dt.created = t.created;
        dt.h = 0;
        dt.n = t.n;
    }
    for (int i = 0; i < Ls.ns; ++i) {  // (every index is < the source's pool sizes: it fits the destination's type)
        const SET<SIX>& se = *(const SET<SIX>*)(src + Ls.off_se + (int64_t)i * Ls.se_bytes);
        auto& de = d.se(i);
        de.type = se.type;
        de.mark = se.mark;
        de.ts = se.ts;
        const SIX* ss = (const SIX*)((const uint8_t*)&se + sizeof(SET<SIX>));
        IX* ds = d.slots(i);
        for (int k = 0; k < Ld.n_states; ++k) ds[k] = (IX)ss[k];
    }
    for (int i = 0; i < Ls.nn; ++i) {
        const NodeT<SIX>& n = ((const NodeT<SIX>*)(src + Ls.off_nd))[i];
        d.nd(i).rec = n.rec;
        d.nd(i).next = n.next;
    }
    for (int i = 0; i < Ls.nr; ++i) {
        const RecT<SIX>& r = *(const RecT<SIX>*)(src + Ls.off_rc + (int64_t)i * Ls.rc_bytes);
        auto& dr = d.rc(i);
        dr.nullmask = r.nullmask;
        dr.ts = r.ts;
        const int64_t* sv = (const int64_t*)((const uint8_t*)&r + sizeof(RecT<SIX>));
        for (int c = 0; c < Ld.n_cols; ++c) d.vals(i)[c] = sv[c];
    }
    d.head().flags &= ~1;
    d.gc();
}

template <bool TM, class IX>
SDG_HD void SEAccT<TM, IX>::load(int slot, int col, int chain, uint8_t kind, int64_t* v, bool* null) {
    (void)kind;
    *v = 0;
    *null = true;
    if (slot < 0 || slot >= c->L.n_states) return;
    IX e = c->chain_at(se, slot, chain);
    if (e == NIL) return;
    IX r = c->nd(e).rec;
    *v = c->vals(r)[col];
    *null = (c->rc(r).nullmask >> col) & 1u;
}
template <bool TM, class IX>
SDG_HD bool SEAccT<TM, IX>::slot_empty(int slot, int chain) {
    if (slot < 0 || slot >= c->L.n_states) return true;
    return c->chain_at(se, slot, chain) == NIL;
}

// one key's rows [b, e) of a batch view (time order within the key)
struct KeyEvents {
    const int64_t* ts;
    const uint8_t* qstream;   // nullptr: single stream
    const uint32_t* orig;     // nullptr: identity
    const void* const* cols;
    const uint8_t* const* nulls;
    int64_t b, e, seq_base;
    int64_t pos_off;          // batch position of view row 0 (row p: pos_off + (orig ? orig[p] : p))
    const uint32_t* vrank = nullptr;  // range partitions: the range a row came from; a stream without a partition key:
                                      // the key's rank in getPartitionKeys() order -- one event sent to several keys
                                      // is processed key after key in that order (PartitionStreamReceiver.receive /
                                      // send(ComplexEvent) :274-283); < 2^23

};

// one key's batch run, in steps (the device composes them in run_key; the host scheduler simulation steps a key
// itself when it has to take it over, sched.h): initPartition on the key's first event ever (unpartitioned
// queries: before position 0, as SiddhiAppRuntime.start does), each row through the receiver, timer fires between
template <bool TM, class IX>
SDG_HD bool key_begin(CtxT<TM, IX>& c, const KeyEvents& ev) {  // returns need_init (a partitioned first-seen key)
    const Plan* P = c.P;
    c.seq_base = ev.seq_base;
    c.fsched = -1;
    c.fi = 0;
    c.pos = -1;
    c.clock = c.T.clock0;
    const bool fresh = !(c.head().flags & 2);
    if (fresh) {
        c.arena_init();
        c.head().flags = 2;
    }
    c.head().kseq = 0;
    for (int i = 0; i < c.L.n_sched; ++i)
        if (c.tq(i).n > 0) c.tq(i).earliest = 0;  // positions restart with every batch
    if (fresh && !P->partitioned) {
        c.init_key();
        return false;
    }
    return fresh;
}
SDG_HD int64_t key_pos(const KeyEvents& ev, int64_t p) { return ev.pos_off + (ev.orig ? (int64_t)ev.orig[p] : p); }
// row p (fires due before it have run); returns false when the key overflowed
template <bool TM, class IX>
SDG_HD bool key_row(CtxT<TM, IX>& c, const KeyEvents& ev, int64_t p, bool& need_init) {
    const Plan* P = c.P;
    const int64_t g = key_pos(ev, p);
    c.pos = g;
    if (TM && P->n_sched) c.clock = c.T.clk[g];
    if (c.purge.clk) {
        const int64_t now = c.purge.clk[g];
        if (!need_init && c.purge.last != INT64_MIN && now >= c.purge.from && c.purge.last + c.purge.idle < now) {
            const uint32_t kseq = c.head().kseq;  // the run's log order continues across the reset
            c.arena_init();  // the key's states destroyed (cleanGroupByStates); its partition key is new again
            c.head().flags = 2;
            c.head().kseq = kseq;
            need_init = true;
            c.purge_pending = true;
            // the key's SchedulerStates are destroyed with them (the scheduler simulation mirrors it)
            if (TM && P->n_sched) c.log_rec(LOG_PURGE, 0, ORIGIN_EVENT, now);
        }
        c.purge.last = now;  // partitionKeys.put(key, currentTime)
    }
    if (need_init) {  // PartitionRuntimeImpl.initPartition for a first-seen key (after the clock advance)
        c.init_key();
        need_init = false;
    }
    c.maybe_gc();
    IX r = c.rc_alloc();
    if (r == NIL) return false;
    auto& rec = c.rc(r);
    const int64_t ts = ev.ts[p];
    rec.ts = ts;
    int64_t* v = c.vals(r);
    uint32_t nm = 0;
    for (int col = 0; col < P->n_cols; ++col) {
        v[col] = load_col(ev.cols[col], P->col_kind[col], p);
        if (ev.nulls[col] && ev.nulls[col][p]) nm |= 1u << col;
    }
    rec.nullmask = nm;
    c.cur_seq = ev.seq_base + g;
    c.cur_sub = ev.vrank ? (int64_t)ev.vrank[p] << 40 : 0;
    c.on_event(ev.qstream ? ev.qstream[p] : 0, r, ts);
    if (TM && P->n_sched) c.absent_gc();
    c.destroyed_gc();
    return !c.ovf();
}
template <bool TM, class IX>
SDG_HD void run_key(CtxT<TM, IX>& c, const KeyEvents& ev) {
    bool need_init = key_begin(c, ev);
    for (int64_t p = ev.b; p < ev.e && !c.ovf(); ++p) {
        c.fire_until(key_pos(ev, p));  // TimeChangeListener.onTimeChange runs before the event is processed
        if (c.ovf() || !key_row(c, ev, p, need_init)) break;
    }
    if (TM && c.P->n_sched && c.T.G > 0 && !c.ovf()) {
        c.fire_until(c.T.G - 1);
        c.clock = c.T.clk[c.T.G - 1];
    }
}

}  // namespace nfa
}  // namespace sdg
