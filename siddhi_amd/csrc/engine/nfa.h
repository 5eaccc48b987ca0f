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
//   receivers                         state/receiver/*.java (stabilizeStates), MultiProcessStreamReceiver.java
// Object identity is kept: StateEvents and StreamEvent nodes are arena objects referenced by index, so clones
// share StreamEvent chains exactly as StateEventCloner does (count-state aliasing, CountPatternTestCase :53-111).
// Memory is reclaimed by a mark-sweep pass over the lists at event boundaries; running out of arena space sets
// the key's overflow flag (reported as SDG_ERR_CAPACITY, never a silent drop).
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
    int32_t ns, nn, nr, lcap, n_states, n_cols;
    int64_t off_ps, off_pend, off_newe, off_ret, off_se, off_nd, off_rc, bytes;
    int32_t se_bytes, rc_bytes;
};

struct KHead {
    int32_t flags;       // bit0 overflow, bit1 key initialised
    int32_t se_free, nd_free, rc_free;
    int32_t se_used, nd_used, rc_used;
    int32_t pad;
};

struct PState {
    uint8_t changed, initialized, success, start_reset, active, started, returned, pad;
    int64_t last_sched;
    int16_t pn, nw;
    int16_t pad2[2];
};

struct SE {
    int16_t free_next;
    uint8_t type, mark;
    int32_t pad;
    int64_t ts;
    // int16_t slot[n_states] follows
};

struct Node {
    int16_t rec, next, free_next;
    uint8_t mark, pad;
};

struct Rec {
    uint32_t nullmask;
    uint8_t mark, pad;
    int16_t free_next;
    int64_t ts;
    // int64_t vals[n_cols] follows
};

inline Layout make_layout(int n_states, int n_cols, int ns) {
    Layout L;
    L.ns = ns;
    L.nn = ns * 4;
    L.nr = ns * 2;
    L.lcap = ns;
    L.n_states = n_states;
    L.n_cols = n_cols;
    L.se_bytes = (int32_t)((sizeof(SE) + 2 * n_states + 7) & ~7);
    L.rc_bytes = (int32_t)(sizeof(Rec) + 8 * n_cols);
    int64_t o = sizeof(KHead);
    L.off_ps = o;
    o += (int64_t)sizeof(PState) * n_states;
    L.off_pend = o;
    o += (int64_t)2 * L.lcap * n_states;
    L.off_newe = o;
    o += (int64_t)2 * L.lcap * n_states;
    L.off_ret = o;  // StateEvents one processAndReturn call returns (emitted after its loop)
    o += (int64_t)2 * L.lcap;
    o = (o + 7) & ~7;
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

// one emitted match
struct Emit {
    int16_t se;
};

struct Ctx;

// bytecode accessor over a StateEvent (StateEvent.getStreamEvent(int[]) + attribute)
struct SEAcc {
    Ctx* c;
    int16_t se;
    SDG_HD void load(int slot, int col, int chain, uint8_t kind, int64_t* v, bool* null);
    SDG_HD bool slot_empty(int slot, int chain);
};

struct Ctx {
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
    unsigned long long* emit_count;
    int64_t emit_cap;
    int* flags;
    uint32_t key;
    int64_t cur_seq;
    int64_t cur_sub;

    // ---- arena access ------------------------------------------------------------------------------------
    SDG_HD KHead& head() { return *(KHead*)base; }
    SDG_HD PState& ps(int p) { return ((PState*)(base + L.off_ps))[p]; }
    SDG_HD int16_t* pend(int p) { return (int16_t*)(base + L.off_pend) + (int64_t)p * L.lcap; }
    SDG_HD int16_t* newe(int p) { return (int16_t*)(base + L.off_newe) + (int64_t)p * L.lcap; }
    SDG_HD SE& se(int i) { return *(SE*)(base + L.off_se + (int64_t)i * L.se_bytes); }
    SDG_HD int16_t* slots(int i) { return (int16_t*)((uint8_t*)&se(i) + sizeof(SE)); }
    SDG_HD Node& nd(int i) { return ((Node*)(base + L.off_nd))[i]; }
    SDG_HD Rec& rc(int i) { return *(Rec*)(base + L.off_rc + (int64_t)i * L.rc_bytes); }
    SDG_HD int64_t* vals(int i) { return (int64_t*)((uint8_t*)&rc(i) + sizeof(Rec)); }
    SDG_HD bool ovf() { return head().flags & 1; }
    SDG_HD void set_ovf() { head().flags |= 1; }

    SDG_HD void arena_init() {
        KHead& h = head();
        h.flags = 0;
        h.se_used = h.nd_used = h.rc_used = 0;
        for (int i = 0; i < L.ns; ++i) se(i).free_next = (int16_t)(i + 1 < L.ns ? i + 1 : NIL);
        for (int i = 0; i < L.nn; ++i) nd(i).free_next = (int16_t)(i + 1 < L.nn ? i + 1 : NIL);
        for (int i = 0; i < L.nr; ++i) rc(i).free_next = (int16_t)(i + 1 < L.nr ? i + 1 : NIL);
        h.se_free = 0;
        h.nd_free = 0;
        h.rc_free = 0;
        for (int p = 0; p < L.n_states; ++p) {
            PState& s = ps(p);
            s.changed = s.initialized = s.success = s.start_reset = s.started = s.returned = 0;
            s.active = 1;
            s.last_sched = 0;
            s.pn = s.nw = 0;
        }
    }

    SDG_HD int16_t se_alloc() {
        KHead& h = head();
        if (h.se_free == NIL) { set_ovf(); return NIL; }
        int16_t i = (int16_t)h.se_free;
        h.se_free = se(i).free_next;
        h.se_used++;
        SE& s = se(i);
        s.type = T_CURRENT;
        s.ts = -1;
        int16_t* sl = slots(i);
        for (int k = 0; k < L.n_states; ++k) sl[k] = NIL;
        return i;
    }
    SDG_HD int16_t nd_alloc(int16_t rec) {
        KHead& h = head();
        if (h.nd_free == NIL) { set_ovf(); return NIL; }
        int16_t i = (int16_t)h.nd_free;
        h.nd_free = nd(i).free_next;
        h.nd_used++;
        nd(i).rec = rec;
        nd(i).next = NIL;
        return i;
    }
    SDG_HD int16_t rc_alloc() {
        KHead& h = head();
        if (h.rc_free == NIL) { set_ovf(); return NIL; }
        int16_t i = (int16_t)h.rc_free;
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
                int16_t* lst = l ? newe(p) : pend(p);
                int n = l ? ps(p).nw : ps(p).pn;
                for (int j = 0; j < n; ++j) {
                    int16_t s = lst[j];
                    if (se(s).mark) continue;
                    se(s).mark = 1;
                    int16_t* sl = slots(s);
                    for (int k = 0; k < L.n_states; ++k)
                        for (int16_t x = sl[k]; x != NIL && !nd(x).mark; x = nd(x).next) {
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
            se(i).free_next = (int16_t)h.se_free;
            h.se_free = i;
        }
        for (int i = L.nn - 1; i >= 0; --i) {
            if (nd(i).mark) { h.nd_used++; continue; }
            nd(i).free_next = (int16_t)h.nd_free;
            h.nd_free = i;
        }
        for (int i = L.nr - 1; i >= 0; --i) {
            if (rc(i).mark) { h.rc_used++; continue; }
            rc(i).free_next = (int16_t)h.rc_free;
            h.rc_free = i;
        }
    }

    // ---- StateEvent helpers ------------------------------------------------------------------------------
    SDG_HD int16_t clone(int16_t o) {  // StateEventCloner.copyStateEvent: slots shared
        int16_t n = se_alloc();
        if (n == NIL) return NIL;
        SE& a = se(n);
        SE& b = se(o);
        a.type = b.type;
        a.ts = b.ts;
        int16_t* sa = slots(n);
        int16_t* sb = slots(o);
        for (int k = 0; k < L.n_states; ++k) sa[k] = sb[k];
        return n;
    }
    SDG_HD int16_t chain_at(int16_t s, int pos, int idx) {  // StateEvent.getStreamEvent(int[])
        int16_t e = slots(s)[pos];
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
        for (int16_t x = e; x != NIL; x = nd(x).next) ++len;
        int k = len + idx;
        if (k < 0) return NIL;
        for (int i = 0; i < k; ++i) e = nd(e).next;
        return e;
    }
    SDG_HD void add_event(int16_t s, int pos, int16_t node) {
        int16_t a = slots(s)[pos];
        if (a == NIL) { slots(s)[pos] = node; return; }
        while (nd(a).next != NIL) a = nd(a).next;
        nd(a).next = node;
    }
    SDG_HD void remove_last_event(int16_t s, int pos) {
        int16_t a = slots(s)[pos];
        if (a == NIL) return;
        while (nd(a).next != NIL) {
            if (nd(nd(a).next).next == NIL) { nd(a).next = NIL; return; }
            a = nd(a).next;
        }
        slots(s)[pos] = NIL;
    }

    // ---- list helpers ------------------------------------------------------------------------------------
    SDG_HD void push(int16_t* lst, int16_t& n, int16_t v) {
        if (n >= L.lcap) { set_ovf(); return; }
        lst[n++] = v;
    }
    SDG_HD static void erase(int16_t* lst, int16_t& n, int j) {
        for (int i = j; i + 1 < n; ++i) lst[i] = lst[i + 1];
        --n;
    }
    SDG_HD void pend_push_newe(int p) {  // newAndEvery.sort(eventTimeComparator) + pending.addAll + clear
        PState& s = ps(p);
        int16_t* nw = newe(p);
        for (int i = 1; i < s.nw; ++i) {  // stable insertion sort; ts == -1 sorts last
            int16_t v = nw[i];
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
        int16_t* pd = pend(p);
        for (int i = 0; i < s.nw; ++i) push(pd, s.pn, nw[i]);
        s.nw = 0;
    }

    // ---- filters / selector ------------------------------------------------------------------------------
    SDG_HD bool filter(int p, int16_t s) {
        const StateRow& r = P->st[p];
        const FastPred& f = P->fast[p];
        SEAcc acc{this, s};
        if (f.kind == FP_TRUE) return true;
        if (f.kind != FP_NONE) return fast_pass(f, acc);
        return pass(code, r.filter, consts, acc, stk, stride);
    }

    SDG_HD void emit(int16_t s) {  // QuerySelector.processNoGroupBy for one StateEvent (insert current events)
        if (se(s).type != T_CURRENT) return;
        unsigned long long slot = __atomic_fetch_add(emit_count, 1ull, __ATOMIC_RELAXED);
        if ((int64_t)slot >= emit_cap) {
            __atomic_fetch_or(flags, 1, __ATOMIC_RELAXED);
            return;
        }
        emit_ts[slot] = se(s).ts;
        emit_seq[slot] = cur_seq;
        emit_sub[slot] = cur_sub++;
        emit_key[slot] = key;
        uint32_t nm = 0;
        SEAcc acc{this, s};
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
    SDG_HD bool is_expired(int16_t s, int64_t now) {
        if (!P->has_within) return false;
        for (int i = 0; i < P->n_states; ++i) {
            if (!P->st[i].is_start) continue;
            int16_t e = slots(s)[i];
            if (e != NIL) {
                int64_t d = rc(nd(e).rec).ts - now;
                if (d < 0) d = -d;
                if (d > P->within_ms) return true;
            }
        }
        return false;
    }

    SDG_HD void add_state(int p, int16_t s) {
        // iterative: a count state with min 0 forwards at once (CountPreStateProcessor.addState :97-125 ->
        // CountPostStateProcessor.processMinCountReached), which may reach another such state. The every clone of
        // each level is pushed before the forward chain continues: the chain only touches lists of later states,
        // the clone the (earlier) every-group start, so the order of the two does not change any list.
        for (int level = 0; level <= MAX_STATES; ++level) {
            const StateRow& r = P->st[p];
            PState& st = ps(p);
            if (r.kind == PK_LOGICAL) {  // LogicalPreStateProcessor.addState :43-62
                int q = r.partner;
                if (r.is_start || r.seq) {
                    if (st.nw == 0) push(newe(p), st.nw, s);
                    if (ps(q).nw == 0) push(newe(q), ps(q).nw, s);
                } else {
                    push(newe(p), st.nw, s);
                    push(newe(q), ps(q).nw, s);
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

    SDG_HD void add_every_state(int p, int16_t s) {
        const StateRow& r = P->st[p];
        int16_t c = clone(s);
        if (c == NIL) return;
        se(c).type = T_CURRENT;
        for (int i = p; i < L.n_states; ++i) slots(c)[i] = NIL;
        push(newe(p), ps(p).nw, c);
        if (r.kind == PK_LOGICAL) {  // :65-84
            slots(c)[r.partner] = NIL;
            push(newe(r.partner), ps(r.partner).nw, c);
        }
    }

    SDG_HD void init(int p) {  // StreamPreStateProcessor.init :178-194
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        if (r.is_start && (!st.initialized || r.next_every >= 0)) {
            int16_t s = se_alloc();
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
        int16_t expired = NIL;
        int16_t* pd = pend(p);
        while (st.pn > 0 && is_expired(pd[0], now)) {
            int16_t s = pd[0];
            erase(pd, st.pn, 0);
            if (se(s).type != T_EXPIRED) { se(s).type = T_EXPIRED; expired = s; }
        }
        int16_t* nw = newe(p);
        for (int j = 0; j < st.nw;) {
            int16_t s = nw[j];
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
    SDG_HD void post_stream(int p, int16_t s) {  // StreamPostStateProcessor.process :64-83
        const StateRow& r = P->st[p];
        ps(p).changed = 1;
        se(s).ts = rc(nd(slots(s)[p]).rec).ts;
        if (r.selector_after) ps(p).returned = 1;
        if (r.next >= 0) add_state(r.next, s);
        if (r.next_every >= 0) add_every_state(r.next_every, s);
        if (r.callback >= 0) start_state_reset(r.callback);
    }
    SDG_HD void count_min_reached(int p, int16_t s) {  // CountPostStateProcessor.processMinCountReached
        const StateRow& r = P->st[p];
        if (r.selector_after) {
            ps(p).changed = 1;
            ps(p).returned = 1;
        }
        if (r.next >= 0) add_state(r.next, s);
        if (r.next_every >= 0) add_every_state(r.next_every, s);
    }
    SDG_HD void post_count(int p, int16_t s) {  // CountPostStateProcessor.process :39-79
        const StateRow& r = P->st[p];
        int16_t e = slots(s)[p];
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
    SDG_HD void post_logical(int p, int16_t s) {  // LogicalPostStateProcessor.process :59-87
        const StateRow& r = P->st[p];
        if (!r.logical_or) {
            if (slots(s)[r.partner] != NIL) post_stream(p, s);
            else ps(p).changed = 1;
        } else {
            post_stream(p, s);
            if (P->st[r.partner].selector_after && r.last == r.partner) ps(r.partner).returned = 1;
        }
    }
    SDG_HD void post(int p, int16_t s) {
        switch (P->st[p].kind) {
            case PK_COUNT: post_count(p, s); break;
            case PK_LOGICAL: post_logical(p, s); break;
            default: post_stream(p, s); break;
        }
    }

    // process(StateEvent): filters then post
    SDG_HD void process_se(int p, int16_t s) {
        ps(p).changed = 0;
        if (filter(p, s)) post(p, s);
    }

    // processAndReturn; the receiver hands the returned StateEvents to the selector after the loop
    // (StateMultiProcessStreamReceiver.processAndClear :47-68), so they are collected first
    SDG_HD void process_and_return(int p, int16_t rec, bool selector) {
        const StateRow& r = P->st[p];
        PState& st = ps(p);
        int16_t* pd = pend(p);
        const int last = r.last;
        int16_t* ret = (int16_t*)(base + L.off_ret);
        int nret = 0;
        for (int j = 0; j < st.pn;) {
            if (ovf()) return;
            int16_t s = pd[j];
            if (r.kind == PK_COUNT) {  // :60-66
                if ((p + 1 < L.n_states && slots(s)[p + 1] != NIL) || (p + 2 < L.n_states && slots(s)[p + 2] != NIL)) {
                    erase(pd, st.pn, j);
                    continue;
                }
                int16_t n = nd_alloc(rec);
                if (n == NIL) return;
                add_event(s, p, n);
                st.success = 0;
            } else if (r.kind == PK_LOGICAL) {
                if (r.logical_or && slots(s)[r.partner] != NIL) {
                    erase(pd, st.pn, j);
                    continue;
                }
                int16_t n = nd_alloc(rec);
                if (n == NIL) return;
                slots(s)[p] = n;
            } else {
                int16_t n = nd_alloc(rec);
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
                if (r.seq) {  // SEQUENCE: no state change -> dropped (removeOnNoStateChange)
                    erase(pd, st.pn, j);
                    erased = true;
                    if (r.kind != PK_LOGICAL && P->st[p].callback >= 0) start_state_reset(P->st[p].callback);
                }
            }
            if (!erased) ++j;
        }
        if (selector)
            for (int i = 0; i < nret; ++i) emit(ret[i]);
    }

    // ---- receiver ----------------------------------------------------------------------------------------
    SDG_HD void init_key() {  // StateStreamRuntime.initPartition
        for (int i = 0; i < P->n_init; ++i) init(P->init_seq[i]);
    }

    SDG_HD void on_event(int qs, int16_t rec, int64_t ts) {
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

SDG_HD void SEAcc::load(int slot, int col, int chain, uint8_t kind, int64_t* v, bool* null) {
    (void)kind;
    *v = 0;
    *null = true;
    if (slot < 0 || slot >= c->L.n_states) return;
    int16_t e = c->chain_at(se, slot, chain);
    if (e == NIL) return;
    int16_t r = c->nd(e).rec;
    *v = c->vals(r)[col];
    *null = (c->rc(r).nullmask >> col) & 1u;
}
SDG_HD bool SEAcc::slot_empty(int slot, int chain) {
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
};

// initPartition on the key's first event ever, then every row through the receiver
SDG_HD void run_key(Ctx& c, const KeyEvents& ev) {
    const Plan* P = c.P;
    const Layout& L = c.L;
    if (!(c.head().flags & 2)) {
        c.arena_init();
        c.head().flags = 2;
        c.init_key();
    }
    for (int64_t p = ev.b; p < ev.e && !c.ovf(); ++p) {
        const KHead& h = c.head();
        if (4 * h.se_used > 3 * L.ns || 4 * h.nd_used > 3 * L.nn || 4 * h.rc_used > 3 * L.nr) c.gc();
        int16_t r = c.rc_alloc();
        if (r == NIL) break;
        Rec& rec = c.rc(r);
        const int64_t ts = ev.ts[p];
        rec.ts = ts;
        int64_t* v = c.vals(r);
        uint32_t nm = 0;
        for (int col = 0; col < P->n_cols; ++col) {
            v[col] = load_col(ev.cols[col], P->col_kind[col], p);
            if (ev.nulls[col] && ev.nulls[col][p]) nm |= 1u << col;
        }
        rec.nullmask = nm;
        c.cur_seq = ev.seq_base + (ev.orig ? (int64_t)ev.orig[p] : p);
        c.cur_sub = 0;
        c.on_event(ev.qstream ? ev.qstream[p] : 0, r, ts);
    }
}

}  // namespace nfa
}  // namespace sdg
