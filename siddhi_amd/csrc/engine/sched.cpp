// Scheduler simulation over the per-key fire/notify logs (see sched.h for the reference semantics it follows).
#include "sched.h"

#include <algorithm>
#include <chrono>
#include <queue>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace sdg {

// Java toString of a partition value (ValuePartitionExecutor.execute) -- Float/Double use the Java layout
std::string java_real_string(double x, bool is_float) {
    if (x != x) return "NaN";
    if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
    if (x == 0) return std::signbit(x) ? "-0.0" : "0.0";
    char buf[64];
    for (int prec = 1; prec <= 17; ++prec) {
        std::snprintf(buf, sizeof buf, "%.*e", prec - 1, x);
        if (is_float ? (std::strtof(buf, nullptr) == (float)x) : (std::strtod(buf, nullptr) == x)) break;
    }
    std::string s(buf);
    bool neg = s[0] == '-';
    if (neg) s = s.substr(1);
    size_t ep = s.find('e');
    int e10 = std::atoi(s.c_str() + ep + 1);
    std::string d;
    for (size_t i = 0; i < ep; ++i) if (s[i] != '.') d += s[i];
    while (d.size() > 1 && d.back() == '0') d.pop_back();
    std::string o;
    double ax = std::fabs(x);
    if (ax >= 1e-3 && ax < 1e7) {
        int pt = e10 + 1;
        if (pt <= 0) o = "0." + std::string(-pt, '0') + d;
        else if ((int)d.size() <= pt) o = d + std::string(pt - d.size(), '0') + ".0";
        else o = d.substr(0, pt) + "." + d.substr(pt);
    } else {
        o = d.substr(0, 1) + "." + (d.size() > 1 ? d.substr(1) : "0") + "E" + std::to_string(e10);
    }
    return neg ? "-" + o : o;
}

int32_t java_spread_hash(const std::string& s) {  // String.hashCode over UTF-16 code units, HashMap.hash()
    uint32_t h = 0;
    size_t i = 0;
    while (i < s.size()) {
        const uint32_t c = (unsigned char)s[i];
        uint32_t cp;
        if (c < 0x80) { cp = c; i += 1; }
        else if ((c >> 5) == 6 && i + 1 < s.size()) { cp = ((c & 0x1f) << 6) | (s[i + 1] & 0x3f); i += 2; }
        else if ((c >> 4) == 14 && i + 2 < s.size()) {
            cp = ((c & 0x0f) << 12) | ((s[i + 1] & 0x3f) << 6) | (s[i + 2] & 0x3f);
            i += 3;
        } else if (i + 3 < s.size()) {
            cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3f) << 12) | ((s[i + 2] & 0x3f) << 6) | (s[i + 3] & 0x3f);
            i += 4;
        } else { cp = c; i += 1; }
        if (cp >= 0x10000) {
            cp -= 0x10000;
            h = 31 * h + (0xD800 + (cp >> 10));
            h = 31 * h + (0xDC00 + (cp & 0x3ff));
        } else {
            h = 31 * h + cp;
        }
    }
    return (int32_t)(h ^ (h >> 16));
}

void SchedSim::queued_keys(std::vector<uint32_t>& out) const {
    for (const SchedState& S : cur_.sc)
        for (size_t k = 0; k < S.ks.size(); ++k)
            if (S.ks[k].n > 0) out.push_back((uint32_t)k);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
}

SchedSim::OKey SchedSim::okey(const SchedState& S, const KS& k, uint32_t key) const {
    if (live_) return OKey{k.cseq, 0, key};                         // (time, creation order)
    if (!partitioned_) return OKey{0, 0, key};                       // one state
    return OKey{(uint32_t)k.hash & (S.cap - 1), ~k.stamp, key};     // HashMap iteration order
}

void SchedSim::qpush(KS& k, int64_t t) {
    if (k.spill < 0 && k.n < (uint32_t)QI) {
        k.a[k.n++] = t;
        return;
    }
    if (k.spill < 0) {  // outgrew the inline slots
        if (!work_.spill_free.empty()) {
            k.spill = work_.spill_free.back();
            work_.spill_free.pop_back();
        } else {
            k.spill = (int32_t)work_.spill.size();
            work_.spill.emplace_back();
        }
        std::deque<int64_t>& d = work_.spill[k.spill];
        d.assign(k.a, k.a + k.n);
    }
    work_.spill[k.spill].push_back(t);
    ++k.n;
}

void SchedSim::qpop(KS& k) {
    if (k.n == 0) return;
    --k.n;
    if (k.spill < 0) {
        for (uint32_t i = 0; i < k.n; ++i) k.a[i] = k.a[i + 1];
        return;
    }
    std::deque<int64_t>& d = work_.spill[k.spill];
    d.pop_front();
    if (k.n <= (uint32_t)QI) {  // back inline
        for (uint32_t i = 0; i < k.n; ++i) k.a[i] = d[i];
        d.clear();
        work_.spill_free.push_back(k.spill);
        k.spill = -1;
    }
}

void SchedSim::heap_fix(SchedState& S, Heap& H) const {
    if (H.cap == S.cap) return;
    size_t w = 0;
    for (size_t i = 0; i < H.h.size(); ++i) {
        DueE e = H.h[i];
        const KS& k = S.ks[e.k.key];
        if (k.ver != e.ver) continue;  // stale
        e.k = okey(S, k, e.k.key);
        H.h[w++] = e;
    }
    H.h.resize(w);
    std::make_heap(H.h.begin(), H.h.end(), std::greater<DueE>());
    H.cap = S.cap;
}

void SchedSim::due_add(SchedState& S, uint32_t key, KS& k) {
    const DueE e{okey(S, k, key), ++k.ver};
    Heap& H = S.due[qfront(k)];
    if (H.h.empty()) H.cap = S.cap;
    else heap_fix(S, H);
    H.h.push_back(e);
    std::push_heap(H.h.begin(), H.h.end(), std::greater<DueE>());
}

bool SchedSim::due_front(SchedState& S, int64_t& t, OKey& k) {
    while (!S.due.empty()) {
        auto it = S.due.begin();
        heap_fix(S, it->second);
        std::vector<DueE>& h = it->second.h;
        while (!h.empty() && stale(S, h.front())) {
            std::pop_heap(h.begin(), h.end(), std::greater<DueE>());
            h.pop_back();
        }
        if (h.empty()) {
            S.due.erase(it);
            continue;
        }
        t = it->first;
        k = h.front().k;
        return true;
    }
    return false;
}

void SchedSim::resize(SchedState& S) {  // HashMap.resize(): 16 / 12, then doubling
    if (S.cap == 0) {
        S.cap = 16;
        S.threshold = 12;
    } else {
        S.cap *= 2;
        S.threshold *= 2;
    }
    S.bin.assign(S.cap, 0);
    for (size_t key = 0; key < S.kend; ++key) {  // (ks is sized for every key of the batch; only these can be in)
        const KS& k = S.ks[key];
        if (k.in_map) S.bin[(uint32_t)k.hash & (S.cap - 1)]++;
    }
    // the due heaps are re-keyed by the new buckets lazily (heap_fix: their cap no longer matches)
}

void SchedSim::notify(int sch, uint32_t key, int64_t t) {
    SchedState& S = work_.sc[sch];
    KS* k = &ks(S, key);
    if (partitioned_) {
        if (S.size > S.threshold || S.cap == 0) resize(S);  // computeIfAbsent: resize before the lookup
        if (!k->in_map) {
            k->hash = (*hash_)[key];
            k->in_map = true;
            S.kend = std::max(S.kend, (size_t)key + 1);
            k->stamp = ++S.stamp;
            k->cseq = ++work_.cseq;
            uint32_t& bc = S.bin[(uint32_t)k->hash & (S.cap - 1)];
            const uint32_t before = bc++;
            ++S.size;
            if (before >= 7 && S.cap < 64) resize(S);  // treeifyBin on a table below MIN_TREEIFY_CAPACITY
        }
    } else if (!k->in_map) {  // SingleStateHolder: created on first use, never removed
        k->in_map = true;
        S.kend = std::max(S.kend, (size_t)key + 1);
        k->cseq = ++work_.cseq;
    }
    const bool was_empty = k->n == 0;
    qpush(*k, t);
    if (was_empty) due_add(S, key, *k);
}

void SchedSim::pop(int sch, uint32_t key) {
    SchedState& S = work_.sc[sch];
    if (key >= S.ks.size()) return;
    KS& k = S.ks[key];
    if (k.n == 0) return;
    due_del(k);
    qpop(k);
    if (k.n) due_add(S, key, k);
}

void SchedSim::remove_if_empty(int sch, uint32_t key) {  // returnState / returnAllStates of a drained state
    if (!partitioned_) return;
    SchedState& S = work_.sc[sch];
    if (key >= S.ks.size()) return;
    KS& k = S.ks[key];
    if (k.n || !k.in_map) return;
    S.bin[(uint32_t)k.hash & (S.cap - 1)]--;
    --S.size;
    k.in_map = false;
    k.stamp = k.cseq = 0;
}

void SchedSim::purge(uint32_t key) {  // @purge: the key's SchedulerState leaves every scheduler (map.remove)
    for (SchedState& S : work_.sc) {
        if (key >= S.ks.size()) continue;
        KS& k = S.ks[key];
        if (k.n) {
            due_del(k);
            if (k.spill >= 0) {
                work_.spill[k.spill].clear();
                work_.spill_free.push_back(k.spill);
                k.spill = -1;
            }
            k.n = 0;
        }
        if (k.in_map && partitioned_) {
            S.bin[(uint32_t)k.hash & (S.cap - 1)]--;
            --S.size;
            k.in_map = false;
            k.stamp = k.cseq = 0;
        }
    }
}

namespace {
// SDG_SCHED_PROF=1: per-section host time of simulate() on stderr (diagnostics)
struct SecProf {
    bool on = std::getenv("SDG_SCHED_PROF") != nullptr;
    double t[12] = {};
    std::chrono::steady_clock::time_point last;
    void start() { if (on) last = std::chrono::steady_clock::now(); }
    void lap(int i) {
        if (!on) return;
        auto n = std::chrono::steady_clock::now();
        t[i] += std::chrono::duration<double, std::milli>(n - last).count();
        last = n;
    }
    void print(const char* tag, size_t nl, size_t ne, int64_t nf) {
        if (!on) return;
        std::fprintf(stderr, "[sched setup: kc %.1f scan %.1f sort %.1f heap %.1f]\n", t[8], t[9], t[10], t[11]);
        std::fprintf(stderr, "[sched %s] logs %zu evpush %zu fires %lld; copy %.1f setup %.1f fires %.1f fireq %.1f rows %.1f pushes %.1f end %.1f next %.1f ms\n", tag, nl, ne, (long long)nf,
                     t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7]);
    }
};
}  // namespace

void SchedSim::simulate(const BatchClock& bc, const std::vector<nfa::SchedLog>& logs,
                        const std::vector<int32_t>& key_hash, const KeyRows& rows,
                        const std::function<KeyRun*(uint32_t)>& take_over, Result& out, bool optimistic) {
    using nfa::SchedLog;
    SecProf prof;
    prof.start();
    work_ = cur_;
    prof.lap(0);
    hash_ = &key_hash;
    out = Result{};
    constexpr size_t NONE = ~size_t(0);
    enum : uint8_t { DEV = 0, PENDING = 1, HOST = 2 };  // the key's history so far: its device run / a device fire
                                                      // the scheduler has not made yet / stepped on the host
    struct KC {                              // 32 bytes: two keys per cache line (the pass is bound by these misses)
        uint32_t i = 0, e = 0;               // cursor into the key's device records (logs.size() < 2^32)
        int32_t fh = -1, ft = -1;            // the scheduler's fires of this key so far (list in `fl`)
        uint32_t nshift = 0;                 // its device fires accepted as shifted
        uint8_t mode = DEV;
        bool reordered = false;              // optimistic pass: the scheduler's order differs from the run's
        bool touched = false;
        KeyRun* run = nullptr;
    };
    static_assert(sizeof(KC) == 32, "KC layout");
    if (logs.size() >= 0xFFFFFFFFull) throw std::runtime_error("scheduler simulation: more than 2^32 log records");
    struct FN {
        nfa::TimerFire f;
        int32_t next;
        uint32_t rank;  // the fire's rank among the fires of its position
    };
    std::vector<FN> fl;
    // optimistic pass: every model change, tagged with the key it was made for (confirm() checks reruns by them)
    struct KOp {
        uint32_t key;
        Op op;
    };
    std::vector<KOp> kops;
    if (optimistic) kops.reserve(logs.size());
    auto rec = [&](uint32_t key, uint32_t g, uint8_t kind, int sch, int64_t t) {
        if (optimistic) kops.push_back(KOp{key, Op{g, kind, (uint8_t)sch, t}});
    };
    // keys: dense ids; the table covers every key with records, rows or a queued state
    size_t nkeys = (size_t)std::max<int64_t>(rows.K, 0);
    for (const SchedState& S : work_.sc) nkeys = std::max(nkeys, S.ks.size());
    if (!logs.empty()) nkeys = std::max(nkeys, (size_t)logs.back().key + 1);
    std::vector<KC> kc(nkeys);
    for (SchedState& S : work_.sc)  // sized once (growing by half inside notify() was ~6% of the pass)
        if (S.ks.size() < nkeys) S.ks.resize(nkeys);
    prof.lap(8);
    std::vector<uint32_t> touched;
    auto K = [&](uint32_t key) -> KC& {
        KC& c = kc[key];
        if (!c.touched) {
            c.touched = true;
            touched.push_back(key);
        }
        return c;
    };
    auto posof = [&](size_t i) -> int64_t { return logs[i].g == 0xFFFFFFFFu ? -1 : (int64_t)logs[i].g; };
    // records made while processing an event (its pushes, a purge before it): applied at their positions
    auto is_evpush = [&](size_t i) {
        return (logs[i].type == nfa::LOG_PUSH && logs[i].origin == nfa::ORIGIN_EVENT) || logs[i].type == nfa::LOG_PURGE;
    };
    std::vector<size_t> evp;  // pushes made while processing events, applied at their positions
    size_t nfire_logs = 0;
    for (size_t i = 0; i < logs.size();) {
        size_t j = i;
        while (j < logs.size() && logs[j].key == logs[i].key) ++j;
        KC& c = K(logs[i].key);
        c.i = (uint32_t)i;
        c.e = (uint32_t)j;
        for (size_t x = i; x < j; ++x) {
            if (is_evpush(x)) evp.push_back(x);
            nfire_logs += logs[x].type == nfa::LOG_FIRE;
        }
        i = j;
    }
    out.rank.reserve(nfire_logs + nfire_logs / 4 + 16);  // ~ one entry per fire (grows if the scheduler fires more)
    prof.lap(9);
    {  // by position, stable: sort (position + 1, record index) packed in one word (no record loads in the sort)
        std::vector<uint64_t> pk(evp.size());
        for (size_t x = 0; x < evp.size(); ++x) pk[x] = ((uint64_t)(posof(evp[x]) + 1) << 32) | (uint64_t)evp[x];
        std::sort(pk.begin(), pk.end());
        for (size_t x = 0; x < evp.size(); ++x) evp[x] = (size_t)(pk[x] & 0xFFFFFFFFu);
    }
    prof.lap(10);
    auto next_fire = [&](KC& c) -> size_t {  // the key's next device fire (event pushes go by position)
        while (c.i < c.e && is_evpush(c.i)) ++c.i;
        return c.i < c.e && logs[c.i].type == nfa::LOG_FIRE ? c.i : NONE;
    };
    using HE = std::pair<int64_t, uint32_t>;
    struct MergeQ {  // a sorted initial run + a heap for later pushes (min first)
        std::vector<HE> a;
        size_t ai = 0;
        std::priority_queue<HE, std::vector<HE>, std::greater<HE>> h;
        bool empty() const { return ai == a.size() && h.empty(); }
        const HE& top() const {
            if (ai == a.size()) return h.top();
            if (h.empty()) return a[ai];
            return h.top() < a[ai] ? h.top() : a[ai];
        }
        void pop() {
            if (ai < a.size() && (h.empty() || !(h.top() < a[ai]))) ++ai;
            else h.pop();
        }
        void push(const HE& x) { h.push(x); }
    };
    MergeQ fireq;
    for (uint32_t key : touched) {
        const size_t f = next_fire(kc[key]);
        if (f != NONE) fireq.a.push_back({(int64_t)logs[f].g, key});
    }
    std::sort(fireq.a.begin(), fireq.a.end());
    std::priority_queue<HE, std::vector<HE>, std::greater<HE>> rowq;
    prof.lap(11);
    auto first_row_at = [&](uint32_t key, int64_t g) -> int64_t {  // position of the key's first row at >= g
        if (key >= (uint32_t)rows.K) return -1;
        int64_t a = rows.seg_b[key], b = rows.seg_e[key];
        while (a < b) {
            const int64_t m = (a + b) >> 1;
            if (rows.pos(m) < g) a = m + 1;
            else b = m;
        }
        return a < (int64_t)rows.seg_e[key] ? rows.pos(a) : -1;
    };
    auto apply_run = [&](KC& c, uint32_t key) {  // the host run's new pops / pushes into the model
        KeyRun* r = c.run;
        for (; r->lread < r->lcount; ++r->lread) {
            const SchedLog& L = r->log[r->lread];
            if (L.type == nfa::LOG_PUSH) notify(L.sched, key, L.t);
            else if (L.type == nfa::LOG_POP) pop(L.sched, key);
            else if (L.type == nfa::LOG_PURGE) purge(key);
        }
    };
    auto add_fire = [&](KC& c, const nfa::TimerFire& f, uint32_t rk) {
        fl.push_back(FN{f, -1, rk});
        const int32_t x = (int32_t)fl.size() - 1;
        if (c.ft >= 0) fl[c.ft].next = x;
        else c.fh = x;
        c.ft = x;
    };
    // replay the key on the host up to position g (its rows < g, the scheduler's fires so far except `skip_last`)
    auto takeover = [&](uint32_t key, int64_t g, bool skip_last) {
        KC& c = K(key);
        c.mode = HOST;
        c.run = take_over(key);
        for (int32_t x = c.fh; x >= 0; x = fl[x].next) {
            if (skip_last && x == c.ft) break;
            c.run->rows_before(fl[x].f.g);
            c.run->fire(fl[x].f.sched, fl[x].f.g, fl[x].f.clock);
            // the replay's records of this fire sit at the scheduler's position (a device fire accepted as
            // shifted was ranked under the device's position)
            out.rank.put(rank_key(fl[x].f.g, fl[x].f.sched, key), Slot{fl[x].f.g, fl[x].rank});
        }
        c.run->rows_before(g);
        c.run->lread = c.run->lcount;  // what the replay pushed / popped is in the model already
        out.taken.push_back(key);
        const int64_t nr = c.run->next_row_pos();
        if (nr >= 0) rowq.push({nr, key});
    };
    uint32_t rank = 0;
    // the scheduler fires (sch, key) at position g with currentTime() = clock
    auto fire = [&](int sch, uint32_t key, uint32_t g, int64_t clock) {
        const uint32_t rk = rank++;
        ++out.n_fires;
        KC& c = K(key);
        add_fire(c, nfa::TimerFire{g, sch, clock}, rk);
        rec(key, g, OP_FIRE, sch, clock);
        if (c.mode != HOST) {
            const size_t f = next_fire(c);
            bool ok = f != NONE && logs[f].sched == sch && (int64_t)logs[f].g <= (int64_t)g;
            size_t end = NONE;
            if (ok) {  // the fire's records end with LOG_FIRE_END (t = the largest clock it holds for)
                for (size_t x = f + 1; x < c.e; ++x)
                    if (logs[x].type == nfa::LOG_FIRE_END) { end = x; break; }
                ok = end != NONE && (logs[f].g == g ? logs[f].t == clock : clock <= logs[end].t && c.mode == PENDING);
                if (!ok && optimistic && end != NONE) {  // apply its records anyway; the device reruns the key
                    ok = true;
                    c.reordered = true;
                }
            }
            if (ok) {
                for (size_t x = f + 1; x < end; ++x) {
                    const SchedLog& L = logs[x];
                    if (L.type == nfa::LOG_POP) {
                        pop(L.sched, key);
                        rec(key, g, OP_POP, L.sched, 0);
                    } else if (L.type == nfa::LOG_PUSH) {
                        notify(L.sched, key, L.t);
                        rec(key, g, OP_NOTIFY, L.sched, L.t);
                    }
                }
                // Scheduler.sendTimerEvents pops every queued time <= currentTime in this one fire. A device fire
                // made at an earlier clock may have left some of them (only the optimistic pass accepts such a
                // fire, c.reordered): without this the model would fire the key again at the next advance -- a
                // fire the reference never makes, which the rerun would then execute
                while (queued(sch, key) && head(sch, key) <= clock) pop(sch, key);
                if (logs[f].g != g) {
                    ++out.n_shifted;
                    ++c.nshift;
                }
                out.rank.put(rank_key(logs[f].g, sch, key), Slot{g, rk});
                c.i = (uint32_t)(end + 1);
                c.mode = DEV;
                const size_t nf = next_fire(c);
                if (nf != NONE) fireq.push({(int64_t)logs[nf].g, key});
                return;
            }
            if (optimistic) {  // no such device fire: model its pops, rerun the key on the device
                c.reordered = true;
                while (queued(sch, key) && head(sch, key) <= clock) pop(sch, key);
                out.rank.put(rank_key(g, sch, key), Slot{g, rk});
                return;
            }
            takeover(key, g, true);
        }
        c.run->rows_before(g);
        c.run->fire(sch, g, clock);
        apply_run(c, key);
        out.rank.put(rank_key(g, sch, key), Slot{g, rk});
    };
    int64_t lb_t = INT64_MIN, lb_v = 0;  // last lower_bound over the clock (the earliest due time rarely changes)
    auto next_due = [&](int64_t from) -> int64_t {
        int64_t hmin = INT64_MAX, t;
        OKey k;
        for (SchedState& S : work_.sc)
            if (due_front(S, t, k)) hmin = std::min(hmin, t);
        if (hmin == INT64_MAX) return bc.G;
        if (hmin != lb_t) {
            lb_t = hmin;
            lb_v = std::lower_bound(bc.clk.begin(), bc.clk.end(), hmin) - bc.clk.begin();
        }
        const int64_t lb = lb_v;
        const int64_t x = std::max(from, lb);
        return x >= bc.G ? bc.G : (int64_t)bc.nadv[x];
    };
    size_t ep = 0;
    for (; ep < evp.size() && posof(evp[ep]) < 0; ++ep) {  // an unpartitioned query's init at start
        const SchedLog& L = logs[evp[ep]];
        if (K(L.key).mode != DEV) continue;
        if (L.type == nfa::LOG_PURGE) {
            purge(L.key);
            rec(L.key, L.g, OP_PURGE, 0, 0);
        } else {
            notify(L.sched, L.key, L.t);
            rec(L.key, L.g, OP_NOTIFY, L.sched, L.t);
        }
    }
    int64_t g = 0;
    std::vector<std::pair<int64_t, uint32_t>> W;
    prof.lap(1);
    while (true) {
        int64_t nxt = ep < evp.size() ? posof(evp[ep]) : bc.G;
        nxt = std::min(nxt, next_due(g));
        if (!fireq.empty()) nxt = std::min(nxt, fireq.top().first);
        if (!rowq.empty()) nxt = std::min(nxt, rowq.top().first);
        nxt = std::max(nxt, g);
        prof.lap(7);
        if (nxt >= bc.G) break;
        g = nxt;
        // 1. the clock advance at g: TimeChangeListeners (playback) / live_fire_until
        if (bc.adv[g]) {
            rank = 0;
            const int64_t clock = bc.clk[g];
            if (!live_) {
                for (int s = 0; s < n_sched_; ++s) {  // registration order; per listener a TreeMultimap, one per time
                    SchedState& S = work_.sc[s];
                    W.clear();
                    for (auto it = S.due.begin(); it != S.due.end() && it->first <= clock;) {
                        heap_fix(S, it->second);
                        std::vector<DueE>& h = it->second.h;
                        while (!h.empty() && stale(S, h.front())) {
                            std::pop_heap(h.begin(), h.end(), std::greater<DueE>());
                            h.pop_back();
                        }
                        if (h.empty()) {
                            it = S.due.erase(it);
                            continue;
                        }
                        W.push_back({it->first, h.front().k.key});
                        ++it;
                    }
                    for (size_t wi = 0; wi < W.size(); ++wi) {
                        if (wi + 4 < W.size()) {  // the keys' cursors and queue entries ahead (random keys)
                            const uint32_t kf = W[wi + 4].second;
                            __builtin_prefetch(&kc[kf]);
                            __builtin_prefetch(&S.ks[kf]);
                            if (kc[kf].i < logs.size()) __builtin_prefetch(&logs[kc[kf].i]);
                        }
                        fire(s, W[wi].second, (uint32_t)g, clock);
                    }
                    for (auto& w : W) remove_if_empty(s, w.second);  // returnAllStates
                }
            } else {
                int64_t now = g > 0 ? bc.clk[g - 1] : bc.clock0;
                while (true) {  // the earliest due (time, creation) across every scheduler, one at a time
                    int bs = -1;
                    int64_t bt = 0, t;
                    OKey bk{}, k;
                    for (int s = 0; s < n_sched_; ++s) {
                        if (!due_front(work_.sc[s], t, k) || t > clock) continue;
                        if (bs < 0 || t < bt || (t == bt && k.a < bk.a)) { bs = s; bt = t; bk = k; }
                    }
                    if (bs < 0) break;
                    now = std::max(now, bt);
                    fire(bs, bk.key, (uint32_t)g, now);
                    remove_if_empty(bs, bk.key);
                }
            }
        }
        prof.lap(2);
        // 2. device fires at <= g the scheduler did not make (yet): the key waits for its delayed fire
        while (!fireq.empty() && fireq.top().first <= g) {
            const uint32_t key = fireq.top().second;
            const int64_t fg = fireq.top().first;
            fireq.pop();
            KC& c = kc[key];
            if (c.mode != DEV) continue;
            const size_t f = next_fire(c);
            if (f == NONE || (int64_t)logs[f].g != fg) continue;  // made already
            c.mode = PENDING;
            const int64_t r = first_row_at(key, fg);  // an event of the key before the delayed fire: diverged
            if (r >= 0) rowq.push({r, key});
        }
        prof.lap(3);
        // 3. rows at g of keys that wait for a delayed fire (diverged) or run on the host
        while (!rowq.empty() && rowq.top().first <= g) {
            const uint32_t key = rowq.top().second;
            rowq.pop();
            KC& c = kc[key];
            if (c.mode == DEV) continue;
            if (c.mode == PENDING && optimistic) {  // its event comes before the delayed fire: reorder
                c.reordered = true;
                continue;
            }
            if (c.mode == PENDING) takeover(key, g, false);
            if (c.run->next_row_pos() != g) continue;
            c.run->row_at(g);
            apply_run(c, key);
            const int64_t nr = c.run->next_row_pos();
            if (nr >= 0) rowq.push({nr, key});
        }
        prof.lap(4);
        // 4. the device keys' pushes made by the event at g
        for (; ep < evp.size() && posof(evp[ep]) == g; ++ep) {
            // the pushes are in position order but the keys' state is scattered: prefetch the log records a few
            // pushes ahead, and the model entries of the nearer ones (the pass was bound by these cache misses)
            if (ep + 16 < evp.size()) __builtin_prefetch(&logs[evp[ep + 16]]);
            if (ep + 8 < evp.size()) {
                const SchedLog& Lf = logs[evp[ep + 8]];
                __builtin_prefetch(&kc[Lf.key]);
                if (Lf.sched < work_.sc.size() && Lf.key < work_.sc[Lf.sched].ks.size()) {
                    __builtin_prefetch(&work_.sc[Lf.sched].ks[Lf.key]);
                    if (Lf.key < key_hash.size()) __builtin_prefetch(&key_hash[Lf.key]);
                }
            }
            const SchedLog& L = logs[evp[ep]];
            const uint8_t m = kc[L.key].mode;
            if (m != DEV && !(optimistic && m == PENDING)) continue;
            if (L.type == nfa::LOG_PURGE) {
                purge(L.key);
                rec(L.key, L.g, OP_PURGE, 0, 0);
            } else {
                notify(L.sched, L.key, L.t);
                rec(L.key, L.g, OP_NOTIFY, L.sched, L.t);
            }
        }
        ++g;
        prof.lap(5);
    }
    std::sort(touched.begin(), touched.end());
    if (optimistic) {  // the reordered keys (incl. device fires never made here), with the scheduler's fire lists
        for (uint32_t k : touched) {
            KC& c = kc[k];
            if (c.reordered || c.mode == PENDING || next_fire(c) != NONE) out.reordered.push_back(k);
        }
        out.fire_off.push_back(0);
        for (uint32_t k : out.reordered) {
            for (int32_t x = kc[k].fh; x >= 0; x = fl[x].next) {
                out.fires.push_back(fl[x].f);
                out.fire_rank.push_back(fl[x].rank);
            }
            out.fire_off.push_back((uint32_t)out.fires.size());
        }
        // the reordered keys' model changes, grouped by key (stable), and the shifted fires of the others
        std::vector<int32_t> rd(nkeys, -1);  // dense (not kc[].rd): the ops are in time order, keys at random
        for (size_t d = 0; d < out.reordered.size(); ++d) rd[out.reordered[d]] = (int32_t)d;
        out.trace_off.assign(out.reordered.size() + 1, 0);
        for (const KOp& o : kops)
            if (rd[o.key] >= 0) ++out.trace_off[rd[o.key] + 1];
        for (size_t d = 0; d < out.reordered.size(); ++d) out.trace_off[d + 1] += out.trace_off[d];
        out.trace.resize(out.trace_off.back());
        {
            std::vector<uint32_t> wp(out.trace_off.begin(), out.trace_off.end() - 1);
            for (const KOp& o : kops)
                if (rd[o.key] >= 0) out.trace[wp[rd[o.key]]++] = o.op;
        }
        for (uint32_t k : touched)
            if (rd[k] < 0) out.n_shifted_kept += kc[k].nshift;
        prof.lap(6);
        prof.print("optimistic", logs.size(), evp.size(), out.n_fires);
        return;
    }
    // device fires the scheduler never made in this batch (delayed past its end): host replay without them
    std::vector<uint32_t> late;
    for (uint32_t k : touched) {
        KC& c = kc[k];
        if (c.mode == PENDING || (c.mode == DEV && next_fire(c) != NONE)) late.push_back(k);
    }
    for (uint32_t key : late) {
        takeover(key, bc.G, false);
        apply_run(kc[key], key);
    }
    for (uint32_t k : touched)
        if (kc[k].mode == HOST) {
            kc[k].run->rows_before(bc.G);
            apply_run(kc[k], k);
        }
    std::sort(out.taken.begin(), out.taken.end());
    prof.lap(6);
    prof.print("exact", logs.size(), evp.size(), out.n_fires);
}

bool SchedSim::confirm(const std::vector<nfa::SchedLog>& logs, Result& res) const {
    using nfa::SchedLog;
    std::vector<Op> got;
    size_t i = 0;
    for (size_t d = 0; d < res.reordered.size(); ++d) {
        const uint32_t key = res.reordered[d];
        i = std::lower_bound(logs.begin() + i, logs.end(), key,
                             [](const SchedLog& L, uint32_t k) { return L.key < k; }) - logs.begin();
        size_t j = i;
        while (j < logs.size() && logs[j].key == key) ++j;
        // the changes the exact pass would make for the key if every fire of its new run is consistent
        got.clear();
        for (size_t x = i; x < j; ++x) {
            const SchedLog& L = logs[x];
            if (L.type == nfa::LOG_PUSH && L.origin == nfa::ORIGIN_EVENT) {
                got.push_back(Op{L.g, OP_NOTIFY, L.sched, L.t});
            } else if (L.type == nfa::LOG_PURGE) {
                got.push_back(Op{L.g, OP_PURGE, 0, 0});
            } else if (L.type == nfa::LOG_FIRE) {
                got.push_back(Op{L.g, OP_FIRE, L.sched, L.t});
                size_t y = x + 1;
                for (; y < j && logs[y].type != nfa::LOG_FIRE_END; ++y) {
                    if (logs[y].type == nfa::LOG_POP) got.push_back(Op{L.g, OP_POP, logs[y].sched, 0});
                    else if (logs[y].type == nfa::LOG_PUSH) got.push_back(Op{L.g, OP_NOTIFY, logs[y].sched, logs[y].t});
                }
                if (y == j) return false;  // a fire without its end record
                x = y;
            } else {
                return false;  // a pop / scheduler push outside a fire: not a shape the comparison covers
            }
        }
        const size_t b = res.trace_off[d], e = res.trace_off[d + 1];
        if (got.size() != e - b || !std::equal(got.begin(), got.end(), res.trace.begin() + b)) {
            if (std::getenv("SDG_SCHED_PROF")) {  // diagnostics: the first difference
                size_t x = 0;
                while (x < got.size() && b + x < e && got[x] == res.trace[b + x]) ++x;
                auto pr = [](const char* w, const Op* o) {
                    if (o) std::fprintf(stderr, "  %s g %u kind %d sched %d t %lld\n", w, o->g, o->kind, o->sched, (long long)o->t);
                    else std::fprintf(stderr, "  %s (none)\n", w);
                };
                std::fprintf(stderr, "[sched confirm] key %u differs at op %zu of %zu / %zu\n", key, x, got.size(), e - b);
                pr("rerun", x < got.size() ? &got[x] : nullptr);
                pr("trace", b + x < e ? &res.trace[b + x] : nullptr);
            }
            return false;
        }
        i = j;
    }
    for (size_t d = 0; d < res.reordered.size(); ++d)  // the reruns' fires sit at the scheduler's positions now
        for (uint32_t x = res.fire_off[d]; x < res.fire_off[d + 1]; ++x) {
            const nfa::TimerFire& f = res.fires[x];
            res.rank.put(rank_key(f.g, f.sched, res.reordered[d]), Slot{f.g, res.fire_rank[x]});
        }
    res.n_shifted = res.n_shifted_kept;
    res.taken.clear();
    return true;
}

namespace {
template <class T>
void put(std::vector<uint8_t>& o, const T& v) {
    const uint8_t* b = (const uint8_t*)&v;
    o.insert(o.end(), b, b + sizeof(T));
}
template <class T>
void put_vec(std::vector<uint8_t>& o, const std::vector<T>& v) {
    put<uint64_t>(o, v.size());
    const uint8_t* b = (const uint8_t*)v.data();
    o.insert(o.end(), b, b + v.size() * sizeof(T));
}
template <class T>
T get(const uint8_t*& p, const uint8_t* end) {
    if (p + sizeof(T) > end) throw std::runtime_error("snapshot: truncated scheduler state");
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
}
template <class T>
void get_vec(const uint8_t*& p, const uint8_t* end, std::vector<T>& v) {
    const uint64_t n = get<uint64_t>(p, end);
    if (n > (uint64_t)(end - p) / sizeof(T)) throw std::runtime_error("snapshot: truncated scheduler state");
    v.resize(n);
    std::memcpy(v.data(), p, n * sizeof(T));
    p += n * sizeof(T);
}
}  // namespace

void SchedSim::save(std::vector<uint8_t>& o) const {
    put<uint32_t>(o, (uint32_t)cur_.sc.size());
    for (const SchedState& S : cur_.sc) {
        put_vec(o, S.ks);
        put<uint64_t>(o, S.due.size());
        for (const auto& kv : S.due) {  // (every heap written keyed for the current capacity)
            put<int64_t>(o, kv.first);
            Heap H = kv.second;
            heap_fix(const_cast<SchedState&>(S), H);
            put_vec(o, H.h);
        }
        put<uint64_t>(o, S.cap);
        put<uint64_t>(o, S.threshold);
        put<uint64_t>(o, S.size);
        put<uint64_t>(o, S.stamp);
        put_vec(o, S.bin);
    }
    put<uint64_t>(o, cur_.spill.size());
    for (const auto& d : cur_.spill) put_vec(o, std::vector<int64_t>(d.begin(), d.end()));
    put_vec(o, cur_.spill_free);
    put<uint64_t>(o, cur_.cseq);
}

const uint8_t* SchedSim::load(const uint8_t* p, const uint8_t* end) {
    State st;
    const uint32_t ns = get<uint32_t>(p, end);
    if ((int)ns != n_sched_) throw std::runtime_error("snapshot: scheduler count differs from the app's");
    st.sc.resize(ns);
    for (SchedState& S : st.sc) {
        get_vec(p, end, S.ks);
        for (size_t i = 0; i < S.ks.size(); ++i)
            if (S.ks[i].in_map) S.kend = i + 1;
        const uint64_t nd = get<uint64_t>(p, end);
        for (uint64_t i = 0; i < nd; ++i) {
            const int64_t t = get<int64_t>(p, end);
            get_vec(p, end, S.due[t].h);
        }
        S.cap = get<uint64_t>(p, end);
        for (auto& kv : S.due) kv.second.cap = S.cap;  // (saved keyed for it)
        S.threshold = get<uint64_t>(p, end);
        S.size = get<uint64_t>(p, end);
        S.stamp = get<uint64_t>(p, end);
        get_vec(p, end, S.bin);
    }
    const uint64_t nsp = get<uint64_t>(p, end);
    st.spill.resize(nsp);
    for (auto& d : st.spill) {
        std::vector<int64_t> v;
        get_vec(p, end, v);
        d.assign(v.begin(), v.end());
    }
    get_vec(p, end, st.spill_free);
    st.cseq = get<uint64_t>(p, end);
    cur_ = std::move(st);
    return p;
}

}  // namespace sdg
