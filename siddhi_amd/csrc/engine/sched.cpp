// Scheduler simulation over the per-key fire/notify logs (see sched.h for the reference semantics it follows).
#include "sched.h"

#include <algorithm>
#include <queue>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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
        for (const auto& kv : S.ks)
            if (!kv.second.q.empty()) out.push_back(kv.first);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
}

SchedSim::OKey SchedSim::okey(const SchedState& S, const KS& k, uint32_t key) const {
    if (live_) return OKey{k.cseq, 0, key};                         // (time, creation order)
    if (!partitioned_) return OKey{0, 0, key};                       // one state
    return OKey{(uint32_t)k.hash & (S.cap - 1), ~k.stamp, key};     // HashMap iteration order
}

void SchedSim::due_add(SchedState& S, uint32_t key, const KS& k) { S.due[k.q.front()].insert(okey(S, k, key)); }

void SchedSim::due_del(SchedState& S, uint32_t key, const KS& k) {
    auto it = S.due.find(k.q.front());
    if (it == S.due.end()) return;
    it->second.erase(okey(S, k, key));
    if (it->second.empty()) S.due.erase(it);
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
    S.due.clear();
    for (auto& kv : S.ks) {
        if (!kv.second.in_map) continue;
        S.bin[(uint32_t)kv.second.hash & (S.cap - 1)]++;
        if (!kv.second.q.empty()) due_add(S, kv.first, kv.second);
    }
}

void SchedSim::notify(int sch, uint32_t key, int64_t t) {
    SchedState& S = work_.sc[sch];
    KS& k = S.ks[key];
    if (partitioned_) {
        if (S.size > S.threshold || S.cap == 0) resize(S);  // computeIfAbsent: resize before the lookup
        if (!k.in_map) {
            k.hash = (*hash_)[key];
            k.in_map = true;
            k.stamp = ++S.stamp;
            k.cseq = ++work_.cseq;
            uint32_t& bc = S.bin[(uint32_t)k.hash & (S.cap - 1)];
            const uint32_t before = bc++;
            ++S.size;
            if (before >= 7 && S.cap < 64) resize(S);  // treeifyBin on a table below MIN_TREEIFY_CAPACITY
        }
    } else if (!k.in_map) {  // SingleStateHolder: created on first use, never removed
        k.in_map = true;
        k.cseq = ++work_.cseq;
    }
    const bool was_empty = k.q.empty();
    k.q.push_back(t);
    if (was_empty) due_add(S, key, k);
}

void SchedSim::pop(int sch, uint32_t key) {
    SchedState& S = work_.sc[sch];
    KS& k = S.ks[key];
    if (k.q.empty()) return;
    due_del(S, key, k);
    k.q.pop_front();
    if (!k.q.empty()) due_add(S, key, k);
}

void SchedSim::remove_if_empty(int sch, uint32_t key) {  // returnState / returnAllStates of a drained state
    if (!partitioned_) return;
    SchedState& S = work_.sc[sch];
    auto it = S.ks.find(key);
    if (it == S.ks.end() || !it->second.q.empty() || !it->second.in_map) return;
    S.bin[(uint32_t)it->second.hash & (S.cap - 1)]--;
    --S.size;
    S.ks.erase(it);
}

void SchedSim::simulate(const BatchClock& bc, const std::vector<nfa::SchedLog>& logs,
                        const std::vector<int32_t>& key_hash, const KeyRows& rows,
                        const std::function<KeyRun*(uint32_t)>& take_over, Result& out, bool optimistic) {
    using nfa::SchedLog;
    work_ = cur_;
    hash_ = &key_hash;
    out = Result{};
    constexpr size_t NONE = ~size_t(0);
    enum : uint8_t { DEV = 0, PENDING = 1, HOST = 2 };  // the key's history so far: its device run / a device fire
                                                      // the scheduler has not made yet / stepped on the host
    struct KC {
        size_t i = 0, e = 0;                 // cursor into the key's device records
        uint8_t mode = DEV;
        bool reordered = false;              // optimistic pass: the scheduler's order differs from the run's
        KeyRun* run = nullptr;
        std::vector<nfa::TimerFire> fires;   // the scheduler's fires of this key so far
    };
    std::unordered_map<uint32_t, KC> kc;
    auto posof = [&](size_t i) -> int64_t { return logs[i].g == 0xFFFFFFFFu ? -1 : (int64_t)logs[i].g; };
    auto is_evpush = [&](size_t i) { return logs[i].type == nfa::LOG_PUSH && logs[i].origin == nfa::ORIGIN_EVENT; };
    std::vector<size_t> evp;  // pushes made while processing events, applied at their positions
    for (size_t i = 0; i < logs.size();) {
        size_t j = i;
        while (j < logs.size() && logs[j].key == logs[i].key) ++j;
        KC& c = kc[logs[i].key];
        c.i = i;
        c.e = j;
        for (size_t x = i; x < j; ++x)
            if (is_evpush(x)) evp.push_back(x);
        i = j;
    }
    std::stable_sort(evp.begin(), evp.end(), [&](size_t a, size_t b) { return posof(a) < posof(b); });
    auto next_fire = [&](KC& c) -> size_t {  // the key's next device fire (event pushes go by position)
        while (c.i < c.e && is_evpush(c.i)) ++c.i;
        return c.i < c.e && logs[c.i].type == nfa::LOG_FIRE ? c.i : NONE;
    };
    using HE = std::pair<int64_t, uint32_t>;
    std::priority_queue<HE, std::vector<HE>, std::greater<HE>> fireq, rowq;
    for (auto& kv : kc) {
        const size_t f = next_fire(kv.second);
        if (f != NONE) fireq.push({(int64_t)logs[f].g, kv.first});
    }
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
        }
    };
    // replay the key on the host up to position g (its rows < g, the scheduler's fires so far except `skip_last`)
    auto takeover = [&](uint32_t key, int64_t g, bool skip_last) {
        KC& c = kc[key];
        c.mode = HOST;
        c.run = take_over(key);
        const size_t nf = c.fires.size() - (skip_last ? 1 : 0);
        for (size_t f = 0; f < nf; ++f) {
            c.run->rows_before(c.fires[f].g);
            c.run->fire(c.fires[f].sched, c.fires[f].g, c.fires[f].clock);
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
        KC& c = kc[key];
        c.fires.push_back(nfa::TimerFire{g, sch, clock});
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
                    if (L.type == nfa::LOG_POP) pop(L.sched, key);
                    else if (L.type == nfa::LOG_PUSH) notify(L.sched, key, L.t);
                }
                if (logs[f].g != g) ++out.n_shifted;
                out.rank[rank_key(logs[f].g, sch, key)] = Slot{g, rk};
                c.i = end + 1;
                c.mode = DEV;
                const size_t nf = next_fire(c);
                if (nf != NONE) fireq.push({(int64_t)logs[nf].g, key});
                return;
            }
            if (optimistic) {  // no such device fire: model its pops, rerun the key on the device
                c.reordered = true;
                KS& k = work_.sc[sch].ks[key];
                while (!k.q.empty() && k.q.front() <= clock) pop(sch, key);
                out.rank[rank_key(g, sch, key)] = Slot{g, rk};
                return;
            }
            takeover(key, g, true);
        }
        c.run->rows_before(g);
        c.run->fire(sch, g, clock);
        apply_run(c, key);
        out.rank[rank_key(g, sch, key)] = Slot{g, rk};
    };
    auto next_due = [&](int64_t from) -> int64_t {
        int64_t hmin = INT64_MAX;
        for (const SchedState& S : work_.sc)
            if (!S.due.empty()) hmin = std::min(hmin, S.due.begin()->first);
        if (hmin == INT64_MAX) return bc.G;
        const int64_t lb = std::lower_bound(bc.clk.begin(), bc.clk.end(), hmin) - bc.clk.begin();
        const int64_t x = std::max(from, lb);
        return x >= bc.G ? bc.G : (int64_t)bc.nadv[x];
    };
    size_t ep = 0;
    for (; ep < evp.size() && posof(evp[ep]) < 0; ++ep)  // an unpartitioned query's init at start
        if (kc[logs[evp[ep]].key].mode == DEV) notify(logs[evp[ep]].sched, logs[evp[ep]].key, logs[evp[ep]].t);
    int64_t g = 0;
    while (true) {
        int64_t nxt = ep < evp.size() ? posof(evp[ep]) : bc.G;
        nxt = std::min(nxt, next_due(g));
        if (!fireq.empty()) nxt = std::min(nxt, fireq.top().first);
        if (!rowq.empty()) nxt = std::min(nxt, rowq.top().first);
        nxt = std::max(nxt, g);
        if (nxt >= bc.G) break;
        g = nxt;
        // 1. the clock advance at g: TimeChangeListeners (playback) / live_fire_until
        if (bc.adv[g]) {
            rank = 0;
            const int64_t clock = bc.clk[g];
            if (!live_) {
                for (int s = 0; s < n_sched_; ++s) {  // registration order; per listener a TreeMultimap, one per time
                    SchedState& S = work_.sc[s];
                    std::vector<std::pair<int64_t, uint32_t>> W;
                    for (auto it = S.due.begin(); it != S.due.end() && it->first <= clock; ++it)
                        W.push_back({it->first, it->second.begin()->key});
                    for (auto& w : W) fire(s, w.second, (uint32_t)g, clock);
                    for (auto& w : W) remove_if_empty(s, w.second);  // returnAllStates
                }
            } else {
                int64_t now = g > 0 ? bc.clk[g - 1] : bc.clock0;
                while (true) {  // the earliest due (time, creation) across every scheduler, one at a time
                    int bs = -1;
                    int64_t bt = 0;
                    OKey bk{};
                    for (int s = 0; s < n_sched_; ++s) {
                        const SchedState& S = work_.sc[s];
                        if (S.due.empty() || S.due.begin()->first > clock) continue;
                        const int64_t t = S.due.begin()->first;
                        const OKey& k = *S.due.begin()->second.begin();
                        if (bs < 0 || t < bt || (t == bt && k.a < bk.a)) { bs = s; bt = t; bk = k; }
                    }
                    if (bs < 0) break;
                    now = std::max(now, bt);
                    fire(bs, bk.key, (uint32_t)g, now);
                    remove_if_empty(bs, bk.key);
                }
            }
        }
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
        // 4. the device keys' pushes made by the event at g
        for (; ep < evp.size() && posof(evp[ep]) == g; ++ep) {
            const uint8_t m = kc[logs[evp[ep]].key].mode;
            if (m == DEV || (optimistic && m == PENDING)) notify(logs[evp[ep]].sched, logs[evp[ep]].key, logs[evp[ep]].t);
        }
        ++g;
    }
    if (optimistic) {  // the reordered keys (incl. device fires never made here), with the scheduler's fire lists
        for (auto& kv : kc)
            if (kv.second.reordered || kv.second.mode == PENDING || next_fire(kv.second) != NONE)
                out.reordered.push_back(kv.first);
        std::sort(out.reordered.begin(), out.reordered.end());
        out.fire_off.push_back(0);
        for (uint32_t k : out.reordered) {
            const KC& c = kc[k];
            out.fires.insert(out.fires.end(), c.fires.begin(), c.fires.end());
            out.fire_off.push_back((uint32_t)out.fires.size());
        }
        return;
    }
    // device fires the scheduler never made in this batch (delayed past its end): host replay without them
    std::vector<uint32_t> late;
    for (auto& kv : kc)
        if (kv.second.mode == PENDING || (kv.second.mode == DEV && next_fire(kv.second) != NONE)) late.push_back(kv.first);
    std::sort(late.begin(), late.end());
    for (uint32_t key : late) {
        takeover(key, bc.G, false);
        apply_run(kc[key], key);
    }
    for (auto& kv : kc)
        if (kv.second.mode == HOST) {
            kv.second.run->rows_before(bc.G);
            apply_run(kv.second, kv.first);
        }
    std::sort(out.taken.begin(), out.taken.end());
}

}  // namespace sdg
