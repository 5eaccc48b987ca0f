// Scheduler simulation over the per-key fire/notify logs (see sched.h for the reference semantics it follows).
#include "sched.h"

#include <algorithm>
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
                        const std::vector<int32_t>& key_hash, Result& out) {
    using nfa::SchedLog;
    work_ = cur_;
    hash_ = &key_hash;
    out = Result{};
    // per-key cursors over the log (sorted by key, kseq); event-origin pushes by position
    struct Cur {
        size_t i = 0, e = 0;
        bool div = false;
        std::vector<nfa::TimerFire> fires;
    };
    std::unordered_map<uint32_t, Cur> cur;
    std::vector<size_t> evp;
    for (size_t i = 0; i < logs.size();) {
        size_t j = i;
        while (j < logs.size() && logs[j].key == logs[i].key) ++j;
        Cur& c = cur[logs[i].key];
        c.i = i;
        c.e = j;
        for (size_t x = i; x < j; ++x)
            if (logs[x].type == nfa::LOG_PUSH && logs[x].origin == nfa::ORIGIN_EVENT) evp.push_back(x);
        i = j;
    }
    // position of a record; UINT32_MAX = before position 0 (an unpartitioned query's init at start)
    auto posof = [&](size_t i) -> int64_t { return logs[i].g == 0xFFFFFFFFu ? -1 : (int64_t)logs[i].g; };
    std::stable_sort(evp.begin(), evp.end(), [&](size_t a, size_t b) { return posof(a) < posof(b); });
    static const bool dbg = getenv("SDG_SCHED_DEBUG") != nullptr;
    if (dbg) {
        fprintf(stderr, "sim: G=%lld clock0=%lld logs=%zu\n", (long long)bc.G, (long long)bc.clock0, logs.size());
        for (int64_t g = 0; g < bc.G; ++g)
            fprintf(stderr, "  pos %lld clk %lld adv %d\n", (long long)g, (long long)bc.clk[g], bc.adv[g]);
        for (const auto& L : logs)
            fprintf(stderr, "  log key %u kseq %u g %u type %d sched %d origin %d t %lld\n", L.key, L.kseq, L.g, L.type,
                    L.sched, L.origin, (long long)L.t);
    }
    auto skip_events = [&](Cur& c) {
        while (c.i < c.e && logs[c.i].type == nfa::LOG_PUSH && logs[c.i].origin == nfa::ORIGIN_EVENT) ++c.i;
    };
    uint32_t rank = 0;
    // one fire of (sch, key) at position g with currentTime() = clock: replay the run's own record of it when
    // the run fired the same way, else model it (pops only) and mark the key for a rerun
    auto fire = [&](int sch, uint32_t key, uint32_t g, int64_t clock) {
        if (dbg) fprintf(stderr, "  sim fire sched %d key %u g %u clock %lld\n", sch, key, g, (long long)clock);
        out.rank[rank_key(g, sch, key)] = rank++;
        ++out.n_fires;
        Cur& c = cur[key];
        c.fires.push_back(nfa::TimerFire{g, sch, clock});
        skip_events(c);
        if (!c.div && c.i < c.e && logs[c.i].type == nfa::LOG_FIRE && logs[c.i].g == g && logs[c.i].sched == sch &&
            logs[c.i].t == clock) {
            ++c.i;
            while (c.i < c.e) {
                const SchedLog& L = logs[c.i];
                if (L.type == nfa::LOG_POP) {
                    const KS& k = work_.sc[L.sched].ks[key];
                    if (L.sched != sch || k.q.empty() || k.q.front() != L.t) {
                        c.div = true;  // inconsistent with the model: redo this key
                        break;
                    }
                    pop(sch, key);
                } else if (L.type == nfa::LOG_PUSH && L.origin == (uint8_t)sch && L.g == g) {
                    notify(L.sched, key, L.t);
                } else {
                    break;
                }
                ++c.i;
            }
            if (!c.div) return;
        }
        c.div = true;
        KS& k = work_.sc[sch].ks[key];  // sendTimerEvents: pop the FIFO while its head is due
        while (!k.q.empty() && k.q.front() <= clock) pop(sch, key);
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
    for (; ep < evp.size() && posof(evp[ep]) < 0; ++ep) notify(logs[evp[ep]].sched, logs[evp[ep]].key, logs[evp[ep]].t);
    int64_t g = 0;
    while (g < bc.G) {
        int64_t nxt = ep < evp.size() ? posof(evp[ep]) : bc.G;
        nxt = std::min(nxt, next_due(g));
        if (nxt >= bc.G) break;
        g = nxt;
        if (bc.adv[g]) {
            rank = 0;
            const int64_t clock = bc.clk[g];
            if (!live_) {
                // TimeChangeListeners in registration order; each: TreeMultimap of the due states, one per time
                for (int s = 0; s < n_sched_; ++s) {
                    SchedState& S = work_.sc[s];
                    std::vector<std::pair<int64_t, uint32_t>> W;
                    for (auto it = S.due.begin(); it != S.due.end() && it->first <= clock; ++it)
                        W.push_back({it->first, it->second.begin()->key});
                    for (auto& w : W) fire(s, w.second, (uint32_t)g, clock);
                    for (auto& w : W) remove_if_empty(s, w.second);  // returnAllStates
                }
            } else {
                // live_fire_until: the earliest due (time, creation) across every scheduler, one at a time
                int64_t now = g > 0 ? bc.clk[g - 1] : bc.clock0;
                while (true) {
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
        while (ep < evp.size() && posof(evp[ep]) == g) {  // the event's own pushes (after the fires)
            const SchedLog& L = logs[evp[ep]];
            notify(L.sched, L.key, L.t);
            ++ep;
        }
        ++g;
    }
    // fires a run performed that the scheduler did not: diverged too
    for (auto& kv : cur) {
        Cur& c = kv.second;
        if (c.div) continue;
        for (size_t x = c.i; x < c.e; ++x)
            if (logs[x].type != nfa::LOG_PUSH || logs[x].origin != nfa::ORIGIN_EVENT) { c.div = true; break; }
    }
    for (auto& kv : cur)
        if (kv.second.div) out.diverged.push_back(kv.first);
    std::sort(out.diverged.begin(), out.diverged.end());
    out.fire_off.push_back(0);
    for (uint32_t k : out.diverged) {
        const Cur& c = cur[k];
        out.fires.insert(out.fires.end(), c.fires.begin(), c.fires.end());
        out.fire_off.push_back((uint32_t)out.fires.size());
    }
}

}  // namespace sdg
