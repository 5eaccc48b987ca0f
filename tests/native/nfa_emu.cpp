#include <chrono>
// TEST-ONLY host harness: runs the product's generic keyed-NFA code (siddhi_amd/csrc/engine/nfa.h, the same
// __host__ __device__ functions the gfx950 kernel nfa_k executes) on the CPU, so its state-machine logic is
// checked against the oracle on every golden fixture without a GPU. Not part of the product: the product library
// has no CPU path, and nothing here is linked into it. Built by tests/native/Makefile into tests/native/_build.
//
// Batch semantics mirror engine.cpp's flush: per query, the pending events of its streams in arrival order,
// grouped by partition key (stable), each key's rows run through nfa::run_key with a per-key arena that persists
// across flushes; matches ordered by (sequence number of the emitting event, emission ordinal).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../siddhi_amd/csrc/engine/compile.h"
#include "../../siddhi_amd/csrc/engine/keyorder.h"
#include "../../siddhi_amd/csrc/engine/nfa.h"
#include "../../siddhi_amd/csrc/engine/keyrun.h"
#include "../../siddhi_amd/csrc/engine/sched.h"
#include "../../siddhi_amd/csrc/siddhiql/parser.h"

using namespace sdg;

namespace {

std::string g_err;
}  // namespace
void sdg::PartitionKeyOrder::throw_corrupt() { throw std::runtime_error("corrupt key order"); }
namespace {

int width_of(uint8_t kind) {
    switch (kind) {
        case VK_I64: case VK_F64: return 8;
        case VK_BOOL: return 1;
        default: return 4;
    }
}

struct Ev {
    int stream;  // -1: an advance_time point
    int64_t ts;
    std::vector<int64_t> vals;
    std::vector<uint8_t> nulls;
};

struct Out {
    int64_t seq, sub, ts;
    std::vector<int64_t> vals;
    uint32_t nulls;
};

struct EmuQuery {
    HostQuery hq;
    nfa::Layout L;
    std::map<std::string, int> keys;
    std::vector<int32_t> key_hash;
    std::vector<std::vector<uint8_t>> arenas;
    SchedSim sim;
    std::vector<Out> outs;
    bool bcast = false;              // a stream without a partition key: rows to every key, in korder order
    PartitionKeyOrder korder;
    struct Spilled {                 // as QueryRt::spill: keys past the device's 4096 partials, 32-bit arenas
        nfa::Layout L{};
        std::vector<uint8_t> arena;
    };
    std::map<uint32_t, Spilled> spill;
};

struct Emu {
    sql::App app;
    Interner strings;
    std::vector<std::unique_ptr<EmuQuery>> qs;
    std::vector<Ev> pending;
    int ns = 64;
    int64_t clock = 0;  // playback: lastEventTimestamp; live: the modelled wall clock
    int64_t seq = 0;    // positions flushed so far
};

std::string key_text(Emu* e, uint8_t kind, int64_t v) {
    switch (kind) {
        case VK_I32: return std::to_string((int32_t)v);
        case VK_I64: return std::to_string(v);
        case VK_F32: return java_real_string(bits_f32(v), true);
        case VK_F64: return java_real_string(bits_f64(v), false);
        case VK_BOOL: return v ? "true" : "false";
        default: return e->strings.strs[(uint32_t)v];
    }
}

// the batch clock over every pending position (TimestampGeneratorImpl.setCurrentTimestamp / live advance)
BatchClock batch_clock(Emu* e) {
    BatchClock bc;
    bc.G = (int64_t)e->pending.size();
    bc.clock0 = e->clock;
    bc.clk.resize(bc.G);
    bc.adv.resize(bc.G);
    bc.nadv.resize(bc.G + 1);
    int64_t c = e->clock;
    for (int64_t g = 0; g < bc.G; ++g) {
        const Ev& ev = e->pending[g];
        if (e->app.playback) {
            bc.adv[g] = ev.ts >= c;
            if (ev.ts >= c) c = ev.ts;
        } else {
            bc.adv[g] = ev.stream < 0;
            if (ev.stream < 0 && ev.ts > c) c = ev.ts;
        }
        bc.clk[g] = c;
    }
    bc.nadv[bc.G] = (uint32_t)bc.G;
    for (int64_t g = bc.G - 1; g >= 0; --g) bc.nadv[g] = bc.adv[g] ? (uint32_t)g : bc.nadv[g + 1];
    return bc;
}

size_t reordered_ = 0, taken_ = 0, exact_passes_ = 0;
double us_[3] = {0, 0, 0};
int g_reclaim = 0;      // emu_set_reclaim: every idle key goes through its idle record after each run (nfa.h to_idle)
int64_t idles_ = 0;     // keys rebuilt from an idle record (all flushes)
int64_t growths_ = 0;
int64_t spills_ = 0;    // keys moved to a 32-bit host arena (all flushes)  // arena doublings (all flushes)  // cumulative: optimistic pass, reruns, exact pass (microseconds)  // last flush's scheduler statistics (tests)

int flush_query(Emu* e, EmuQuery& q, const BatchClock& bc) {
    HostQuery& h = q.hq;
    const Plan& P = h.plan;
    const int nc = P.n_cols;
    std::vector<const Ev*> rows;
    std::vector<int> rkey;
    std::vector<uint32_t> rpos, rrank;
    for (int64_t g = 0; g < bc.G; ++g) {
        const Ev& ev = e->pending[g];
        if (ev.stream < 0) continue;
        int qpos = h.stream_pos(ev.stream);
        if (qpos < 0) continue;
        int key = 0;
        if (P.partitioned && h.key_attr[qpos] == -3) {  // every initialised key, in getPartitionKeys() order
            const std::vector<uint32_t>& o = q.korder.order();
            if (q.korder.tree_bins()) throw std::runtime_error("broadcast order: a tree bin (not modelled)");
            for (size_t x = 0; x < o.size(); ++x) {
                rows.push_back(&ev);
                rkey.push_back((int)o[x]);
                rpos.push_back((uint32_t)g);
                rrank.push_back((uint32_t)x);
            }
            continue;
        }
        if (P.partitioned) {
            int ai = h.key_attr[qpos];
            if (ev.nulls[ai]) continue;  // null partition key: dropped
            std::string kt = key_text(e, h.key_kind[qpos], ev.vals[ai]);
            auto it = q.keys.find(kt);
            if (it == q.keys.end()) {
                it = q.keys.emplace(kt, (int)q.keys.size()).first;
                q.key_hash.push_back(java_spread_hash(kt));
            }
            key = it->second;
            if (q.bcast) q.korder.add((uint32_t)key, q.key_hash[key]);
        }
        rows.push_back(&ev);
        rkey.push_back(key);
        rpos.push_back((uint32_t)g);
        rrank.push_back(0);
    }
    const int64_t n = (int64_t)rows.size();
    const int K = P.partitioned ? (int)q.keys.size() : 1;
    // stable grouping by key
    std::vector<uint32_t> order(n);
    for (int64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return rkey[a] < rkey[b]; });
    std::vector<int64_t> ts(std::max<int64_t>(n, 1));
    std::vector<uint8_t> qs(std::max<int64_t>(n, 1));
    std::vector<uint32_t> gpos(std::max<int64_t>(n, 1)), vrank(std::max<int64_t>(n, 1));
    std::vector<std::vector<uint8_t>> cols(nc), nulls(nc);
    std::vector<const void*> cptr(MAX_COLS, nullptr);
    std::vector<const uint8_t*> nptr(MAX_COLS, nullptr);
    for (int k = 0; k < nc; ++k) {
        cols[k].assign((size_t)std::max<int64_t>(n, 1) * width_of(P.col_kind[k]), 0);
        nulls[k].assign((size_t)std::max<int64_t>(n, 1), 0);
        cptr[k] = cols[k].data();
        nptr[k] = nulls[k].data();
    }
    std::vector<uint32_t> seg_b(K, 0), seg_e(K, 0);
    for (int64_t p = 0; p < n; ++p) {
        const Ev& ev = *rows[order[p]];
        int qpos = h.stream_pos(ev.stream);
        ts[p] = ev.ts;
        qs[p] = (uint8_t)qpos;
        gpos[p] = rpos[order[p]];
        vrank[p] = rrank[order[p]];
        for (int k = 0; k < nc; ++k) {
            int ai = h.col_attr[qpos][k];
            int w = width_of(P.col_kind[k]);
            if (ai < 0 || ev.nulls[ai]) {
                nulls[k][p] = 1;
                continue;
            }
            int64_t v = ev.vals[ai];
            std::memcpy(&cols[k][(size_t)p * w], &v, w);  // little endian: low bytes
        }
        int key = rkey[order[p]];
        if (p == 0 || rkey[order[p - 1]] != key) seg_b[key] = (uint32_t)p;
        seg_e[key] = (uint32_t)(p + 1);
    }
    while ((int)q.arenas.size() < K) q.arenas.emplace_back((size_t)q.L.bytes, 0);
    // keys this batch runs: rows, queued timers, the unpartitioned query's single key (initialised at start)
    std::vector<uint32_t> run;
    if (q.sim.active()) q.sim.queued_keys(run);
    for (int k = 0; k < K; ++k)
        if (seg_b[k] < seg_e[k] || !P.partitioned) run.push_back((uint32_t)k);
    std::sort(run.begin(), run.end());
    run.erase(std::unique(run.begin(), run.end()), run.end());
    std::map<uint32_t, std::vector<uint8_t>> backup;
    for (uint32_t k : run) backup[k] = q.arenas[k];
    std::map<uint32_t, std::vector<Out>> kout;
    std::map<uint32_t, std::vector<nfa::SchedLog>> klog;
    std::vector<int64_t> stk(STACK);
    bool arena_ovf = false;
    auto run_one = [&](uint32_t k, const nfa::TimerFire* fires, int nfires) -> int {
        const int64_t cap = 2 * (seg_e[k] - seg_b[k]) + 4096 + 64 * (int64_t)std::max(nfires, 0);
        // scratch reused across runs (grow-only: a per-key allocation of the log alone was 2 MB)
        static std::vector<int64_t> o_ts, o_vals, o_seq, o_sub;
        static std::vector<uint32_t> o_nulls, o_key;
        static std::vector<nfa::SchedLog> logs(1 << 16);
        auto grow = [](auto& v, size_t n) { if (v.size() < n) v.resize(n); };
        grow(o_ts, cap); grow(o_vals, (size_t)std::max(P.n_out, 1) * cap); grow(o_seq, cap); grow(o_sub, cap);
        grow(o_nulls, cap); grow(o_key, cap);
        unsigned long long count = 0, lcount = 0;
        int flags[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        auto setup = [&](auto& c, const nfa::Layout& L, uint8_t* base) {
            count = lcount = 0;
            std::fill(flags, flags + 8, 0);
            c.P = &P;
            c.code = h.code.data();
            c.consts = h.consts.data();
            c.L = L;
            c.base = base;
            c.stk = stk.data();
            c.stride = 1;
            c.emit_ts = o_ts.data();
            c.emit_vals = o_vals.data();
            c.emit_nulls = o_nulls.data();
            c.emit_seq = o_seq.data();
            c.emit_sub = o_sub.data();
            c.emit_key = o_key.data();
            c.emit_round = nullptr;
            c.round = 0;
            c.emit_count = &count;
            c.emit_cap = cap;
            c.flags = flags;
            c.key = k;
            c.T.G = bc.G;
            c.T.clk = bc.clk.data();
            c.T.nadv = bc.nadv.data();
            c.T.clock0 = bc.clock0;
            c.T.live = !e->app.playback;
            c.T.log = q.sim.active() ? logs.data() : nullptr;
            c.T.log_count = &lcount;
            c.T.log_cap = (int64_t)logs.size();
            c.fires = fires;
            c.nfires = nfires;
        };
        nfa::KeyEvents kev{ts.data(), qs.data(), gpos.data(), cptr.data(), nptr.data(), seg_b.size() > k ? seg_b[k] : 0,
                           seg_e.size() > k ? seg_e[k] : 0, e->seq, 0, q.bcast ? vrank.data() : nullptr};
        if (kev.b > kev.e) kev.b = kev.e;
        nfa::CtxT<true> c;
        auto spilled = q.spill.find(k);
        if (spilled == q.spill.end()) {
            setup(c, q.L, q.arenas[k].data());
            nfa::run_key(c, kev);
            // as the engine: a key past the largest device layout goes on on the host in a 32-bit layout of twice
            // the slots (queries without timers), from its batch-start state
            if (c.ovf() && q.L.ns >= 4096 && P.n_sched == 0 && !(P.purge && P.n_agg > 0)) {
                EmuQuery::Spilled& sp = q.spill[k];
                sp.L = nfa::make_layout<int32_t>(P.n_states, std::max(nc, 1), 2 * q.L.ns, P.n_sched);
                sp.arena.assign((size_t)sp.L.bytes, 0);
                nfa::CtxT<true, int32_t> d;
                d.P = &P;
                d.L = sp.L;
                d.base = sp.arena.data();
                nfa::migrate_key<int16_t>(d, backup[k].data(), q.L);
                q.arenas[k] = backup[k];
                ++spills_;
                spilled = q.spill.find(k);
            }
        }
        if (spilled != q.spill.end()) {
            EmuQuery::Spilled& sp = spilled->second;
            for (;;) {
                std::vector<uint8_t> work = sp.arena;  // batch-start state
                nfa::CtxT<true, int32_t> c32;
                setup(c32, sp.L, work.data());
                nfa::run_key(c32, kev);
                if (!c32.ovf()) {
                    sp.arena.swap(work);
                    break;
                }
                if (sp.L.ns >= (1 << 22)) {
                    g_err = "query '" + h.name + "': partial-match arena overflow (spilled key)";
                    return 3;
                }
                const nfa::Layout Ln = nfa::make_layout<int32_t>(P.n_states, std::max(nc, 1), 2 * sp.L.ns, P.n_sched);
                std::vector<uint8_t> na((size_t)Ln.bytes, 0);
                nfa::CtxT<true, int32_t> d;
                d.P = &P;
                d.L = Ln;
                d.base = na.data();
                nfa::migrate_key<int32_t>(d, sp.arena.data(), sp.L);
                sp.arena.swap(na);
                sp.L = Ln;
            }
        } else if (c.ovf()) {
            g_err = "query '" + h.name + "': partial-match arena overflow";
            arena_ovf = true;
            return 3;
        }
        if (flags[0] || flags[5]) {
            g_err = "output / scheduler log overflow";
            return 3;
        }
        std::vector<Out>& ko = kout[k];
        ko.clear();
        for (unsigned long long i = 0; i < count; ++i) {
            Out o{o_seq[i], o_sub[i], o_ts[i], {}, o_nulls[i]};
            for (int j = 0; j < P.n_out; ++j) o.vals.push_back(o_vals[(size_t)j * cap + i]);
            ko.push_back(std::move(o));
        }
        klog[k].assign(logs.begin(), logs.begin() + (int64_t)lcount);
        // as the engine's reclaiming queries: a key that ends idle keeps only its idle record; its arena is rebuilt
        // from it (here at once, on the device at the key's next batch -- the same state)
        if (g_reclaim && P.partitioned && P.n_sched == 0 && !P.purge && spilled == q.spill.end()) {
            std::vector<uint8_t> rec((size_t)nfa::idle_bytes(P.n_states));
            if (nfa::to_idle(c, rec.data())) {
                std::fill(q.arenas[k].begin(), q.arenas[k].end(), 0);
                nfa::CtxT<true> c2;
                c2.P = &P;
                c2.L = q.L;
                c2.base = q.arenas[k].data();
                nfa::from_idle(c2, rec.data());
                ++idles_;
            }
        }
        return 0;
    };
    // as the engine: a key out of partial-match slots doubles every key's arena (nfa.h migrate_key from the
    // batch-start state) and the batch reruns
    for (bool again = true; again;) {
        again = false;
        for (uint32_t k : run) {
            if (k >= seg_b.size() && P.partitioned) {  // a key of an earlier batch with queued timers only
                seg_b.resize(k + 1, 0);
                seg_e.resize(k + 1, 0);
            }
            arena_ovf = false;
            int rc = run_one(k, nullptr, -1);  // ideal mode
            if (rc && arena_ovf && q.L.ns < 4096) {
                const nfa::Layout Ln = nfa::make_layout(P.n_states, std::max(nc, 1), std::min(2 * q.L.ns, 4096), P.n_sched);
                for (size_t kk = 0; kk < q.arenas.size(); ++kk) {
                    auto bk = backup.find((uint32_t)kk);
                    const std::vector<uint8_t>& src = bk != backup.end() ? bk->second : q.arenas[kk];
                    std::vector<uint8_t> dst((size_t)Ln.bytes, 0);
                    nfa::CtxT<true> mc;
                    mc.P = &P;
                    mc.L = Ln;
                    mc.base = dst.data();
                    nfa::migrate_key(mc, src.data(), q.L);
                    q.arenas[kk] = dst;
                    if (bk != backup.end()) bk->second = dst;
                }
                q.L = Ln;
                kout.clear();
                klog.clear();
                ++growths_;
                again = true;
                break;
            }
            if (rc) return rc;
        }
    }
    SchedSim::Result res;
    std::vector<std::unique_ptr<KeyRun>> runs;
    if (q.sim.active()) {
        // one pass of the global scheduler (sched.h) over the runs' logs; keys it takes over run here on the host
        std::vector<nfa::SchedLog> all;
        for (auto& kv : klog) all.insert(all.end(), kv.second.begin(), kv.second.end());
        KeyRows kr;
        kr.seg_b = seg_b.data();
        kr.seg_e = seg_e.data();
        kr.K = (int64_t)seg_b.size();
        kr.orig = gpos.data();
        kr.n = n;
        nfa::TimerIn T{};
        T.G = bc.G;
        T.clk = bc.clk.data();
        T.nadv = bc.nadv.data();
        T.clock0 = bc.clock0;
        T.live = !e->app.playback;
        auto take = [&](uint32_t k) -> KeyRun* {
            runs.emplace_back(new KeyRun());
            KeyRun* r = runs.back().get();
            r->key = k;
            r->arena = backup[k];
            const int64_t b = k < seg_b.size() ? seg_b[k] : 0, en = k < seg_e.size() ? seg_e[k] : 0;
            for (int64_t p = b; p < en; ++p) {
                r->ts.push_back(ts[p]);
                r->qs.push_back(qs[p]);
                r->pos.push_back(gpos[p]);
                if (q.bcast) r->vrank.push_back(vrank[p]);
            }
            r->has_qs = true;
            r->cols.resize(nc);
            r->nulls.resize(nc);
            for (int c = 0; c < nc; ++c) {
                const int w = width_of(P.col_kind[c]);
                r->cols[c].assign(cols[c].begin() + b * w, cols[c].begin() + en * w);
                r->nulls[c].assign(nulls[c].begin() + b, nulls[c].begin() + en);
            }
            r->start(&P, h.code.data(), h.consts.data(), q.L, T, e->seq);
            return r;
        };
        if (const char* dump = getenv("SDG_SIM_DUMP")) {  // the optimistic pass's inputs (scripts/simbench.cpp)
            FILE* f = std::fopen(dump, "wb");
            auto wv = [&](const auto& v) {
                const uint64_t m = v.size();
                std::fwrite(&m, 8, 1, f);
                if (m) std::fwrite(v.data(), sizeof(v[0]), m, f);
            };
            const int64_t hdr[6] = {bc.G, bc.clock0, (int64_t)P.n_sched, (int64_t)P.partitioned,
                                    (int64_t)!e->app.playback, n};
            std::fwrite(hdr, 8, 6, f);
            wv(bc.clk); wv(bc.adv); wv(bc.nadv); wv(all); wv(q.key_hash); wv(seg_b); wv(seg_e);
            wv(std::vector<uint32_t>(gpos.begin(), gpos.begin() + n));
            std::fclose(f);
        }
        // optimistic pass: keys the scheduler reorders are rerun with its fire order (the device does this in one
        // launch), then the exact pass decides, replaying on the host only what still differs
        auto t0 = std::chrono::steady_clock::now();
        q.sim.simulate(bc, all, q.key_hash, kr, take, res, true);
        auto t1 = std::chrono::steady_clock::now();
        if (!res.reordered.empty()) {
            for (size_t d = 0; d < res.reordered.size(); ++d) {
                const uint32_t k = res.reordered[d];
                q.arenas[k] = backup[k];
                int rc = run_one(k, res.fires.data() + res.fire_off[d], (int)(res.fire_off[d + 1] - res.fire_off[d]));
                if (rc) return rc;
            }
            all.clear();
            for (auto& kv : klog) all.insert(all.end(), kv.second.begin(), kv.second.end());
        }
        reordered_ = res.reordered.size();
        auto t2 = std::chrono::steady_clock::now();
        if (getenv("SDG_SCHED_EXACT") || !q.sim.confirm(all, res)) {
            q.sim.simulate(bc, all, q.key_hash, kr, take, res);
            ++exact_passes_;
        }
        auto t3 = std::chrono::steady_clock::now();
        us_[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
        us_[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
        us_[2] += std::chrono::duration<double, std::micro>(t3 - t2).count();
        taken_ = res.taken.size();
        q.sim.commit();
        for (auto& r : runs) {  // the host runs replace those keys' device results
            if (r->overflow()) {
                g_err = "query '" + h.name + "': partial-match arena overflow (host run)";
                return 3;
            }
            q.arenas[r->key] = r->arena;
            std::vector<Out>& ko = kout[r->key];
            ko.clear();
            const int64_t cap = (int64_t)r->o_ts.size();
            for (unsigned long long i = 0; i < r->count; ++i) {
                Out o{r->o_seq[i], r->o_sub[i], r->o_ts[i], {}, r->o_nulls[i]};
                for (int j = 0; j < P.n_out; ++j) o.vals.push_back(r->o_vals[(size_t)j * cap + i]);
                ko.push_back(std::move(o));
            }
        }
    }
    std::vector<Out> batch;
    for (auto& kv : kout)
        for (Out& o : kv.second) {
            if (o.sub < 0) {  // timer match: its fire's place in the scheduler's order (position, rank)
                const int sch = (int)((o.sub >> 48) & 0x7F);
                const uint32_t g = (uint32_t)(o.seq - e->seq);
                const SchedSim::Slot* it = res.rank.find(SchedSim::rank_key(g, sch, kv.first));
                if (it) {
                    o.seq = e->seq + it->g;
                    o.sub = INT64_MIN | ((int64_t)it->rank << 24) | (o.sub & 0xFFFFFF);
                }
            }
            batch.push_back(std::move(o));
        }
    std::stable_sort(batch.begin(), batch.end(),
                     [](const Out& a, const Out& b) { return a.seq != b.seq ? a.seq < b.seq : a.sub < b.sub; });
    for (auto& o : batch) q.outs.push_back(std::move(o));
    return 0;
}

}  // namespace

extern "C" {

const char* emu_error() { return g_err.c_str(); }

void* emu_create(const char* text, int max_partials) {
    try {
        auto e = std::make_unique<Emu>();
        e->app = sql::parse_app(text);
        if (max_partials > 0) e->ns = max_partials;
        auto hqs = compile_app(e->app, e->strings);
        for (auto& h : hqs) {
            auto q = std::make_unique<EmuQuery>();
            q->hq = std::move(h);
            const Plan& P = q->hq.plan;
            if (P.has_post)  // the selector's post pass runs on the device only (order.hip select_post)
                throw std::runtime_error("selector post pass (aggregators / having) is device-only");
            for (int ka : q->hq.key_attr) {
                if (ka == -2) throw std::runtime_error("range partitions: the engine's batch assembly only");
                if (ka == -3) q->bcast = true;
            }
            if (P.purge) throw std::runtime_error("@purge: the engine's kernel arguments only");
            if (P.n_list_cols) throw std::runtime_error("multi-value selections: the engine's poll only");
            q->L = nfa::make_layout(P.n_states, std::max(P.n_cols, 1), e->ns, P.n_sched);
            q->sim.setup(P.n_sched, P.partitioned, !e->app.playback);
            e->qs.push_back(std::move(q));
        }
        return e.release();
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return nullptr;
    }
}

void emu_destroy(void* h) { delete (Emu*)h; }

int emu_stream_index(void* h, const char* sid) { return ((Emu*)h)->app.stream_index(sid); }

int emu_stream_nattrs(void* h, int s) { return (int)((Emu*)h)->app.streams[s].attrs.size(); }
int emu_stream_attr_type(void* h, int s, int a) { return (int)((Emu*)h)->app.streams[s].attrs[a].type; }

uint32_t emu_intern(void* h, const char* s) { return ((Emu*)h)->strings.get(s); }

const char* emu_string(void* h, uint32_t id) {
    Emu* e = (Emu*)h;
    return id < e->strings.strs.size() ? e->strings.strs[id].c_str() : "";
}

// one event: vals in stream attribute order (int/long as integers, float/double as raw IEEE bits, bool 0/1,
// string as interned id)
int emu_send(void* h, int stream, int64_t ts, const int64_t* vals, const uint8_t* nulls) {
    Emu* e = (Emu*)h;
    int na = (int)e->app.streams[stream].attrs.size();
    Ev ev{stream, ts, std::vector<int64_t>(vals, vals + na), std::vector<uint8_t>(nulls, nulls + na)};
    e->pending.push_back(std::move(ev));
    return 0;
}

// n events (stream[i], ts[i], the row's attribute slots at slots + offsets[i]) in order
int emu_send_batch(void* h, int64_t n, const int32_t* stream, const int64_t* ts, const int64_t* offsets,
                   const int64_t* slots, const uint8_t* nulls) {
    Emu* e = (Emu*)h;
    for (int64_t i = 0; i < n; ++i) {
        const int na = (int)e->app.streams[stream[i]].attrs.size();
        const int64_t* v = slots + offsets[i];
        Ev ev{stream[i], ts[i], std::vector<int64_t>(v, v + na), std::vector<uint8_t>(na, 0)};
        if (nulls) ev.nulls.assign(nulls + offsets[i], nulls + offsets[i] + na);
        e->pending.push_back(std::move(ev));
    }
    return 0;
}

// advance_time: a position of its own (playback: setCurrentTimestamp; live: the wall clock moved)
int emu_advance(void* h, int64_t ts) {
    Emu* e = (Emu*)h;
    e->pending.push_back(Ev{-1, ts, {}, {}});
    return 0;
}

// SiddhiAppRuntime.start: the live clock starts at ts (playback: the clock is event time, starting at 0)
int emu_start(void* h, int64_t ts) {
    Emu* e = (Emu*)h;
    if (!e->app.playback) e->clock = ts;
    return 0;
}

void emu_set_reclaim(int on) { g_reclaim = on; }
int64_t emu_idles() { return idles_; }

int emu_flush(void* h) {
    Emu* e = (Emu*)h;
    try {
        BatchClock bc = batch_clock(e);
        for (auto& q : e->qs) {
            int rc = flush_query(e, *q, bc);
            if (rc) {
                e->pending.clear();
                return rc;
            }
        }
        if (bc.G > 0) e->clock = bc.clk[bc.G - 1];
        e->seq += bc.G;
    } catch (const std::exception& ex) {
        g_err = ex.what();
        e->pending.clear();
        return 5;
    }
    e->pending.clear();
    return 0;
}

int64_t emu_sched_stat(int which) {
    return which == 0 ? (int64_t)reordered_ : which == 1 ? (int64_t)taken_ : which == 5 ? growths_
         : which == 6 ? (int64_t)exact_passes_ : which == 7 ? spills_ : (int64_t)us_[which - 2];
}
int emu_num_queries(void* h) { return (int)((Emu*)h)->qs.size(); }
const char* emu_query_name(void* h, int q) { return ((Emu*)h)->qs[q]->hq.name.c_str(); }
const char* emu_query_target(void* h, int q) { return ((Emu*)h)->qs[q]->hq.target.c_str(); }
int emu_query_nout(void* h, int q) { return (int)((Emu*)h)->qs[q]->hq.out_types.size(); }
int emu_query_out_type(void* h, int q, int j) { return ((Emu*)h)->qs[q]->hq.out_types[j]; }
int emu_query_chain(void* h, int q) { return ((Emu*)h)->qs[q]->hq.plan.chain; }
int64_t emu_num_out(void* h, int q) { return (int64_t)((Emu*)h)->qs[q]->outs.size(); }
void emu_out(void* h, int q, int64_t i, int64_t* ts, int64_t* vals, uint32_t* nulls, int64_t* seq) {
    const Out& o = ((Emu*)h)->qs[q]->outs[i];
    *ts = o.ts;
    if (seq) { seq[0] = o.seq; seq[1] = o.sub; }
    for (size_t j = 0; j < o.vals.size(); ++j) vals[j] = o.vals[j];
    *nulls = o.nulls;
}

}  // extern "C"

// ---- test-only sampling profiler for the host harness (SIGPROF, program counters of the sampled thread) ----
#include <dlfcn.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>
namespace {
std::vector<uintptr_t> g_samples(1 << 22);
volatile size_t g_nsamp = 0;
void on_prof(int, siginfo_t*, void* uc) {
    const size_t i = g_nsamp;
    if (i < g_samples.size()) {
        g_samples[i] = (uintptr_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
        g_nsamp = i + 1;
    }
}
}  // namespace
extern "C" {
void emu_prof_start() {
    struct sigaction sa;
    std::memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, nullptr);
    g_nsamp = 0;
    itimerval tv{{0, 200}, {0, 200}};
    setitimer(ITIMER_PROF, &tv, nullptr);
}
// writes "object offset" per sample (objects: this library's path or the hex address)
void emu_prof_stop(const char* path) {
    itimerval tv{{0, 0}, {0, 0}};
    setitimer(ITIMER_PROF, &tv, nullptr);
    FILE* f = std::fopen(path, "w");
    for (size_t i = 0; i < g_nsamp; ++i) {
        Dl_info di;
        if (dladdr((void*)g_samples[i], &di) && di.dli_fname)
            std::fprintf(f, "%s 0x%lx\n", di.dli_fname, (unsigned long)(g_samples[i] - (uintptr_t)di.dli_fbase));
        else
            std::fprintf(f, "? 0x%lx\n", (unsigned long)g_samples[i]);
    }
    std::fclose(f);
}
}
