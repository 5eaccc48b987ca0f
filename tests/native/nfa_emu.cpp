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
#include "../../siddhi_amd/csrc/engine/nfa.h"
#include "../../siddhi_amd/csrc/siddhiql/parser.h"

using namespace sdg;

namespace {

std::string g_err;

int width_of(uint8_t kind) {
    switch (kind) {
        case VK_I64: case VK_F64: return 8;
        case VK_BOOL: return 1;
        default: return 4;
    }
}

struct Ev {
    int stream;
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
    std::vector<std::vector<uint8_t>> arenas;
    int64_t seq = 0;
    std::vector<Out> outs;
};

struct Emu {
    sql::App app;
    Interner strings;
    std::vector<std::unique_ptr<EmuQuery>> qs;
    std::vector<Ev> pending;
    int ns = 64;
};

std::string key_text(Emu* e, uint8_t kind, int64_t v) {
    char buf[64];
    switch (kind) {
        case VK_I32: return std::to_string((int32_t)v);
        case VK_I64: return std::to_string(v);
        case VK_F32: std::snprintf(buf, sizeof buf, "%.9g", (double)bits_f32(v)); return buf;
        case VK_F64: std::snprintf(buf, sizeof buf, "%.17g", bits_f64(v)); return buf;
        case VK_BOOL: return v ? "true" : "false";
        default: return e->strings.strs[(uint32_t)v];
    }
}

int flush_query(Emu* e, EmuQuery& q) {
    HostQuery& h = q.hq;
    const Plan& P = h.plan;
    const int nc = P.n_cols;
    std::vector<const Ev*> rows;
    std::vector<int> rkey;
    for (const Ev& ev : e->pending) {
        int qpos = h.stream_pos(ev.stream);
        if (qpos < 0) continue;
        int key = 0;
        if (P.partitioned) {
            int ai = h.key_attr[qpos];
            if (ev.nulls[ai]) continue;  // null partition key: dropped
            std::string kt = key_text(e, h.key_kind[qpos], ev.vals[ai]);
            auto it = q.keys.find(kt);
            if (it == q.keys.end()) it = q.keys.emplace(kt, (int)q.keys.size()).first;
            key = it->second;
        }
        rows.push_back(&ev);
        rkey.push_back(key);
    }
    const int64_t n = (int64_t)rows.size();
    const int K = P.partitioned ? (int)q.keys.size() : 1;
    // stable grouping by key
    std::vector<uint32_t> order(n);
    for (int64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return rkey[a] < rkey[b]; });
    std::vector<int64_t> ts(std::max<int64_t>(n, 1));
    std::vector<uint8_t> qs(std::max<int64_t>(n, 1));
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
    int64_t cap = 2 * n + 4096;
    std::vector<int64_t> o_ts(cap), o_vals((size_t)std::max(P.n_out, 1) * cap), o_seq(cap), o_sub(cap);
    std::vector<uint32_t> o_nulls(cap), o_key(cap);
    unsigned long long count = 0;
    int flags[4] = {0, 0, 0, 0};
    std::vector<int64_t> stk(STACK);
    for (int k = 0; k < K; ++k) {
        if (seg_b[k] >= seg_e[k]) continue;
        nfa::Ctx c;
        c.P = &P;
        c.code = h.code.data();
        c.consts = h.consts.data();
        c.L = q.L;
        c.base = q.arenas[k].data();
        c.stk = stk.data();
        c.stride = 1;
        c.emit_ts = o_ts.data();
        c.emit_vals = o_vals.data();
        c.emit_nulls = o_nulls.data();
        c.emit_seq = o_seq.data();
        c.emit_sub = o_sub.data();
        c.emit_key = o_key.data();
        c.emit_count = &count;
        c.emit_cap = cap;
        c.flags = flags;
        c.key = (uint32_t)k;
        nfa::KeyEvents kev{ts.data(), qs.data(), order.data(), cptr.data(), nptr.data(), seg_b[k], seg_e[k], q.seq};
        nfa::run_key(c, kev);
        if (c.ovf()) {
            g_err = "query '" + h.name + "': partial-match arena overflow";
            return 3;
        }
    }
    if (flags[0]) {
        g_err = "output overflow";
        return 3;
    }
    std::vector<Out> batch;
    for (unsigned long long i = 0; i < count; ++i) {
        Out o{o_seq[i], o_sub[i], o_ts[i], {}, o_nulls[i]};
        for (int j = 0; j < P.n_out; ++j) o.vals.push_back(o_vals[(size_t)j * cap + i]);
        batch.push_back(std::move(o));
    }
    std::stable_sort(batch.begin(), batch.end(),
                     [](const Out& a, const Out& b) { return a.seq != b.seq ? a.seq < b.seq : a.sub < b.sub; });
    for (auto& o : batch) q.outs.push_back(std::move(o));
    q.seq += n;
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
            for (int i = 0; i < h.plan.n_states; ++i)
                if (h.plan.st[i].kind == PK_ABSENT) throw CompileError(4, "absent states not in this build");
            auto q = std::make_unique<EmuQuery>();
            q->hq = std::move(h);
            q->L = nfa::make_layout(q->hq.plan.n_states, std::max(q->hq.plan.n_cols, 1), e->ns);
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

int emu_flush(void* h) {
    Emu* e = (Emu*)h;
    try {
        for (auto& q : e->qs) {
            int rc = flush_query(e, *q);
            if (rc) return rc;
        }
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return 5;
    }
    e->pending.clear();
    return 0;
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
