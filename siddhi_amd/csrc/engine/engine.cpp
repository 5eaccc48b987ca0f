// Engine runtime behind include/siddhi_amd.h: ingestion buffers, device residency, flush orchestration,
// output delivery. One engine == one HIP device + one stream; calls on a handle are serialised by the caller
// (the reference serialises a query under patternSyncObject, MultiProcessStreamReceiver.java:97).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/siddhi_amd.h"
#include "../kernels/kernels.h"
#include "../siddhiql/parser.h"
#include "compile.h"
#include "keyorder.h"
#include "keyrun.h"
#include "hostpar.h"
#include "sched.h"

namespace sdg {
namespace {

thread_local std::string g_err;

struct DeviceError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIPCHECK(x)                                                                                   \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) throw DeviceError(std::string(#x) + ": " + hipGetErrorString(e_));       \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
        return *this;
    }
    ~DevBuf() { if (p) (void)hipFree(p); }
    // `need` bytes, reallocating (with a quarter of slack) only when they do not fit: a slightly larger flush than the
    // last must not reallocate GBs (an ensure(need + need / 4) would, whenever need grows at all)
    void* ensure_slack(size_t need) { return need > cap ? ensure(need + need / 4) : p; }
    void* ensure(size_t bytes) {
        if (bytes == 0) bytes = 8;
        if (bytes > cap) {
            if (p) HIPCHECK(hipFree(p));
            p = nullptr;
            size_t c = std::max(bytes, cap + cap / 2);
            HIPCHECK(hipMalloc(&p, c));
            cap = c;
        }
        return p;
    }
    template <class T>
    T* as() const { return (T*)p; }
};

// pinned host staging for the per-flush kernel arguments and read-backs: hipMemcpyAsync from pageable memory
// goes through a bounce buffer on the host thread (tens of us per copy on the flush's critical path)
struct HostPin {
    void* p = nullptr;
    size_t cap = 0;
    HostPin() = default;
    HostPin(const HostPin&) = delete;
    HostPin& operator=(const HostPin&) = delete;
    ~HostPin() { if (p) (void)hipHostFree(p); }
    void* ensure_slack(size_t need) { return need > cap ? ensure(need + need / 8) : p; }  // (as DevBuf::ensure_slack)
    void* ensure(size_t bytes) {
        if (bytes > cap) {
            if (p) HIPCHECK(hipHostFree(p));
            p = nullptr;
            HIPCHECK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
            cap = bytes;
        }
        return p;
    }
};

enum KeyClass { KC_NONE = 0, KC_INT = 1, KC_F32 = 2, KC_F64 = 3, KC_BOOL = 4 };
int key_class_of(uint8_t kind) {
    switch (kind) {
        case VK_I32: case VK_I64: return KC_INT;
        case VK_F32: return KC_F32;
        case VK_F64: return KC_F64;
        case VK_BOOL: return KC_BOOL;
        default: return KC_NONE;
    }
}
// the device key table's 64-bit value of a key (keytab.hip kt_value) <-> the key's toString (the dictionary text)
int64_t key_value_of_string(int kc, const std::string& s) {
    switch (kc) {
        case KC_F64: {
            const double d = std::strtod(s.c_str(), nullptr);  // Java's toString: "NaN", "Infinity", "1.0E10" parse
            int64_t b;
            std::memcpy(&b, &d, 8);
            return std::isnan(d) ? 0x7FF8000000000000ll : b;
        }
        case KC_F32: {
            const float f = std::strtof(s.c_str(), nullptr);
            uint32_t b;
            std::memcpy(&b, &f, 4);
            return std::isnan(f) ? 0x7FC00000ll : (int64_t)b;
        }
        case KC_BOOL: return s == "true" ? 1 : 0;
        default: return std::stoll(s);
    }
}
std::string key_string_of_value(int kc, int64_t v) {
    switch (kc) {
        case KC_F64: return java_real_string(bits_f64(v), false);
        case KC_F32: return java_real_string(bits_f32(v), true);
        case KC_BOOL: return v ? "true" : "false";
        default: return std::to_string(v);
    }
}

int width_of(uint8_t kind) {
    switch (kind) {
        case VK_I64: case VK_F64: return 8;
        case VK_BOOL: return 1;
        default: return 4;
    }
}

struct PushChunk {
    int stream;          // -1: an sdg_advance_time point (one position, no data); -2: mixed (rstream per row)
    int64_t n;
    bool device;
    bool no_adv = false; // rows of an InputHandler.send(Event[]): they do not move the playback clock
    std::vector<int32_t> rstream;   // mixed: stream of each row; cols[a] then hold 64-bit slots of attribute a
    std::vector<int64_t> ts;
    std::vector<std::vector<uint8_t>> cols;
    std::vector<std::vector<uint8_t>> nulls;
    const int64_t* d_ts = nullptr;
    std::vector<const void*> d_cols;
    std::vector<const uint8_t*> d_nulls;
    // a host push staged in HBM at push time (device == true): its rows are [stage_off, stage_off + n) of the
    // engine's staging columns of its stream; d_ts / d_cols / d_nulls are resolved when the flush starts
    int64_t stage_off = -1;
    // a mixed chunk's raw rows in HBM (uploaded at the first flush that builds a query view from them on the device)
    bool m_up = false;
    DevBuf m_streams, m_ts, m_slots, m_nulls;
    std::vector<char> m_has_null;
};

// the device staging of one stream's host pushes (sdg_push / sdg_push_events): columns appended in push order, so
// a query of that stream sees every staged push of a batch as one contiguous device range (zero-copy flush path)
struct Stage {
    DevBuf ts;
    std::vector<DevBuf> cols, nulls;
    std::vector<char> has_nulls;
    int64_t n = 0, cap = 0;
};

// integral partition values -> dictionary id (open addressing). Java's toString is injective on int/long and
// equal values of either type print the same, so the value itself can stand for its string in front of keydict.
struct IntKeyCache {
    std::vector<int64_t> k;
    std::vector<uint32_t> v;  // id + 1 (0 = empty slot)
    size_t n = 0;
    static uint64_t mix(uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    // batch loops prefetch the slot of the key a few rows ahead: the lookups are cache misses over a table of
    // up to millions of keys, so one at a time they are latency-bound (C4's 2 x 10^7 rows: 1.3 s)
    void prefetch(int64_t x) const {
        if (k.empty()) return;
        const size_t i = mix((uint64_t)x) & (k.size() - 1);
        __builtin_prefetch(&k[i]);
        __builtin_prefetch(&v[i]);
    }
    bool find(int64_t x, uint32_t* id) const {
        if (k.empty()) return false;
        const size_t m = k.size() - 1;
        for (size_t i = mix((uint64_t)x) & m;; i = (i + 1) & m) {
            if (!v[i]) return false;
            if (k[i] == x) { *id = v[i] - 1; return true; }
        }
    }
    void insert(int64_t x, uint32_t id) {
        if (2 * (n + 1) > k.size()) {
            std::vector<int64_t> ok;
            std::vector<uint32_t> ov;
            ok.swap(k);
            ov.swap(v);
            const size_t cap = std::max<size_t>(1024, ok.size() * 2);
            k.assign(cap, 0);
            v.assign(cap, 0);
            n = 0;
            for (size_t i = 0; i < ok.size(); ++i)
                if (ov[i]) insert(ok[i], ov[i] - 1);
        }
        const size_t m = k.size() - 1;
        size_t i = mix((uint64_t)x) & m;
        while (v[i]) i = (i + 1) & m;
        k[i] = x;
        v[i] = id + 1;
        ++n;
    }
};

struct QueryRt {
    HostQuery hq;
    IntKeyCache intkeys;
    DevBuf d_plan, d_code, d_consts, d_args, o_mq, o_ovf, o_ovfc, o_dqs, d_sub_args;
    HostPin h_args, h_ret;  // chain path: ChainArgs pair; counters (16 B) | flags (16 B) | overflow count (8 B)
    HostPin h_sub_args;     // fused sub-batches: the two ChainArgs (sub_dead 1 / 0)
    bool string_keys = true;                        // all partition keys are string attributes (ids used as keys)
    // device key table (device-resident batches): the class every partition key attribute of the query shares --
    // KC_INT (int / long), KC_F32, KC_F64, KC_BOOL -- or KC_NONE (string keys, mixed classes, range partitions)
    int key_class = 0;
    // device key table (keytab.hip) for device-resident batches of int / long keys: a mirror of keydict's ids
    DevBuf kt_keys, kt_cnt, kt_pairs, kt_vals, kt_slots;  // kt_keys: the table's KtSlot array
    uint64_t kt_cap = 0;
    size_t kt_synced = 0;                           // keydict ids [0, kt_synced) are in the table
    HostPin kt_ret;
    std::unordered_map<std::string, uint32_t> keydict;  // (not kept for KC_INT queries: intkeys maps their values)
    std::vector<std::string> keystr;                // key id -> key text (numeric keys)
    // a stream of the query without a partition key (key_attr -3): its events go to every key the partition has
    // initialised, in getPartitionKeys() order (keyorder.h); host batch assembly only
    bool broadcast = false;
    PartitionKeyOrder korder;
    bool ranked = false;  // range partitions or broadcast rows: delivery ranks in bits 40..62 of `sub`
    int sub_bits() const { return ranked ? 64 : 48; }
    // absent states: the scheduler simulation, per-key HashMap hashes, double-buffered arenas, the run's log
    SchedSim sim;
    std::vector<int32_t> key_hash;
    DevBuf arena2, cur_bits, ran_bits, o_round, d_log, d_list, d_foff, d_fires, d_vpos;
    int64_t log_cap = 0;
    // timer-match ordering of the last flush (drain): each fire's slot in the scheduler's order; the keys the
    // scheduler replayed on the host (their device records are void) and those replays
    bool last_timers = false;
    int64_t last_seq_base = 0;
    // delivery order on the device (order.hip): the flush's first position, and whether `sub` holds the e1 event's
    // position (chain path) or an ordinal within the emitting event (generic NFA)
    int64_t emit_base = 0;
    int64_t emit_span = 0;  // positions of that flush (emit - emit_base < emit_span)
    bool sub_is_seq = false;
    DevBuf ord_ws, g_ts, g_emit, g_vals, g_nulls, g_key, gather_ws;
    // the selector's post pass (aggregators / having): per-key aggregator state, persistent; staging
    DevBuf agg_state, ps_key, ps_vals, ps_nulls, ps_pass, ps_ws;
    int64_t agg_keys = 0;
    // @purge: per-key clock reading at the key's last event (stored XOR INT64_MIN: zero bytes = never seen), its
    // copy at the batch start (a rerun starts from it), the partition's first initPartition reading
    DevBuf last_seen, last_seen_bak;
    // @purge with aggregators: per record "purged since the key's previous record" (aggregator states restart), per
    // key "purged after its last record" (applied after the post pass)
    DevBuf o_flags, g_flags, ps_reset, agg_reset_flags;
    bool purge_agg = false;
    int64_t purge_first = INT64_MIN;
    SchedSim::RankMap last_rank;
    std::vector<uint32_t> reordered;  // keys rerun with the scheduler's fire order (sorted)
    std::vector<uint32_t> taken;
    std::vector<std::unique_ptr<KeyRun>> runs;
    // batch staging
    DevBuf st_ts, st_qs, st_key, st_vrank, st_cols[MAX_COLS], st_nulls[MAX_COLS];
    // broadcast rows expanded on the device (bcast_expand): the expanded view and the expansion's tables
    DevBuf bx_ts, bx_vpos, bx_qs, bx_key, bx_vrank, bx_cols[MAX_COLS], bx_nulls[MAX_COLS], bx_off, bx_ph, bx_ord;
    DevBuf mv_work, mv_tot, mv_args, kt_vals_in;  // device-side views of mixed pushes
    // sorted view
    DevBuf so_ts, so_qs, so_key, so_orig, so_vrank, so_cols[MAX_COLS], so_nulls[MAX_COLS], seg, kg_counts, kg_gsum;
    DevBuf so_lkey;                                 // fused path: u8 local keys of the bucket view
    DevBuf sv_tsbase;                               // sorted view: base of its u32 ts offsets (ts_window_base)
    DevBuf bk_plan;                                 // fused path: bstart[257] + bseg[257]
    DevBuf bk_tm;                                   // fused path: time-major block plan (ChainArgs::tm)
    DevBuf bk_own;                                  // fused sub-batches: bown[257] (ChainArgs::bown)
    bool no_sub = false;                            // fused sub-batches off for good (a halo check failed)
    std::vector<hipEvent_t> sub_ev;                 // per sub-batch timing marks (4 each)
    // carries (double buffered)
    struct Carry {
        DevBuf key, ts, seq, vals, nulls;
        int64_t n = 0, cap = 0;
    } carry[2];
    int cur = 0;
    // a chain query that met decreasing per-key timestamps runs on the generic NFA from then on; its carried
    // partials are replayed into the arenas first (replay_carries)
    bool replay_carries = false;
    DevBuf rp_ts, rp_qs, rp_seg, rp_segend, rp_cols[MAX_COLS], rp_nulls[MAX_COLS];
    // generic NFA: per-key partial-match arenas (persist across batches)
    DevBuf arena;
    int64_t arena_keys = 0;                         // arenas allocated (per key; reclaiming queries: per slot)
    // reclaiming queries (nfa.h to_idle): keys whose state the reference destroys down to the start processors' seeds
    // give their arena slot back and keep an idle record; arenas are sized by live keys, not by keys ever seen
    bool reclaim = false;
    int64_t map_keys = 0;                           // keys covered by slot_of / idle_rec
    DevBuf slot_of, idle_rec, slot_key, init_from, releasable, idle_out, free_slots, pool_ctr;
    HostPin pool_ret;
    nfa::Layout L{};
    // spilled keys: a partition key that outgrows the device arena's largest layout (4096 partial matches) goes on
    // on the host from its batch-start state, in an arena of 32-bit indices that doubles whenever the key needs
    // more (KeyRunT<int32_t>); the device skips it from then on (KH_HOST in its arena head, or slot_of -3 for
    // reclaiming queries). Its records of the flush that overflowed are dropped (q.taken) for the host run's.
    struct Spilled {
        nfa::Layout L{};
        std::vector<uint8_t> arena;
        int64_t purge_last = INT64_MIN;  // @purge: the key's last activity reading (PurgeIn::last)
    };
    std::map<uint32_t, Spilled> spill;
    std::vector<std::unique_ptr<KeyRunT<int32_t>>> spill_runs;  // the last flush's host runs of spilled keys
    DevBuf d_ovf;                                               // overflowed keys: [0] count, [1..] keys
    // the register sequence kernel (seq3.hip) instead of the generic NFA: its per-key state, SoA with stride s3_kcap
    bool seq3 = false;
    Seq3Spec s3{};
    DevBuf s3_hdr, s3_pn, s3_qn, s3_vals, s3_ts;
    int64_t s3_kcap = 0;
    // outputs
    DevBuf o_ts, o_key, o_vals, o_nulls, o_emit, o_first, counters, flags;
    int64_t out_n = 0, out_cap = 0;
    bool polled = true;
    bool nulls_valid = true;                        // false: the last flush wrote no null bits (none possible)
    bool carry_nullable = false;                    // the carried partials came from a batch with null columns
    // delivered rows not yet polled, in delivery order (drain(): an auto-flush inside sdg_push, or several
    // sdg_flush calls before one sdg_poll, keep appending here -- never overwritten)
    // (acc_* and h_* swap at each poll, so their columns keep their capacity from poll to poll)
    HostVec<int64_t> acc_ts, acc_seq;
    std::vector<HostVec<int64_t>> acc_vals;
    std::vector<HostVec<uint8_t>> acc_nulls;
    HostPin h_rb;                                   // pinned read-back staging
    // pinned delivery (round 6): a flush whose records come out of the device already in delivery order, drained
    // into an empty backlog, is read back straight into one of two pinned buffers that sdg_poll then hands out (no
    // host copy into acc_*; the two alternate so the previous poll's arrays stay valid until the next poll)
    HostPin del_buf[2];
    int del_cur = 0;                                // the buffer the last sdg_poll handed out
    int64_t del_n = -1;                             // >= 0: the backlog is these records in del_buf[del_cur ^ 1]
    int del_nu = 0;                                 // their user-visible columns
    bool del_nulls = false;                         // their null bytes are in the buffer (else the zero page)
    std::vector<uint8_t> del_zero[2];               // zeros per buffer: expired flags / null bytes of null-free records
    // host copies for sdg_poll
    HostVec<int64_t> h_ts, h_seq;
    HostVec<uint8_t> h_expired;
    std::vector<HostVec<int64_t>> h_vals;
    std::vector<HostVec<uint8_t>> h_nulls;
    std::vector<const int64_t*> h_vptr;
    std::vector<const uint8_t*> h_nptr;
};

}  // namespace
}  // namespace sdg

using namespace sdg;

struct sdg_engine {
    sql::App app;
    Interner strings;
    std::vector<std::unique_ptr<QueryRt>> qs;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;   // the fused path's carry-in pass runs here, beside the matcher
    hipEvent_t ev[12] = {};
    hipEvent_t fork = nullptr, join = nullptr;
    std::vector<PushChunk> pending;
    int64_t capacity = 1 << 24;
    int32_t max_partials = 8;  // starting slots per key (arenas double on overflow): small arenas stage in LDS
    int64_t pending_n = 0;
    int64_t seq = 0;             // batch positions flushed so far (sequence number of the next batch's position 0)
    int64_t flush_G = 0;         // positions of the flush being run (its records' emitting events are < seq + flush_G)
    int64_t clock = 0;           // currentTime(): playback = max event ts seen; live = the modelled wall clock
    bool any_sched = false;      // some query has absent states (the batch clock is built)
    bool any_purge = false;      // some query's partition purges idle keys (the batch clock is built)
    BatchClock bc;
    DevBuf d_clk, d_nadv;
    sdg_stats stats{};
    std::vector<std::vector<int32_t>> stream_types;
    std::vector<std::vector<int32_t>> out_types;
    std::vector<std::vector<const char*>> out_names;
    bool compile_only = false;
    bool force_generic = false;
    bool no_fused = false;
    bool no_seq3 = false;        // SDG_NO_SEQ3 / SDG_FORCE_GENERIC: seq3-shaped sequences on the generic NFA
    bool sched_exact = false;    // SDG_SCHED_EXACT (flag or env): the scheduler's exact pass always runs
    bool sched_host = false;     // SDG_SCHED_HOST: exact pass over the first run, diverged keys replayed on the host
    bool no_sorted = false;      // SDG_NO_SORTED: the radix chain path keeps the lane deque kernels
    uint64_t app_hash = 0;       // FNV-1a of the app text: a snapshot restores only into the app it came from
    std::vector<uint8_t> snap;   // the last sdg_snapshot's bytes (valid until the next snapshot / destroy)
    std::string states_json;     // the last sdg_snapshot_states text
    std::vector<Stage> stage;    // per stream: host pushes staged in HBM (see stage_push)
    std::vector<char> stage_ok;  // per stream: every query of the stream takes device-resident batches
    std::vector<char> host_pending;  // per stream: the pending batch holds host rows of it (no staging until flush)
    bool no_stage = false;       // mixed pushes seen: host assembly for every stream from then on
    HostPin bounce[2];           // pinned chunks of the pageable host -> HBM copies (h2d)
    hipEvent_t bounce_ev[2] = {};
};

namespace {

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

void upload_plan(sdg_engine* e, QueryRt& q) {
    HostQuery& h = q.hq;
    void* dp = q.d_plan.ensure(sizeof(Plan));
    HIPCHECK(hipMemcpyAsync(dp, &h.plan, sizeof(Plan), hipMemcpyHostToDevice, e->stream));
    if (!h.code.empty()) {
        void* dc = q.d_code.ensure(h.code.size() * sizeof(Instr));
        HIPCHECK(hipMemcpyAsync(dc, h.code.data(), h.code.size() * sizeof(Instr), hipMemcpyHostToDevice, e->stream));
    } else {
        q.d_code.ensure(sizeof(Instr));
    }
    if (!h.consts.empty()) {
        void* dk = q.d_consts.ensure(h.consts.size() * 8);
        HIPCHECK(hipMemcpyAsync(dk, h.consts.data(), h.consts.size() * 8, hipMemcpyHostToDevice, e->stream));
    } else {
        q.d_consts.ensure(8);
    }
    HIPCHECK(hipStreamSynchronize(e->stream));
}

// a new key of an int / long keyed query (KC_INT): the next id, its text for snapshots and scheduler hashes; the
// value cache is the dictionary (no string map: a million new keys cost ~0.2 s of string-map inserts, C4 r5h)
bool new_int_key(QueryRt& q, int64_t iv, uint32_t* key) {
    *key = (uint32_t)q.keystr.size();
    q.keystr.push_back(std::to_string(iv));
    q.intkeys.insert(iv, *key);
    return true;
}


// key of one host row (ValuePartitionExecutor: toString, null -> dropped)
bool host_key(sdg_engine* e, QueryRt& q, int qpos, const PushChunk& c, int64_t row, uint32_t* key) {
    int ai = q.hq.key_attr[qpos];
    if (!c.nulls[ai].empty() && c.nulls[ai][row]) return false;
    const uint8_t* col = c.cols[ai].data();
    uint8_t kind = q.hq.key_kind[qpos];
    if (q.string_keys) {
        *key = ((const uint32_t*)col)[row];
        return true;
    }
    int64_t iv = 0;
    const bool integral = kind == VK_I32 || kind == VK_I64;
    if (integral) {
        iv = kind == VK_I32 ? (int64_t)((const int32_t*)col)[row] : ((const int64_t*)col)[row];
        if (q.intkeys.find(iv, key)) return true;
        if (q.key_class == KC_INT) return new_int_key(q, iv, key);
    }
    std::string s;
    switch (kind) {
        case VK_I32: s = std::to_string(((const int32_t*)col)[row]); break;
        case VK_I64: s = std::to_string(((const int64_t*)col)[row]); break;
        case VK_F32: s = java_real_string(((const float*)col)[row], true); break;
        case VK_F64: s = java_real_string(((const double*)col)[row], false); break;
        case VK_BOOL: s = col[row] ? "true" : "false"; break;
        default: s = e->strings.strs[((const uint32_t*)col)[row]]; break;
    }
    auto it = q.keydict.find(s);
    if (it == q.keydict.end()) {
        it = q.keydict.emplace(s, (uint32_t)q.keydict.size()).first;
        q.keystr.push_back(s);
    }
    *key = it->second;
    if (integral) q.intkeys.insert(iv, *key);
    return true;
}

// key of a mixed-chunk row from its 64-bit attribute slot (same toString rules as host_key)
bool slot_key(sdg_engine* e, QueryRt& q, int qpos, int64_t slot, uint32_t* key) {
    const uint8_t kind = q.hq.key_kind[qpos];
    if (q.string_keys) {
        *key = (uint32_t)slot;
        return true;
    }
    const bool integral = kind == VK_I32 || kind == VK_I64;
    const int64_t iv = kind == VK_I32 ? (int64_t)(int32_t)slot : slot;
    if (integral && q.intkeys.find(iv, key)) return true;
    if (integral && q.key_class == KC_INT) return new_int_key(q, iv, key);
    std::string s;
    switch (kind) {
        case VK_I32: case VK_I64: s = std::to_string(iv); break;
        case VK_F32: s = java_real_string(bits_f32(slot), true); break;
        case VK_F64: s = java_real_string(bits_f64(slot), false); break;
        case VK_BOOL: s = slot ? "true" : "false"; break;
        default: s = e->strings.strs[(uint32_t)slot]; break;
    }
    auto it = q.keydict.find(s);
    if (it == q.keydict.end()) {
        it = q.keydict.emplace(s, (uint32_t)q.keydict.size()).first;
        q.keystr.push_back(s);
    }
    *key = it->second;
    if (integral) q.intkeys.insert(iv, *key);
    return true;
}

// RangePartitionExecutor.execute (core/partition/executor/RangePartitionExecutor.java): the range condition over
// one pushed row (the same bytecode interpreter as the device, eval.h, on the row's attributes). Keys are computed
// on the host for host pushes, like the value partitions' toString keys.
struct RowAcc {
    const HostQuery* h;
    int qpos;
    const PushChunk* c;
    int64_t r;
    bool mixed;  // attribute a of row r is the 64-bit slot cols[a][r]
    void load(int, int col, int, uint8_t kind, int64_t* v, bool* null) {
        const int ai = h->col_attr[qpos][col];
        *v = 0;
        *null = true;
        if (ai < 0) return;
        *null = !c->nulls[ai].empty() && c->nulls[ai][r];
        if (mixed) *v = ((const int64_t*)c->cols[ai].data())[r];
        else *v = load_col(c->cols[ai].data(), kind, r);
    }
    bool slot_empty(int, int) { return false; }
    void agg(int, int64_t* v, bool* n) { *v = 0; *n = true; }
};
int64_t range_stack[STACK];
bool range_holds(const HostQuery& h, const HostQuery::RangeKey& rk, int qpos, const PushChunk& c, int64_t r, bool mixed) {
    RowAcc acc{&h, qpos, &c, r, mixed};
    return pass(h.code.data(), rk.cond, h.consts.data(), acc, range_stack, 1);
}

// The register sequence kernel (seq3.hip) covers SEQUENCE `every e1=S[f1], e2=S[f2]<m:n>, e3=S[f3]` over one stream
// (StateInputStreamParser.java:76-408 wiring: e1 the every-start re-armed by its own post processor, e2 a count
// state with min >= 1 forwarding to e3, e3 the last), without timers, @purge, aggregators, range partitions or
// streams without a partition key, with FastPred filters and plain-attribute selects whose state events are e1,
// e2[0], e2[last] or e3. `within` is covered: a partial expires as StreamPreStateProcessor.isExpired decides it
// (|e1.ts - now| > within, :118-129), checked before each event, as the generic NFA does.
// Fills the spec (operands resolved per processor context) or returns false (the generic NFA runs the query).
bool seq3_spec_(const HostQuery& h, Seq3Spec& s, int& why);
bool seq3_spec(const HostQuery& h, Seq3Spec& s) {
    int why = 0;
    const bool ok = seq3_spec_(h, s, why);
    if (!ok && getenv("SDG_SEQ3_WHY")) fprintf(stderr, "seq3: query '%s' not eligible (check %d)\n", h.name.c_str(), why);
    return ok;
}
bool seq3_spec_(const HostQuery& h, Seq3Spec& s, int& why) {
    const Plan& P = h.plan;
    if (P.chain || !P.seq || P.n_states != 3 || P.n_sched || P.purge || P.has_post) return why = 1, false;
    if (h.streams.size() != 1 || P.n_cols < 1 || P.n_cols > S3_MAX_COLS || P.n_out > S3_MAX_OUT) return why = 2, false;
    for (int x : h.key_attr)
        if (x == -2 || x == -3) return why = 3, false;  // range partitions, broadcast streams
    const StateRow &r0 = P.st[0], &r1 = P.st[1], &r2 = P.st[2];
    if (r0.kind != PK_STREAM || !r0.is_start || r0.next != 1 || r0.next_every != 0 || (r0.within_every != -1 && r0.within_every != 0) ||
        r0.callback != -1)
        return why = 4, false;
    if (r1.kind != PK_COUNT || r1.is_start || r1.next != 2 || r1.next_every != -1 || r1.callback != -1 ||
        r1.min_count < 1 || r1.min_count > (1 << 23) || (r1.max_count != INT32_MAX && r1.max_count > (1 << 23)) ||
        r1.max_count < r1.min_count)
        return why = 5, false;
    if (r2.kind != PK_STREAM || r2.is_start || r2.next != -1 || r2.next_every != -1 || r2.callback != -1) return why = 6, false;
    if (r0.stream != r1.stream || r1.stream != r2.stream) return why = 7, false;
    const RecvRow& rv = P.recv[0];
    if (rv.n != 3 || !rv.multi || rv.procs[rv.order[0]] != 2 || rv.procs[rv.order[1]] != 1 || rv.procs[rv.order[2]] != 0)
        return why = 8, false;
    for (int j = 0; j < P.n_out; ++j)
        if (P.out_multi[j] || P.out_post[j]) return why = 9, false;
    std::memset(&s, 0, sizeof s);
    s.nc = P.n_cols;
    s.n_out = P.n_out;
    s.min_count = r1.min_count;
    s.max_count = r1.max_count;
    s.has_within = P.has_within;
    s.within_ms = P.within_ms;
    for (int c = 0; c < P.n_cols; ++c) s.col_kind[c] = P.col_kind[c];
    // (slot, chain index) of a state event -> the register event of processor context `ctx`
    // (0: the e1 filter, the event is e1; 1: the e2 filter, Q with the event as e2[last]; 2: the e3 filter / select)
    auto src = [](int ctx, int slot, int chain, int8_t* out) -> bool {
        if (chain != 0 && chain != -1) return false;
        if (ctx == 0) *out = slot == 0 ? S3_Y : S3_NULL;
        else if (ctx == 1) *out = slot == 0 ? S3_E1 : slot == 1 ? (chain == 0 ? S3_E2F : S3_Y) : S3_NULL;
        else *out = slot == 0 ? S3_E1 : slot == 1 ? (chain == 0 ? S3_E2F : S3_E2L) : slot == 2 ? S3_Y : S3_NULL;
        return slot >= 0 && slot < 3;
    };
    for (int p = 0; p < 3; ++p) {
        const FastPred& f = P.fast[p];
        S3Pred& d = s.f[p];
        if (f.kind == FP_TRUE || (f.kind == FP_NONE && P.st[p].filter.len == 0)) {
            d.kind = FP_TRUE;
            continue;
        }
        if (f.kind != FP_CONST && f.kind != FP_SLOT) return why = 11, false;
        d.kind = f.kind;
        d.op = f.op;
        d.t = f.t;
        d.konst = f.konst;
        if (!src(p, f.sa, f.ia, &d.a.src) || f.ca < 0 || f.ca >= P.n_cols) return why = 12, false;
        d.a.col = (uint8_t)f.ca;
        d.a.kind = f.ka;
        if (f.kind == FP_SLOT) {
            if (!src(p, f.sb, f.ib, &d.b.src) || f.cb < 0 || f.cb >= P.n_cols) return why = 13, false;
            d.b.col = (uint8_t)f.cb;
            d.b.kind = f.kb;
        }
    }
    for (int j = 0; j < P.n_out; ++j) {
        const Prog pr = P.out_prog[j];
        if (pr.len != 1 || h.code[pr.start].op != OP_LOAD) return why = 14, false;
        const Instr in = h.code[pr.start];
        if (!src(2, in.a, in.c, &s.out[j].src) || in.b < 0 || in.b >= P.n_cols) return why = 15, false;
        s.out[j].col = (uint8_t)in.b;
        s.out[j].kind = in.k;
    }
    return true;
}

// chain_match_k's LDS tile: the columns the state-1 filter reads from its own event (the scanned rows), and
// whether any filter / select needs the bytecode interpreter (its stack lives in LDS)
void chain_staging(const HostQuery& h, ChainArgs& a, bool carry_nullable) {
    const Plan& P = h.plan;
    ChainSpec& sp = a.sp;
    sp.n_states = P.n_states;
    sp.has_within = P.has_within;
    sp.within_ms = P.within_ms;
    sp.f0 = P.fast[0];
    sp.prog0 = P.st[0].filter;
    if (P.n_states > 1) {
        sp.f1 = P.fast[1];
        sp.prog1 = P.st[1].filter;
    }
    sp.n_out = P.n_out;
    sp.n_cols = P.n_cols;
    for (int c = 0; c < P.n_cols; ++c) sp.col_kind[c] = P.col_kind[c];
    for (int j = 0; j < P.n_out; ++j) {
        const Prog pr = P.out_prog[j];
        sp.out_prog[j] = pr;
        sp.out_direct[j] = pr.len == 1 && h.code[pr.start].op == OP_LOAD;
        if (sp.out_direct[j]) sp.out_ins[j] = h.code[pr.start];
    }
    for (int c = 0; c < MAX_COLS; ++c) a.stage_of[c] = -1;
    a.n_stage = 0;
    auto stage = [&](int col) {
        if (col < 0 || col >= P.n_cols || a.stage_of[col] >= 0 || a.n_stage >= CM_SCOLS) return;
        a.stage_of[col] = (int8_t)a.n_stage;
        a.stage_col[a.n_stage++] = col;
    };
    bool stack = P.fast[0].kind == FP_NONE;
    // e2 filter as a typed scan (chain.hip scan_typed) when it has one of the common shapes
    sp.scan_mode = SCAN_GENERIC;
    if (P.n_states > 1) {
        const FastPred& f = P.fast[1];
        auto plain = [](int8_t i) { return i == 0 || i == -1; };
        if (f.kind == FP_TRUE) {
            sp.scan_mode = SCAN_TRUE;
            sp.scan_t = VK_I64;
        } else if (f.kind == FP_CONST && f.sa == 1 && plain(f.ia)) {
            sp.scan_mode = SCAN_CONST;
            sp.scan_col = f.ca; sp.scan_col_kind = f.ka; sp.scan_t = f.t; sp.scan_op = f.op; sp.scan_e2_left = 1;
            sp.scan_konst = f.konst;
        } else if (f.kind == FP_SLOT && plain(f.ia) && plain(f.ib) && f.sa == 1 && f.sb == 0) {
            sp.scan_mode = SCAN_E1;
            sp.scan_col = f.ca; sp.scan_col_kind = f.ka; sp.scan_t = f.t; sp.scan_op = f.op; sp.scan_e2_left = 1;
            sp.e1_col = f.cb; sp.e1_col_kind = f.kb;
        } else if (f.kind == FP_SLOT && plain(f.ia) && plain(f.ib) && f.sa == 0 && f.sb == 1) {
            sp.scan_mode = SCAN_E1;
            sp.scan_col = f.cb; sp.scan_col_kind = f.kb; sp.scan_t = f.t; sp.scan_op = f.op; sp.scan_e2_left = 0;
            sp.e1_col = f.ca; sp.e1_col_kind = f.ka;
        }
        if (f.kind == FP_CONST || f.kind == FP_SLOT) {
            if (f.sa == 1) stage(f.ca);
            if (f.kind == FP_SLOT && f.sb == 1) stage(f.cb);
        } else if (f.kind == FP_NONE) {
            stack = true;
            const Prog pr = P.st[1].filter;
            for (int i = pr.start; i < pr.start + pr.len; ++i)
                if (h.code[i].op == OP_LOAD && h.code[i].a == 1) stage(h.code[i].b);
        }
    }
    for (int j = 0; j < P.n_out; ++j) {
        const Prog pr = P.out_prog[j];
        if (!(pr.len == 1 && h.code[pr.start].op == OP_LOAD)) stack = true;
    }
    a.lds_stack = stack;
    a.generic = stack || (P.n_states > 1 && sp.scan_mode == SCAN_GENERIC);
    a.scan_lds = (sp.scan_mode == SCAN_CONST || sp.scan_mode == SCAN_E1) && a.stage_of[sp.scan_col] >= 0 &&
                 a.nulls[sp.scan_col] == nullptr;
    // outputs are plain attributes of null-free columns: no output can be null
    bool nullable = false;
    for (int j = 0; j < P.n_out; ++j) {
        if (!sp.out_direct[j]) { nullable = true; break; }
        const Instr& in = sp.out_ins[j];
        if (!(in.c == 0 || in.c == -1) || in.a >= P.n_states || a.nulls[in.b]) nullable = true;
    }
    if (a.cin_n > 0 && carry_nullable) nullable = true;  // carried partials keep their batch's null bits
    a.write_nulls = nullable;
    // deque path (chain.hip chain_deque_k): one stream, c1 = `e2.x OP e1.x` (OP ordering) or independent of e1,
    // c0 a FastPred, plain-attribute selects
    a.deque_mode = DQ_OFF;
    const bool one_stream = P.n_states == 2 && a.qstream == nullptr && P.st[0].stream == P.st[1].stream;
    const bool ordering = sp.scan_op == CMP_GT || sp.scan_op == CMP_GE || sp.scan_op == CMP_LT || sp.scan_op == CMP_LE;
    if (one_stream && !a.generic && P.fast[0].kind != FP_NONE) {
        if (sp.scan_mode == SCAN_E1 && ordering && sp.e1_col == sp.scan_col && sp.e1_col_kind == sp.scan_col_kind)
            a.deque_mode = DQ_STACK;
        else if (sp.scan_mode == SCAN_CONST || sp.scan_mode == SCAN_TRUE)
            a.deque_mode = DQ_ALL;
    }
    if (a.deque_mode == DQ_ALL && sp.scan_mode == SCAN_TRUE) sp.scan_col = 0, sp.scan_col_kind = P.col_kind[0];
    const FastPred& f0 = P.fast[0];
    a.f0_on_x = f0.kind == FP_CONST && f0.sa == 0 && (f0.ia == 0 || f0.ia == -1) && f0.ca == sp.scan_col &&
                f0.ka == sp.scan_col_kind;
}

// the batch view of a query whose rows all come from mixed pushes, built on the device (ingest.hip): each chunk's
// raw rows go to HBM once per flush, then a stable compaction writes the query's view rows (its streams, null keys
// dropped), physical columns, stream positions, batch positions and key values. Returns the view's row count.
int64_t mixed_view(sdg_engine* e, QueryRt& q, const std::vector<const PushChunk*>& parts,
                   const std::vector<int64_t>& part_pos, int64_t n, const int64_t** d_ts, const uint8_t** d_qs,
                   const void** d_cols, const uint8_t** d_nulls, const uint32_t** d_vpos) {
    const HostQuery& h = q.hq;
    const Plan& P = h.plan;
    hipStream_t st = e->stream;
    const int nc = P.n_cols;
    const bool multi = h.streams.size() > 1;
    MixedViewArgs proto;
    std::memset(&proto, 0, sizeof proto);
    for (int s2 = 0; s2 < MV_MAX_STREAMS; ++s2) proto.qpos[s2] = -1;
    for (size_t i = 0; i < h.streams.size(); ++i) proto.qpos[h.streams[i]] = (int8_t)i;
    proto.partitioned = P.partitioned;
    for (size_t i = 0; i < h.streams.size(); ++i) {
        proto.key_attr[i] = P.partitioned ? h.key_attr[i] : -1;
        proto.key_kind[i] = P.partitioned ? h.key_kind[i] : 0;
        for (int k = 0; k < nc; ++k) proto.col_attr[i][k] = (int8_t)h.col_attr[i][k];
    }
    proto.n_cols = nc;
    for (int k = 0; k < nc; ++k) proto.col_width[k] = (uint8_t)width_of(P.col_kind[k]);
    // raw rows to HBM (once per chunk and flush) and the per-chunk view row counts
    std::vector<MixedViewArgs> args(parts.size(), proto);
    bool col_null[MAX_COLS] = {};
    size_t wsz = 0;
    for (const PushChunk* pc : parts) wsz = std::max(wsz, mixed_view_workspace(pc->n));
    uint8_t* work = (uint8_t*)q.mv_work.ensure(parts.size() * ((wsz + 255) & ~(size_t)255) + 256);
    int64_t* d_tot = (int64_t*)q.mv_tot.ensure(parts.size() * 8 + 8);
    MixedViewArgs* d_args = (MixedViewArgs*)q.mv_args.ensure(parts.size() * sizeof(MixedViewArgs));
    for (size_t pi = 0; pi < parts.size(); ++pi) {
        PushChunk& c = const_cast<PushChunk&>(*parts[pi]);
        const int na = (int)c.cols.size();
        if (!c.m_up) {
            c.m_streams.ensure((size_t)c.n * 4);
            c.m_ts.ensure((size_t)c.n * 8);
            c.m_slots.ensure((size_t)std::max(na, 1) * c.n * 8);
            HIPCHECK(hipMemcpyAsync(c.m_streams.p, c.rstream.data(), (size_t)c.n * 4, hipMemcpyHostToDevice, st));
            HIPCHECK(hipMemcpyAsync(c.m_ts.p, c.ts.data(), (size_t)c.n * 8, hipMemcpyHostToDevice, st));
            for (int a = 0; a < na; ++a)
                HIPCHECK(hipMemcpyAsync((int64_t*)c.m_slots.p + (size_t)a * c.n, c.cols[a].data(), (size_t)c.n * 8,
                                        hipMemcpyHostToDevice, st));
            c.m_has_null.assign(na, 0);
            int nn = 0;
            for (int a = 0; a < na; ++a)
                if (!c.nulls[a].empty())
                    for (int64_t r = 0; r < c.n && !c.m_has_null[a]; ++r) c.m_has_null[a] = c.nulls[a][r] != 0;
            for (int a = 0; a < na; ++a) nn += c.m_has_null[a];
            if (nn) {
                c.m_nulls.ensure((size_t)na * c.n);
                for (int a = 0; a < na; ++a)
                    if (c.m_has_null[a])
                        HIPCHECK(hipMemcpyAsync((uint8_t*)c.m_nulls.p + (size_t)a * c.n, c.nulls[a].data(), (size_t)c.n,
                                                hipMemcpyHostToDevice, st));
            }
            c.m_up = true;
        }
        MixedViewArgs& a = args[pi];
        a.n = c.n;
        a.pos0 = part_pos[pi];
        a.streams = c.m_streams.as<int32_t>();
        a.ts = c.m_ts.as<int64_t>();
        for (int x = 0; x < na; ++x) {
            a.slots[x] = c.m_slots.as<int64_t>() + (size_t)x * c.n;
            a.slot_nulls[x] = c.m_has_null[x] ? (const uint8_t*)c.m_nulls.p + (size_t)x * c.n : nullptr;
        }
        for (size_t i = 0; i < h.streams.size(); ++i)
            for (int k = 0; k < nc; ++k) {
                const int ai = h.col_attr[i][k];
                if (ai >= 0 && ai < na && c.m_has_null[ai]) col_null[k] = true;
            }
    }
    HIPCHECK(hipMemcpyAsync(d_args, args.data(), parts.size() * sizeof(MixedViewArgs), hipMemcpyHostToDevice, st));
    for (size_t pi = 0; pi < parts.size(); ++pi)
        mixed_view_count(args[pi], d_args + pi, work + pi * ((wsz + 255) & ~(size_t)255), d_tot + pi, st);
    std::vector<int64_t> tot(parts.size());
    HIPCHECK(hipMemcpyAsync(tot.data(), d_tot, parts.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    int64_t rows = 0;
    for (int64_t t : tot) rows += t;
    const size_t cnt = (size_t)std::max<int64_t>(rows, 1);
    int64_t* ots = (int64_t*)q.st_ts.ensure(cnt * 8);
    uint32_t* opos = (uint32_t*)q.d_vpos.ensure(cnt * 4);
    uint8_t* oqs = multi ? (uint8_t*)q.st_qs.ensure(cnt) : nullptr;
    int64_t* okey = P.partitioned ? (int64_t*)q.kt_vals_in.ensure(cnt * 8) : nullptr;
    for (int k = 0; k < nc; ++k) {
        d_cols[k] = q.st_cols[k].ensure(cnt * width_of(P.col_kind[k]));
        d_nulls[k] = col_null[k] ? (const uint8_t*)q.st_nulls[k].ensure(cnt) : nullptr;
    }
    int64_t o = 0;
    for (size_t pi = 0; pi < parts.size(); ++pi) {
        MixedViewArgs& a = args[pi];
        a.out_ts = ots + o;
        a.out_pos = opos + o;
        a.out_qs = oqs ? oqs + o : nullptr;
        a.out_key = okey ? okey + o : nullptr;
        for (int k = 0; k < nc; ++k) {
            a.out_cols[k] = (uint8_t*)d_cols[k] + (size_t)o * width_of(P.col_kind[k]);
            a.out_nulls[k] = d_nulls[k] ? (uint8_t*)d_nulls[k] + o : nullptr;
        }
        o += tot[pi];
    }
    HIPCHECK(hipMemcpyAsync(d_args, args.data(), parts.size() * sizeof(MixedViewArgs), hipMemcpyHostToDevice, st));
    for (size_t pi = 0; pi < parts.size(); ++pi)
        mixed_view_write(args[pi], d_args + pi, work + pi * ((wsz + 255) & ~(size_t)255), st);
    if (P.partitioned && q.string_keys && rows > 0) {  // string ids are the key ids
        uint32_t* k32 = (uint32_t*)q.st_key.ensure(cnt * 4);
        narrow_u32(okey, rows, k32, st);
    }
    HIPCHECK(hipStreamSynchronize(st));  // (args / totals are host vectors)
    *d_ts = ots;
    *d_qs = oqs;
    *d_vpos = opos;
    (void)n;
    return rows;
}

// ---- spilled keys (QueryRt::spill) ---------------------------------------------------------------------------
// the flush's sorted view, as the generic NFA kernel reads it
struct SpillView {
    const int64_t* ts;
    const uint8_t* qs;        // nullptr: single stream
    const uint32_t* vrank;
    const uint32_t* orig;     // view row -> batch position - pos_off (nullptr: identity)
    int64_t pos_off;
    const uint32_t* seg_b;    // nullptr: unpartitioned (one key, every row)
    const uint32_t* seg_e;
    int64_t K;
    int64_t n;
    const void* const* cols;
    const uint8_t* const* nulls;
    int nc;
};

// Takes the keys that overflowed the device's largest layout over to the host (their batch-start state, migrated
// into a 32-bit layout of twice the slots), then runs every spilled key's rows of this flush there
// (KeyRunT<int32_t>, the same nfa.h code), doubling a key's layout and rerunning it from its batch-start state
// whenever it outgrows it. The runs' records join the device's in drain().
void spill_keys(sdg_engine* e, QueryRt& q, const std::vector<uint32_t>& fresh, const SpillView& v,
                const nfa::TimerIn& T, int64_t purge_from, int64_t purge_idle) {
    const Plan& P = q.hq.plan;
    const int64_t kb = q.L.bytes;
    const int ncols = std::max(P.n_cols, 1);
    HIPCHECK(hipStreamSynchronize(e->stream));
    for (uint32_t k : fresh) {
        std::vector<uint8_t> start((size_t)kb, 0);  // the key's committed state (zeros: fresh)
        int64_t s = k;
        uint8_t from = 0;
        if (q.reclaim) {
            int32_t so = -1;
            HIPCHECK(hipMemcpy(&so, q.slot_of.as<int32_t>() + k, 4, hipMemcpyDeviceToHost));
            if (so < 0) throw DeviceError("spilled key without an arena slot");
            s = so;
            HIPCHECK(hipMemcpy(&from, q.init_from.as<uint8_t>() + s, 1, hipMemcpyDeviceToHost));
        }
        if (from == 0) {
            uint8_t cur = 0;
            HIPCHECK(hipMemcpy(&cur, q.cur_bits.as<uint8_t>() + s, 1, hipMemcpyDeviceToHost));
            const uint8_t* committed = (cur ? q.arena2.as<uint8_t>() : q.arena.as<uint8_t>()) + s * kb;
            HIPCHECK(hipMemcpy(start.data(), committed, (size_t)kb, hipMemcpyDeviceToHost));
        } else if (from == 2) {  // rebuilt from its idle record, as the kernel did
            const int ib = nfa::idle_bytes(P.n_states);
            std::vector<uint8_t> rec((size_t)ib);
            HIPCHECK(hipMemcpy(rec.data(), q.idle_rec.as<uint8_t>() + (int64_t)k * ib, (size_t)ib, hipMemcpyDeviceToHost));
            nfa::CtxT<true> c;
            c.P = &P;
            c.L = q.L;
            c.base = start.data();
            nfa::from_idle(c, rec.data());
        }
        QueryRt::Spilled& sp = q.spill[k];
        sp.L = nfa::make_layout<int32_t>(P.n_states, ncols, 2 * q.L.ns, P.n_sched);
        sp.arena.assign((size_t)sp.L.bytes, 0);
        nfa::CtxT<true, int32_t> d;
        d.P = &P;
        d.L = sp.L;
        d.base = sp.arena.data();
        nfa::migrate_key<int16_t>(d, start.data(), q.L);
        if (P.purge) {
            int64_t ls = 0;
            HIPCHECK(hipMemcpy(&ls, q.last_seen_bak.as<int64_t>() + k, 8, hipMemcpyDeviceToHost));
            sp.purge_last = ls ^ INT64_MIN;
        }
        e->stats.spilled_keys += 1;
    }
    if (!v.ts && v.n > 0) throw DeviceError("spilled keys: the batch view has no timestamps");
    for (auto& kv : q.spill) {
        const uint32_t k = kv.first;
        QueryRt::Spilled& sp = kv.second;
        int64_t b = 0, en = v.n;
        if (v.seg_b) {
            if ((int64_t)k >= v.K) continue;  // no rows in this flush (nothing runs without rows: no timers)
            uint32_t be[2];
            HIPCHECK(hipMemcpy(&be[0], v.seg_b + k, 4, hipMemcpyDeviceToHost));
            HIPCHECK(hipMemcpy(&be[1], v.seg_e + k, 4, hipMemcpyDeviceToHost));
            b = be[0];
            en = be[1];
        }
        const int64_t m = en - b;
        if (m <= 0) continue;
        // the key's rows (view order = its time order)
        KeyRunT<int32_t> rows;
        rows.ts.resize(m);
        rows.pos.resize(m);
        HIPCHECK(hipMemcpy(rows.ts.data(), v.ts + b, (size_t)m * 8, hipMemcpyDeviceToHost));
        if (v.orig) {
            std::vector<uint32_t> o(m);
            HIPCHECK(hipMemcpy(o.data(), v.orig + b, (size_t)m * 4, hipMemcpyDeviceToHost));
            for (int64_t p = 0; p < m; ++p) rows.pos[p] = (uint32_t)(v.pos_off + o[p]);
        } else {
            for (int64_t p = 0; p < m; ++p) rows.pos[p] = (uint32_t)(v.pos_off + b + p);
        }
        if (v.vrank) {
            rows.vrank.resize(m);
            HIPCHECK(hipMemcpy(rows.vrank.data(), v.vrank + b, (size_t)m * 4, hipMemcpyDeviceToHost));
        }
        rows.has_qs = v.qs != nullptr;
        if (v.qs) {
            rows.qs.resize(m);
            HIPCHECK(hipMemcpy(rows.qs.data(), v.qs + b, (size_t)m, hipMemcpyDeviceToHost));
        }
        rows.cols.resize(v.nc);
        rows.nulls.resize(v.nc);
        for (int c = 0; c < v.nc; ++c) {
            const int w = width_of(P.col_kind[c]);
            rows.cols[c].resize((size_t)m * w);
            HIPCHECK(hipMemcpy(rows.cols[c].data(), (const uint8_t*)v.cols[c] + b * w, (size_t)m * w, hipMemcpyDeviceToHost));
            if (v.nulls[c]) {
                rows.nulls[c].resize(m);
                HIPCHECK(hipMemcpy(rows.nulls[c].data(), v.nulls[c] + b, (size_t)m, hipMemcpyDeviceToHost));
            }
        }
        int64_t slack = 4096;
        for (;;) {
            std::unique_ptr<KeyRunT<int32_t>> r(new KeyRunT<int32_t>());
            r->slack = slack;
            r->key = k;
            r->arena = sp.arena;  // batch-start state (kept until the run succeeds)
            r->ts = rows.ts;
            r->pos = rows.pos;
            r->vrank = rows.vrank;
            r->qs = rows.qs;
            r->has_qs = rows.has_qs;
            r->cols = rows.cols;
            r->nulls = rows.nulls;
            if (P.purge) {
                const nfa::PurgeIn pin{e->bc.clk.data(), purge_from, purge_idle, sp.purge_last};
                r->start(&P, q.hq.code.data(), q.hq.consts.data(), sp.L, T, e->seq, &pin);
            } else {
                r->start(&P, q.hq.code.data(), q.hq.consts.data(), sp.L, T, e->seq);
            }
            r->rows_before(INT64_MAX);
            if (!r->arena_overflow() && r->output_overflow()) {  // one event completed more partials than the
                slack = (int64_t)r->emitted() + 4096;                // sink's slack: again with room for all of them
                continue;
            }
            if (!r->arena_overflow()) {
                if (r->overflow()) throw DeviceError("spilled key: host run sink overflow");
                sp.arena.swap(r->arena);
                if (P.purge) sp.purge_last = r->purge_last();
                e->stats.host_rows += m;
                q.spill_runs.push_back(std::move(r));
                break;
            }
            if (sp.L.ns >= (1 << 22))
                throw CompileError(SDG_ERR_CAPACITY, "query '" + q.hq.name + "': a partition key holds more than " +
                                                         std::to_string(sp.L.ns) + " live partial matches");
            const nfa::Layout Ln = nfa::make_layout<int32_t>(P.n_states, ncols, 2 * sp.L.ns, P.n_sched);
            std::vector<uint8_t> na((size_t)Ln.bytes, 0);
            nfa::CtxT<true, int32_t> d;
            d.P = &P;
            d.L = Ln;
            d.base = na.data();
            nfa::migrate_key<int32_t>(d, sp.arena.data(), sp.L);
            sp.arena.swap(na);
            sp.L = Ln;
        }
    }
}

// after the flush's commit: the device skips the newly spilled keys from now on (reclaiming queries: the key's
// slot returns to the pool and slot_of says -3; others: KH_HOST in both copies of the key's arena head)
void mark_spilled(sdg_engine* e, QueryRt& q, const std::vector<uint32_t>& keys, const SlotPool& sp) {
    HIPCHECK(hipStreamSynchronize(e->stream));
    if (q.reclaim) {
        unsigned int top = 0;
        HIPCHECK(hipMemcpy(&top, sp.counters, 4, hipMemcpyDeviceToHost));
        for (uint32_t k : keys) {
            int32_t s = -1;
            HIPCHECK(hipMemcpy(&s, sp.slot_of + k, 4, hipMemcpyDeviceToHost));
            if (s >= 0) {
                HIPCHECK(hipMemcpy(sp.free_slots + top, &s, 4, hipMemcpyHostToDevice));
                ++top;
            }
            const int32_t host = -3;
            HIPCHECK(hipMemcpy(sp.slot_of + k, &host, 4, hipMemcpyHostToDevice));
        }
        HIPCHECK(hipMemcpy(sp.counters, &top, 4, hipMemcpyHostToDevice));
        return;
    }
    const int64_t kb = q.L.bytes;
    for (uint32_t k : keys) {
        for (uint8_t* base : {q.arena.as<uint8_t>(), q.arena2.as<uint8_t>()}) {
            if (!base) continue;
            int32_t f = 0;
            HIPCHECK(hipMemcpy(&f, base + (int64_t)k * kb, 4, hipMemcpyDeviceToHost));
            f = (f & ~1) | 2 | nfa::KH_HOST;
            HIPCHECK(hipMemcpy(base + (int64_t)k * kb, &f, 4, hipMemcpyHostToDevice));
        }
    }
}

// A chain query moving to the generic NFA: its carried partials (e1 events still pending at the end of the last
// committed batch) are run through the NFA as events of the state-0 stream, in arrival order per key, before the
// batch. That rebuilds exactly the pending lists the reference holds: none of them can complete or expire another
// (each survived every later event of its key, these included, in the real history), and each re-creates its
// partial. The replay must therefore emit nothing; it is checked.
void replay_carries(sdg_engine* e, QueryRt& q, const NfaArgs& a0, bool multi_stream) {
    q.replay_carries = false;
    const Plan& P = q.hq.plan;
    hipStream_t st = e->stream;
    QueryRt::Carry& cin = q.carry[q.cur];
    const int64_t n = cin.n;
    const int nc = P.n_cols;
    cin.n = 0;
    if (n <= 0) return;
    std::vector<uint32_t> key(n);
    std::vector<int64_t> ts(n), seq(n), vals((size_t)std::max(nc, 1) * n);
    std::vector<uint32_t> nm(n);
    HIPCHECK(hipMemcpy(key.data(), cin.key.p, n * 4, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(ts.data(), cin.ts.p, n * 8, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(seq.data(), cin.seq.p, n * 8, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(nm.data(), cin.nulls.p, n * 4, hipMemcpyDeviceToHost));
    for (int j = 0; j < nc; ++j)
        HIPCHECK(hipMemcpy(vals.data() + (size_t)j * n, (const int64_t*)cin.vals.p + (size_t)j * cin.cap, n * 8,
                           hipMemcpyDeviceToHost));
    std::vector<int64_t> ord(n);
    for (int64_t i = 0; i < n; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return key[x] != key[y] ? key[x] < key[y] : seq[x] < seq[y]; });
    const int64_t KS = P.partitioned ? a0.K : 1;
    std::vector<uint32_t> sb(KS, 0), se(KS, 0);
    std::vector<int64_t> rts(n);
    std::vector<std::vector<uint8_t>> cols(nc), nulls(nc);
    for (int j = 0; j < nc; ++j) {
        cols[j].resize((size_t)n * width_of(P.col_kind[j]));
        nulls[j].assign(n, 0);
    }
    bool any_null[MAX_COLS] = {};
    for (int64_t r = 0; r < n; ++r) {
        const int64_t i = ord[r];
        const uint32_t k = P.partitioned ? key[i] : 0;
        if (k >= (uint32_t)KS) throw DeviceError("carried partial of an unknown key");
        if (r == 0 || (P.partitioned && key[ord[r - 1]] != key[i])) sb[k] = (uint32_t)r;
        se[k] = (uint32_t)(r + 1);
        rts[r] = ts[i];
        for (int j = 0; j < nc; ++j) {
            const int w = width_of(P.col_kind[j]);
            std::memcpy(&cols[j][(size_t)r * w], &vals[(size_t)j * n + i], w);  // the slot's low bytes
            if ((nm[i] >> j) & 1u) {
                nulls[j][r] = 1;
                any_null[j] = true;
            }
        }
    }
    NfaArgs b = a0;
    b.n = n;
    b.ts = (const int64_t*)q.rp_ts.ensure(n * 8);
    HIPCHECK(hipMemcpy((void*)b.ts, rts.data(), n * 8, hipMemcpyHostToDevice));
    b.qstream = nullptr;
    if (multi_stream) {
        std::vector<uint8_t> qs(n, (uint8_t)q.hq.stream_pos(P.st[0].stream));
        b.qstream = (const uint8_t*)q.rp_qs.ensure(n);
        HIPCHECK(hipMemcpy((void*)b.qstream, qs.data(), n, hipMemcpyHostToDevice));
    }
    if (P.partitioned) {
        b.seg_start = (const uint32_t*)q.rp_seg.ensure(KS * 4);
        b.seg_end = (const uint32_t*)q.rp_segend.ensure(KS * 4);
        HIPCHECK(hipMemcpy((void*)b.seg_start, sb.data(), KS * 4, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy((void*)b.seg_end, se.data(), KS * 4, hipMemcpyHostToDevice));
    }
    b.orig = nullptr;
    b.pos_off = 0;
    for (int j = 0; j < nc; ++j) {
        b.cols[j] = q.rp_cols[j].ensure(cols[j].size());
        HIPCHECK(hipMemcpy((void*)b.cols[j], cols[j].data(), cols[j].size(), hipMemcpyHostToDevice));
        b.nulls[j] = nullptr;
        if (any_null[j]) {
            b.nulls[j] = (const uint8_t*)q.rp_nulls[j].ensure(n);
            HIPCHECK(hipMemcpy((void*)b.nulls[j], nulls[j].data(), n, hipMemcpyHostToDevice));
        }
    }
    const int64_t cap = 2 * n + 4096;
    b.out_cap = cap;
    b.out_ts = (int64_t*)q.o_ts.ensure(cap * 8);
    b.out_key = (uint32_t*)q.o_key.ensure(cap * 4);
    b.out_vals = (int64_t*)q.o_vals.ensure((size_t)std::max(P.n_out, 1) * cap * 8);
    b.out_nulls = (uint32_t*)q.o_nulls.ensure(cap * 4);
    b.out_emit_seq = (int64_t*)q.o_emit.ensure(cap * 8);
    b.out_sub = (int64_t*)q.o_first.ensure(cap * 8);
    b.out_round = nullptr;
    unsigned long long* counters = (unsigned long long*)q.counters.ensure(16);
    b.out_count = counters;
    b.flags = (int*)q.flags.ensure(32);
    b.list = nullptr;
    b.nlist = 0;
    HIPCHECK(hipMemsetAsync(counters, 0, 16, st));
    HIPCHECK(hipMemsetAsync(b.flags, 0, 32, st));
    NfaArgs* h_na = (NfaArgs*)q.h_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));
    NfaArgs* d_na = (NfaArgs*)q.d_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));
    *h_na = b;
    HIPCHECK(hipMemcpyAsync(d_na, h_na, sizeof(NfaArgs), hipMemcpyHostToDevice, st));
    nfa_run(b, d_na, st);
    unsigned long long hc[2];
    int hf[8];
    HIPCHECK(hipMemcpyAsync(hc, counters, 16, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(hf, b.flags, 32, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (hf[2])
        throw CompileError(SDG_ERR_CAPACITY, "query '" + q.hq.name + "': a partition key exceeded max_partials replaying "
                                                                     "its carried partials");
    if (hc[0] != 0 || hf[0]) throw DeviceError("query '" + q.hq.name + "': replaying carried partials emitted matches");
    e->stats.match_launches += 1;
    nfa_commit(q.cur_bits.as<uint8_t>(), q.ran_bits.as<uint8_t>(), q.arena_keys, st);  // the batch starts from it
}

// per-kernel HIP event timing (sdg_stats); SDG_NO_EVENTS=1 drops the event records (measuring their cost)
const bool g_no_events = getenv("SDG_NO_EVENTS") != nullptr;
void ev_record(hipEvent_t ev, hipStream_t st) {
    if (!g_no_events) HIPCHECK(hipEventRecord(ev, st));
}
void ev_elapsed(float* ms, hipEvent_t a, hipEvent_t b) {
    *ms = 0;
    if (!g_no_events) HIPCHECK(hipEventElapsedTime(ms, a, b));
}

// SDG_HOST_PROF: host timestamps of a flush's phases (where the host, not the device, sets the pace)
struct HostProf {
    bool on = getenv("SDG_HOST_PROF") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
    std::string s;
    void mark(const char* what) {
        if (!on) return;
        auto t = std::chrono::steady_clock::now();
        s += std::string(" ") + what + "=" + std::to_string(std::chrono::duration<double, std::micro>(t - last).count());
        last = t;
    }
    ~HostProf() {
        if (on) std::fprintf(stderr, "[host us]%s\n", s.c_str());
    }
};

KeyTab kt_view(QueryRt& q) {
    return KeyTab{q.kt_keys.as<KtSlot>(), q.kt_cap - 1, q.kt_cap};
}

// the host dictionary's ids [kt_synced, K) into the device key table (keys the host path assigned)
void kt_sync(sdg_engine* e, QueryRt& q) {
    const size_t K = q.keystr.size();
    if (q.kt_synced >= K) return;
    std::vector<int64_t> vals(K - q.kt_synced);
    for (size_t i = q.kt_synced; i < K; ++i) vals[i - q.kt_synced] = key_value_of_string(q.key_class, q.keystr[i]);
    int64_t* d_vals = (int64_t*)q.kt_vals.ensure(vals.size() * 8);
    int* d_flags = (int*)((uint8_t*)q.kt_cnt.ensure(32) + 8);
    HIPCHECK(hipMemcpy(d_vals, vals.data(), vals.size() * 8, hipMemcpyHostToDevice));
    HIPCHECK(hipMemsetAsync(d_flags, 0, 8, e->stream));
    kt_load(kt_view(q), d_vals, (uint32_t)q.kt_synced, (int64_t)vals.size(), d_flags, e->stream);
    int hf = 0;
    HIPCHECK(hipMemcpyAsync(&hf, d_flags, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHECK(hipStreamSynchronize(e->stream));
    if (hf) throw DeviceError("device key table: probe limit while loading the dictionary");
    q.kt_synced = K;
}

void kt_rebuild(sdg_engine* e, QueryRt& q, uint64_t cap) {
    uint64_t c = 1;
    while (c < cap) c <<= 1;
    q.kt_cap = c;
    q.kt_keys.ensure((size_t)(c + 1) * sizeof(KtSlot));
    kt_clear(kt_view(q), e->stream);
    q.kt_synced = 0;
    kt_sync(e, q);
}

// dense key ids of a device-resident batch keyed by an int / long attribute: looked up (and new keys inserted) in
// the device key table; new keys get the next ids in order of their first row, as host_key assigns them, and
// enter the host dictionary too (snapshots, scheduler hashes, later host pushes)
const uint32_t* device_key_ids(sdg_engine* e, QueryRt& q, const void* col, int kind, int64_t n) {
    hipStream_t st = e->stream;
    uint32_t* out = (uint32_t*)q.st_key.ensure((size_t)std::max<int64_t>(n, 1) * 4);
    if (n <= 0) return out;
    uint64_t want = 0;
    for (int attempt = 0;; ++attempt) {
        if (attempt > 8) throw DeviceError("device key table: could not size the table");
        const size_t K0 = q.keystr.size();
        want = std::max<uint64_t>(want, std::max<uint64_t>(1u << 16, 4 * (uint64_t)K0));
        if (q.kt_cap < want) kt_rebuild(e, q, want);
        else kt_sync(e, q);
        const KeyTab t = kt_view(q);
        uint8_t* d_c = (uint8_t*)q.kt_cnt.ensure(32);
        unsigned long long* d_cnt = (unsigned long long*)d_c;
        int* d_flags = (int*)(d_c + 8);
        HIPCHECK(hipMemsetAsync(d_c, 0, 32, st));
        kt_probe(t, col, kind, n, out, d_cnt, t.cap / 2 - K0, d_flags, st);  // (cap >= 4 K0)
        uint8_t* hr = (uint8_t*)q.kt_ret.ensure(16);
        HIPCHECK(hipMemcpyAsync(hr, d_c, 16, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        const uint64_t cnt = *(unsigned long long*)hr;
        const int flags = *(int*)(hr + 8) | *(int*)(hr + 12);
        if (flags || K0 + cnt > t.cap / 2) {  // probe limit / over half full (pass stopped): larger table, again
            want = std::max<uint64_t>(4 * (K0 + cnt), 8 * t.cap);
            q.kt_cap = 0;
            continue;
        }
        if (cnt == 0) return out;
        // the probe inserted the new keys (ids 0) into the table: if anything below fails, the table is rebuilt from
        // the dictionary at the next batch and the dictionary itself is rolled back to its K0 ids
        struct Rollback {
            QueryRt& q;
            size_t K0;
            bool armed = true;
            ~Rollback() {
                if (!armed) return;
                q.kt_cap = 0;
                q.kt_synced = 0;
                for (size_t i = K0; i < q.keystr.size(); ++i) q.keydict.erase(q.keystr[i]);
                q.keystr.resize(K0);
                q.intkeys = IntKeyCache();
                if (q.key_class == KC_INT)
                    for (size_t i = 0; i < K0; ++i) q.intkeys.insert(std::stoll(q.keystr[i]), (uint32_t)i);
            }
        } rollback{q, K0};
        unsigned long long* d_pairs = (unsigned long long*)q.kt_pairs.ensure(cnt * 8);
        int64_t* d_vals = (int64_t*)q.kt_vals.ensure(cnt * 8);
        unsigned long long* d_n2 = (unsigned long long*)(d_c + 16);
        kt_collect(t, d_pairs, d_vals, d_n2, (int64_t)cnt, st);
        std::vector<unsigned long long> pairs(cnt);
        std::vector<int64_t> vals(cnt);
        HIPCHECK(hipMemcpyAsync(pairs.data(), d_pairs, cnt * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(vals.data(), d_vals, cnt * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        // new keys in order of their first row (pairs: first row << 32 | slot; first rows are distinct): an LSD
        // radix sort of the indices on the first row, 8 bits a pass (passes whose digit is constant skipped)
        std::vector<uint32_t> order(cnt), tmp(cnt);
        for (uint32_t i = 0; i < cnt; ++i) order[i] = i;
        for (int sh = 32; sh < 64; sh += 8) {
            size_t hist[257] = {};
            for (uint64_t i = 0; i < cnt; ++i) ++hist[((pairs[i] >> sh) & 0xFF) + 1];
            bool one = false;
            for (int d = 0; d < 256 && !one; ++d) one = hist[d + 1] == cnt;
            if (one) continue;
            for (int d = 0; d < 256; ++d) hist[d + 1] += hist[d];
            for (uint64_t j = 0; j < cnt; ++j) tmp[hist[(pairs[order[j]] >> sh) & 0xFF]++] = order[j];
            order.swap(tmp);
        }
        std::vector<uint32_t> slots(cnt);
        if (q.key_class != KC_INT) q.keydict.reserve(K0 + cnt);  // one rehash, not ~log2(cnt) of them
        q.keystr.reserve(K0 + cnt);
        for (uint64_t j = 0; j < cnt; ++j) {
            const uint32_t i = order[j];
            const uint32_t id = (uint32_t)(K0 + j);
            slots[j] = (uint32_t)(pairs[i] & 0xFFFFFFFFull);
            std::string ks = key_string_of_value(q.key_class, vals[i]);
            if (q.key_class != KC_INT && !q.keydict.emplace(ks, id).second)  // (KC_INT: intkeys is the dictionary)
                throw DeviceError("device key table out of step with the dictionary");
            q.keystr.push_back(std::move(ks));
            if (q.key_class == KC_INT) q.intkeys.insert(vals[i], id);
        }
        uint32_t* d_slots = (uint32_t*)q.kt_slots.ensure(cnt * 4);
        HIPCHECK(hipMemcpy(d_slots, slots.data(), cnt * 4, hipMemcpyHostToDevice));
        kt_assign(t, d_slots, (uint32_t)K0, (int64_t)cnt, st);
        kt_fix(t, col, kind, n, out, st);
        q.kt_synced = q.keystr.size();
        rollback.armed = false;
        return out;
    }
}

void flush_query(sdg_engine* e, QueryRt& q) {
    HostProf hp;
    HostQuery& h = q.hq;
    Plan& P = h.plan;
    hipStream_t st = e->stream;
    const int nc = P.n_cols;
    // ---- 1. batch view -------------------------------------------------------------------------------
    // the query's chunks and their batch positions (every pending chunk, any stream, and every advance_time point
    // takes positions: the clock and the sequence numbers count them all)
    std::vector<const PushChunk*> parts;
    std::vector<int64_t> part_pos;
    int64_t n = 0, gpos = 0;
    for (auto& c : e->pending) {
        bool mine = h.stream_pos(c.stream) >= 0;
        if (c.stream == -2)
            for (int s2 : h.streams) mine |= std::find(c.rstream.begin(), c.rstream.end(), s2) != c.rstream.end();
        if (mine) {
            parts.push_back(&c);
            part_pos.push_back(gpos);
            n += c.n;
        }
        gpos += c.n;
    }
    int64_t pos_off = 0;                  // position of view row 0 when rows map to positions contiguously
    const uint32_t* d_vpos = nullptr;     // [nrows] view row -> batch position otherwise
    const bool partitioned = P.partitioned;
    const bool multi_stream = h.streams.size() > 1;
    const int64_t* d_ts = nullptr;
    const uint8_t* d_qs = nullptr;
    const uint32_t* d_key = nullptr;
    const void* d_cols[MAX_COLS] = {};
    const uint8_t* d_nulls[MAX_COLS] = {};
    int64_t nrows = 0;
    const bool ranged = std::find(h.key_attr.begin(), h.key_attr.end(), -2) != h.key_attr.end() || q.broadcast;
    const uint32_t* d_vrank = nullptr;
    bool zero_copy = parts.size() == 1 && parts[0]->device && !multi_stream && parts[0]->stream >= 0 && !q.broadcast;
    // several staged host pushes of the query's one stream: consecutive rows of the stream's staging
    bool staged_run = !zero_copy && !multi_stream && !parts.empty() && !q.broadcast;
    for (size_t i = 0; i < parts.size() && staged_run; ++i)
        staged_run = parts[i]->device && parts[i]->stage_off >= 0 && parts[i]->stream == parts[0]->stream &&
                     (i == 0 || parts[i]->stage_off == parts[i - 1]->stage_off + parts[i - 1]->n);
    if (staged_run) zero_copy = true;
    if (zero_copy) {
        const PushChunk& c = *parts[0];
        int qpos = h.stream_pos(c.stream);
        pos_off = part_pos[0];
        bool contiguous = true;  // batch positions of the rows: one run, or a map (other streams' rows between)
        for (size_t i = 1; i < parts.size(); ++i) contiguous &= part_pos[i] == part_pos[i - 1] + parts[i - 1]->n;
        if (!contiguous) {
            std::vector<uint32_t> vpos((size_t)n);
            size_t o = 0;
            for (size_t i = 0; i < parts.size(); ++i)
                for (int64_t r = 0; r < parts[i]->n; ++r) vpos[o++] = (uint32_t)(part_pos[i] + r);
            d_vpos = (const uint32_t*)q.d_vpos.ensure((size_t)std::max<int64_t>(n, 1) * 4);
            HIPCHECK(hipMemcpy((void*)d_vpos, vpos.data(), (size_t)n * 4, hipMemcpyHostToDevice));
            pos_off = 0;
        }
        d_ts = c.d_ts;
        for (int k = 0; k < nc; ++k) {
            int ai = h.col_attr[qpos][k];
            d_cols[k] = ai >= 0 ? c.d_cols[ai] : nullptr;
            d_nulls[k] = ai >= 0 ? c.d_nulls[ai] : nullptr;
            if (!d_cols[k]) d_cols[k] = q.st_cols[k].ensure((size_t)std::max<int64_t>(n, 1) * width_of(P.col_kind[k]));
        }
        if (partitioned) {
            if (ranged) throw CompileError(SDG_ERR_UNSUPPORTED, "device-resident batches of a range partition");
            if (!q.string_keys && q.key_class == KC_NONE)
                throw CompileError(SDG_ERR_UNSUPPORTED, "device-resident batches of a partition whose key attributes mix "
                                                        "types");
            int ai = h.key_attr[qpos];
            if (c.d_nulls[ai]) throw CompileError(SDG_ERR_UNSUPPORTED, "null partition keys in device-resident batches");
            if (q.string_keys) d_key = (const uint32_t*)c.d_cols[ai];
            else d_key = device_key_ids(e, q, c.d_cols[ai], h.key_kind[qpos], n);
        }
        nrows = n;
    }
    // mixed pushes only (C4's interleaved streams): the view is built on the device from the raw slot rows
    bool dev_mixed = !zero_copy && !parts.empty() && !ranged && !q.broadcast && !getenv("SDG_NO_DEVMIX") &&
                     (!partitioned || q.string_keys || q.key_class != KC_NONE) &&
                     e->stream_types.size() <= (size_t)MV_MAX_STREAMS;
    for (const PushChunk* c : parts) dev_mixed &= c->stream == -2 && !c->device && c->cols.size() <= (size_t)MV_MAX_ATTRS;
    if (dev_mixed) {
        hp.mark("parts");
        nrows = mixed_view(e, q, parts, part_pos, n, &d_ts, &d_qs, d_cols, d_nulls, &d_vpos);
        hp.mark("mixed_view");
        if (partitioned) {
            if (q.string_keys) d_key = q.st_key.as<uint32_t>();
            else d_key = device_key_ids(e, q, q.kt_vals_in.as<int64_t>(), VK_I64, nrows);
        }
    } else if (zero_copy) {
    } else {
        // assemble on the host (host chunks) / device-to-device (device chunks)
        std::vector<int64_t> ts;
        std::vector<uint8_t> qs;
        std::vector<uint32_t> keys;
        std::vector<std::vector<uint8_t>> cols(nc), nulls(nc);
        std::vector<bool> any_null(nc, false);
        std::vector<uint32_t> vpos;
        std::vector<uint32_t> vrank;  // range partitions: the range each view row came from; broadcast rows: the key's
                                      // rank in getPartitionKeys() order (the delivery sub-order)
        // partitionKeys.put of a keyed row (broadcast queries): the key set and order the next broadcast row sees
        auto key_seen = [&](uint32_t key) {
            if (!q.broadcast) return;
            while (q.key_hash.size() <= (size_t)key) {
                const size_t k = q.key_hash.size();
                q.key_hash.push_back(java_spread_hash(q.string_keys ? e->strings.strs[k] : q.keystr[k]));
            }
            q.korder.add(key, q.key_hash[key]);
        };
        auto bcast_order = [&]() -> const std::vector<uint32_t>& {
            const std::vector<uint32_t>& o = q.korder.order();
            if (o.size() >= ((size_t)1 << 23))  // (the delivery rank sits in bits 40..62 of the record's sub key)
                throw CompileError(SDG_ERR_CAPACITY, "a broadcast to more than 2^23 partition keys");
            if (q.korder.tree_bins())  // the JDK's tree-bin iteration order is not modelled (keyorder.h)
                throw CompileError(SDG_ERR_UNSUPPORTED, "query '" + q.hq.name + "': the partition's key set has a "
                                                        "hash bin the JDK would turn into a tree bin; its broadcast "
                                                        "order is not modelled");
            return o;
        };
        // Broadcast rows are expanded on the device (bcast_expand, SDG_BCAST_HOST: here, row by row): the view holds one
        // placeholder row per event of a stream without a partition key (key BX_PLACEHOLDER) and the key order that
        // event saw, stored once per distinct order (keyorder.h version) -- host work O(events + orders x keys)
        // instead of O(events x keys)
        static const bool bc_host = getenv("SDG_BCAST_HOST") != nullptr;
        const bool bc_dev = q.broadcast && !bc_host;
        std::vector<uint32_t> bc_row, bc_off, bc_k, bc_ord;  // placeholders: compact row, order start, order length
        uint64_t bc_ver = ~0ull;
        auto bc_order_now = [&](uint32_t& off, uint32_t& k) {  // the current order, appended when it changed
            const std::vector<uint32_t>& o = bcast_order();
            if (bc_ver != q.korder.version() || bc_ord.empty()) {
                if (bc_ord.size() + o.size() > ((size_t)1 << 28))
                    throw CompileError(SDG_ERR_CAPACITY, "query '" + h.name + "': the broadcast key orders of one flush "
                                                         "exceed 2^28 entries (flush more often)");
                bc_ver = q.korder.version();
                bc_ord.insert(bc_ord.end(), o.begin(), o.end());
            }
            k = (uint32_t)o.size();
            off = (uint32_t)(bc_ord.size() - o.size());
        };
        ts.reserve(n);
        vpos.reserve(n);
        for (int k = 0; k < nc; ++k) cols[k].reserve((size_t)n * width_of(P.col_kind[k]));
        for (size_t pi = 0; pi < parts.size(); ++pi) {
            const PushChunk* c = parts[pi];
            if (c->device) throw CompileError(SDG_ERR_UNSUPPORTED, "mixed / multi-stream device-resident batches");
            if (c->stream == -2) {  // mixed chunk (attributes as 64-bit slots): the view rows first, then one fill
                struct VRow {
                    int64_t r;
                    uint32_t key;
                    uint32_t rank;
                    uint8_t qpos;
                };
                std::vector<VRow> vr;
                vr.reserve((size_t)c->n);
                std::vector<uint32_t> ph_j, ph_off, ph_k;  // placeholders among vr (their compact row follows below)
                constexpr int64_t PF = 16;
                auto pf = [&](int64_t r) {  // the integral key slot of row r, ahead of its lookup
                    const int qp = h.stream_pos(c->rstream[r]);
                    if (qp < 0 || h.key_attr[qp] < 0) return;
                    const uint8_t kk = h.key_kind[qp];
                    if (kk != VK_I32 && kk != VK_I64) return;
                    const int64_t sv = ((const int64_t*)c->cols[h.key_attr[qp]].data())[r];
                    q.intkeys.prefetch(kk == VK_I32 ? (int64_t)(int32_t)sv : sv);
                };
                const bool do_pf = partitioned && !q.string_keys;
                for (int64_t r = 0; r < c->n; ++r) {
                    if (do_pf && r + PF < c->n) pf(r + PF);
                    const int qpos = h.stream_pos(c->rstream[r]);
                    if (qpos < 0) continue;
                    if (partitioned && h.key_attr[qpos] == -2) {  // one view row per range that holds, in range order
                        const auto& rs = h.key_ranges[qpos];
                        for (size_t x = 0; x < rs.size(); ++x)
                            if (range_holds(h, rs[x], qpos, *c, r, true)) vr.push_back({r, rs[x].label, (uint32_t)x, (uint8_t)qpos});
                    } else if (partitioned && h.key_attr[qpos] == -3) {  // one view row per initialised key, in order
                        if (bc_dev) {
                            uint32_t off = 0, k = 0;
                            bc_order_now(off, k);
                            ph_j.push_back((uint32_t)vr.size());
                            ph_off.push_back(off);
                            ph_k.push_back(k);
                            vr.push_back({r, BX_PLACEHOLDER, 0, (uint8_t)qpos});
                            continue;
                        }
                        const std::vector<uint32_t>& o = bcast_order();
                        for (size_t x = 0; x < o.size(); ++x) vr.push_back({r, o[x], (uint32_t)x, (uint8_t)qpos});
                    } else if (partitioned) {
                        const int ai = h.key_attr[qpos];
                        if (!c->nulls[ai].empty() && c->nulls[ai][r]) continue;  // null partition key: dropped
                        uint32_t key = 0;
                        if (!slot_key(e, q, qpos, ((const int64_t*)c->cols[ai].data())[r], &key)) continue;
                        key_seen(key);
                        vr.push_back({r, key, 0, (uint8_t)qpos});
                    } else {
                        vr.push_back({r, 0, 0, (uint8_t)qpos});
                    }
                }
                const size_t base = ts.size(), m = vr.size();
                for (size_t x = 0; x < ph_j.size(); ++x) {
                    bc_row.push_back((uint32_t)(base + ph_j[x]));
                    bc_off.push_back(ph_off[x]);
                    bc_k.push_back(ph_k[x]);
                }
                ts.resize(base + m);
                vpos.resize(base + m);
                qs.resize(base + m);
                if (partitioned) keys.resize(base + m);
                if (ranged) vrank.resize(base + m);
                for (int k = 0; k < nc; ++k) {
                    cols[k].resize((base + m) * width_of(P.col_kind[k]), 0);
                    nulls[k].resize(base + m, 0);
                }
                for (size_t j = 0; j < m; ++j) {
                    const VRow& v = vr[j];
                    const size_t row = base + j;
                    ts[row] = c->ts[v.r];
                    vpos[row] = (uint32_t)(part_pos[pi] + v.r);
                    qs[row] = v.qpos;
                    if (partitioned) keys[row] = v.key;
                    if (ranged) vrank[row] = v.rank;
                    for (int k = 0; k < nc; ++k) {
                        const int ai = h.col_attr[v.qpos][k];
                        if (ai < 0) continue;  // a column of another stream of the query: zeros, not null
                        const int w = width_of(P.col_kind[k]);
                        const int64_t sv = ((const int64_t*)c->cols[ai].data())[v.r];
                        std::memcpy(&cols[k][row * w], &sv, w);  // little endian: the slot's low bytes
                        if (!c->nulls[ai].empty() && c->nulls[ai][v.r]) {
                            nulls[k][row] = 1;
                            any_null[k] = true;
                        }
                    }
                }
                continue;
            }
            const int qpos = h.stream_pos(c->stream);
            // rows kept (null partition key: dropped), then each column appended as a whole (bulk copy when no
            // row was dropped)
            std::vector<int64_t> kept;
            bool all = true;
            const size_t base = ts.size();
            if (partitioned && h.key_attr[qpos] == -2) {  // one view row per range that holds (in range order)
                all = false;
                const auto& rs = h.key_ranges[qpos];
                for (int64_t r = 0; r < c->n; ++r)
                    for (size_t x = 0; x < rs.size(); ++x)
                        if (range_holds(h, rs[x], qpos, *c, r, false)) {
                            keys.push_back(rs[x].label);
                            kept.push_back(r);
                            vrank.push_back((uint32_t)x);
                        }
            } else if (partitioned && h.key_attr[qpos] == -3 && bc_dev) {  // one placeholder per event (one order: no
                all = false;                                                // keyed row of this chunk changes it)
                uint32_t off = 0, k = 0;
                bc_order_now(off, k);
                for (int64_t r = 0; r < c->n; ++r) {
                    bc_row.push_back((uint32_t)(base + kept.size()));
                    bc_off.push_back(off);
                    bc_k.push_back(k);
                    keys.push_back(BX_PLACEHOLDER);
                    kept.push_back(r);
                    vrank.push_back(0);
                }
            } else if (partitioned && h.key_attr[qpos] == -3) {  // one view row per initialised key (a chunk of one
                all = false;                                      // stream: the key set is the same for all its rows)
                const std::vector<uint32_t>& o = bcast_order();
                for (int64_t r = 0; r < c->n; ++r)
                    for (size_t x = 0; x < o.size(); ++x) {
                        keys.push_back(o[x]);
                        kept.push_back(r);
                        vrank.push_back((uint32_t)x);
                    }
            } else if (partitioned) {
                keys.reserve(keys.size() + (size_t)c->n);
                const uint8_t kk = h.key_kind[qpos];
                const bool do_pf = !q.string_keys && (kk == VK_I32 || kk == VK_I64);
                const uint8_t* kcol = c->cols[h.key_attr[qpos]].data();
                for (int64_t r = 0; r < c->n; ++r) {
                    if (do_pf && r + 16 < c->n)
                        q.intkeys.prefetch(kk == VK_I32 ? (int64_t)((const int32_t*)kcol)[r + 16] : ((const int64_t*)kcol)[r + 16]);
                    uint32_t key = 0;
                    if (!host_key(e, q, qpos, *c, r, &key)) {
                        if (all) {
                            all = false;
                            kept.reserve((size_t)c->n);
                            for (int64_t r2 = 0; r2 < r; ++r2) kept.push_back(r2);
                        }
                        continue;
                    }
                    keys.push_back(key);
                    key_seen(key);
                    if (!all) kept.push_back(r);
                }
            }
            const size_t m = all ? (size_t)c->n : kept.size();
            if (ranged && h.key_attr[qpos] != -2 && h.key_attr[qpos] != -3) vrank.resize(base + m, 0);
            if (all) ts.insert(ts.end(), c->ts.begin(), c->ts.begin() + c->n);
            else for (int64_t r : kept) ts.push_back(c->ts[r]);
            if (all) for (int64_t r = 0; r < c->n; ++r) vpos.push_back((uint32_t)(part_pos[pi] + r));
            else for (int64_t r : kept) vpos.push_back((uint32_t)(part_pos[pi] + r));
            qs.resize(base + m, (uint8_t)qpos);
            for (int k = 0; k < nc; ++k) {
                const int w = width_of(P.col_kind[k]);
                const int ai = h.col_attr[qpos][k];
                const size_t off = cols[k].size();
                cols[k].resize(off + m * w, 0);
                nulls[k].resize(base + m, 0);
                if (ai < 0) continue;  // a column of another stream of the query: zeros, not null
                const uint8_t* src = c->cols[ai].data();
                const bool has_nulls = !c->nulls[ai].empty();
                if (all) {
                    std::memcpy(&cols[k][off], src, m * w);
                    if (has_nulls) std::memcpy(&nulls[k][base], c->nulls[ai].data(), m);
                } else {
                    for (size_t j = 0; j < m; ++j) {
                        std::memcpy(&cols[k][off + j * w], src + kept[j] * w, w);
                        if (has_nulls) nulls[k][base + j] = c->nulls[ai][kept[j]];
                    }
                }
                if (has_nulls)
                    for (size_t j = 0; j < m && !any_null[k]; ++j) any_null[k] = nulls[k][base + j] != 0;
            }
        }
        nrows = (int64_t)ts.size();
        size_t cnt = (size_t)std::max<int64_t>(nrows, 1);
        bool identity = true;
        for (int64_t i = 0; i < nrows && identity; ++i) identity = vpos[i] == (uint32_t)(vpos[0] + i);
        if (identity) {
            pos_off = nrows ? vpos[0] : 0;
        } else {
            d_vpos = (const uint32_t*)q.d_vpos.ensure(cnt * 4);
            HIPCHECK(hipMemcpyAsync((void*)d_vpos, vpos.data(), nrows * 4, hipMemcpyHostToDevice, st));
        }
        d_ts = (const int64_t*)q.st_ts.ensure(cnt * 8);
        if (nrows) HIPCHECK(hipMemcpyAsync((void*)d_ts, ts.data(), nrows * 8, hipMemcpyHostToDevice, st));
        if (multi_stream) {
            d_qs = (const uint8_t*)q.st_qs.ensure(cnt);
            if (nrows) HIPCHECK(hipMemcpyAsync((void*)d_qs, qs.data(), nrows, hipMemcpyHostToDevice, st));
        }
        if (partitioned) {
            d_key = (const uint32_t*)q.st_key.ensure(cnt * 4);
            if (nrows) HIPCHECK(hipMemcpyAsync((void*)d_key, keys.data(), nrows * 4, hipMemcpyHostToDevice, st));
        }
        if (ranged) {
            d_vrank = (const uint32_t*)q.st_vrank.ensure(cnt * 4);
            if (nrows) HIPCHECK(hipMemcpyAsync((void*)d_vrank, vrank.data(), nrows * 4, hipMemcpyHostToDevice, st));
        }
        for (int k = 0; k < nc; ++k) {
            int w = width_of(P.col_kind[k]);
            d_cols[k] = q.st_cols[k].ensure(cnt * w);
            if (nrows) HIPCHECK(hipMemcpyAsync((void*)d_cols[k], cols[k].data(), nrows * w, hipMemcpyHostToDevice, st));
            if (any_null[k]) {
                d_nulls[k] = (const uint8_t*)q.st_nulls[k].ensure(cnt);
                HIPCHECK(hipMemcpyAsync((void*)d_nulls[k], nulls[k].data(), nrows, hipMemcpyHostToDevice, st));
            }
        }
        if (!bc_row.empty()) {  // ---- the placeholders expanded on the device (kernels.h bcast_expand)
            std::vector<uint32_t> off((size_t)nrows + 1);
            uint64_t o = 0;
            size_t ph = 0;
            int64_t kmax = 0;
            for (int64_t r = 0; r < nrows; ++r) {
                off[r] = (uint32_t)o;
                if (ph < bc_row.size() && bc_row[ph] == (uint32_t)r) {
                    o += bc_k[ph];
                    kmax = std::max<int64_t>(kmax, bc_k[ph]);
                    ++ph;
                } else {
                    o += 1;
                }
                if (o >= (uint64_t)0xFFFFFFF0) throw CompileError(SDG_ERR_CAPACITY, "a flush holds more than 2^32 - 16 view rows");
            }
            off[nrows] = (uint32_t)o;
            if (ph != bc_row.size()) throw DeviceError("broadcast placeholders out of order");
            const int64_t nx = (int64_t)o;
            const size_t cx = (size_t)std::max<int64_t>(nx, 1);
            BcastExpandArgs bx;
            std::memset(&bx, 0, sizeof bx);
            bx.n = nrows;
            uint32_t* d_off = (uint32_t*)q.bx_off.ensure(off.size() * 4);
            HIPCHECK(hipMemcpyAsync(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice, st));
            bx.off = d_off;
            bx.nph = (int64_t)bc_row.size();
            uint32_t* d_ph = (uint32_t*)q.bx_ph.ensure(3 * bc_row.size() * 4);
            HIPCHECK(hipMemcpyAsync(d_ph, bc_row.data(), bc_row.size() * 4, hipMemcpyHostToDevice, st));
            HIPCHECK(hipMemcpyAsync(d_ph + bc_row.size(), bc_off.data(), bc_row.size() * 4, hipMemcpyHostToDevice, st));
            HIPCHECK(hipMemcpyAsync(d_ph + 2 * bc_row.size(), bc_k.data(), bc_row.size() * 4, hipMemcpyHostToDevice, st));
            bx.ph_row = d_ph;
            bx.ph_ord = d_ph + bc_row.size();
            bx.ph_k = d_ph + 2 * bc_row.size();
            uint32_t* d_ord = (uint32_t*)q.bx_ord.ensure(std::max<size_t>(bc_ord.size(), 1) * 4);
            if (!bc_ord.empty()) HIPCHECK(hipMemcpyAsync(d_ord, bc_ord.data(), bc_ord.size() * 4, hipMemcpyHostToDevice, st));
            bx.ord = d_ord;
            if (!d_vpos) {  // (the compact positions were contiguous: upload them anyway, the expansion repeats them)
                d_vpos = (const uint32_t*)q.d_vpos.ensure(cnt * 4);
                HIPCHECK(hipMemcpyAsync((void*)d_vpos, vpos.data(), nrows * 4, hipMemcpyHostToDevice, st));
            }
            bx.ts = d_ts;
            bx.vpos = d_vpos;
            bx.qs = d_qs;
            bx.key = d_key;
            bx.vrank = d_vrank;
            bx.ncols = nc;
            bx.o_ts = (int64_t*)q.bx_ts.ensure(cx * 8);
            bx.o_vpos = (uint32_t*)q.bx_vpos.ensure(cx * 4);
            bx.o_qs = d_qs ? (uint8_t*)q.bx_qs.ensure(cx) : nullptr;
            bx.o_key = (uint32_t*)q.bx_key.ensure(cx * 4);
            bx.o_vrank = (uint32_t*)q.bx_vrank.ensure(cx * 4);
            for (int k = 0; k < nc; ++k) {
                bx.width[k] = (uint8_t)width_of(P.col_kind[k]);
                bx.cols[k] = d_cols[k];
                bx.nulls[k] = d_nulls[k];
                bx.o_cols[k] = q.bx_cols[k].ensure(cx * bx.width[k]);
                bx.o_nulls[k] = d_nulls[k] ? (uint8_t*)q.bx_nulls[k].ensure(cx) : nullptr;
            }
            bcast_expand(bx, kmax, st);
            d_ts = bx.o_ts;
            d_vpos = bx.o_vpos;
            pos_off = 0;
            d_qs = bx.o_qs;
            d_key = bx.o_key;
            d_vrank = bx.o_vrank;
            for (int k = 0; k < nc; ++k) {
                d_cols[k] = bx.o_cols[k];
                d_nulls[k] = bx.o_nulls[k];
            }
            nrows = nx;
        }
        // hipMemcpyAsync from pageable memory: keep the host vectors alive until the copies land
        HIPCHECK(hipStreamSynchronize(st));
    }
    // sorted positions and original rows are 32-bit on the device
    if (nrows >= (int64_t)0xFFFFFFF0) throw CompileError(SDG_ERR_CAPACITY, "a flush holds more than 2^32 - 16 events");
    uint32_t K = 1;
    if (partitioned) K = q.string_keys ? (uint32_t)std::max<size_t>(e->strings.strs.size(), 1) : (uint32_t)std::max<size_t>(q.keystr.size(), 1);
    // fused bucket path (chain.hip chain_fused_k): one radix pass into 2^bbits buckets + per-block regrouping in LDS
    // instead of the full key sort. Shapes it covers: see kernels.h; anything else (or a batch that breaks its
    // time-order precondition) runs the radix path below.
    int kbits = 0;
    while ((1ll << kbits) < (int64_t)K) ++kbits;
    bool try_fused = false;
    // (round 5: one-key batches -- an unpartitioned chain query, C1 -- take the fused matcher too: the batch is one
    // bucket of one key, so there is no bucket pass; SDG_FU_NO_ONEKEY keeps them on the lane kernels)
    static const bool no_onekey = getenv("SDG_FU_NO_ONEKEY") != nullptr;
    if (P.chain && (partitioned || !no_onekey) && !multi_stream && nrows > 0 && !e->no_fused && P.n_states == 2 &&
        P.has_within && nc >= 1 && kbits <= 16 && P.fast[0].kind != FP_NONE) {
        ChainArgs pa;
        std::memset(&pa, 0, sizeof pa);
        for (int k = 0; k < nc; ++k) pa.nulls[k] = d_nulls[k];
        pa.cin_n = q.carry[q.cur].n;
        chain_staging(h, pa, q.carry_nullable);
        const ChainSpec& ps = pa.sp;
        const bool typed = ps.scan_mode == SCAN_TRUE ||
                           ((ps.scan_mode == SCAN_CONST || ps.scan_mode == SCAN_E1) && ps.scan_col < nc && !d_nulls[ps.scan_col]);
        try_fused = !pa.generic && typed && ps.scan_col >= 0 && ps.scan_col < nc;
    }
    // sorted-view matcher (chain.hip chain_sorted_k) on the radix path: the shapes of the fused matcher without the
    // key-count limit; the carried partials fold into the key sort (their values must not be null: none of the
    // query's columns may hold nulls)
    bool sorted_now = false;
    if (P.chain && partitioned && !multi_stream && nrows > 0 && !e->no_sorted && P.n_states == 2 && nc >= 1 &&
        P.fast[0].kind != FP_NONE && !q.carry_nullable && nrows + q.carry[q.cur].n < ((int64_t)1 << 31) &&
        (int64_t)K < ((int64_t)1 << 31)) {
        ChainArgs pa;
        std::memset(&pa, 0, sizeof pa);
        bool nulls = false;
        for (int k = 0; k < nc; ++k) nulls |= d_nulls[k] != nullptr;
        chain_staging(h, pa, false);
        const ChainSpec& ps = pa.sp;
        const bool typed = ps.scan_mode == SCAN_TRUE || ps.scan_mode == SCAN_CONST || ps.scan_mode == SCAN_E1;
        sorted_now = !nulls && !pa.generic && typed && ps.scan_col >= 0 && ps.scan_col < nc;
    }
    e->stats.fused = 0;
    const bool carry_nullable0 = q.carry_nullable;
    bool sub_retry = false;  // the fused run with sub-batches failed its halo check: once more without them
    // returns false when the fused path found its precondition broken (nothing of the batch is committed then)
    auto run = [&](bool fused) -> bool {
    const bool sorted = !fused && sorted_now && P.chain;
    // sorted view rows: the batch plus the carried partials folded in as leading rows of their keys
    const int64_t nv = nrows + (sorted ? q.carry[q.cur].n : 0);
    // ---- 2. key grouping ---------------------------------------------------------------------------------
    const int64_t* v_ts = d_ts;
    const uint8_t* v_qs = d_qs;
    const uint32_t* v_vrank = d_vrank;
    const uint32_t* v_key = nullptr;
    const uint32_t* v_seg = nullptr;
    const uint32_t* v_orig = d_vpos;  // partitioned: replaced by orig_sorted (positions when d_vpos is set)
    const void* v_cols[MAX_COLS];
    const uint8_t* v_nulls[MAX_COLS];
    for (int k = 0; k < nc; ++k) { v_cols[k] = d_cols[k]; v_nulls[k] = d_nulls[k]; }
    hp.mark("view");
    ev_record(e->ev[0], st);
    const uint32_t* v_segend = nullptr;
    const uint32_t* v_ts32 = nullptr;  // fused path's slim bucket view / sorted view: ts as u32 offsets from *v_tsbase
    const int64_t* v_tsbase = d_ts;
    const uint8_t* v_lkey = nullptr;
    int* flags = (int*)q.flags.ensure(32);  // [0] output overflow [1] decreasing ts [2] bounds [3] mono [4] key range
    int bbits = 0;
    uint32_t* b_start = nullptr;
    uint32_t* b_seg = nullptr;
    uint32_t* b_tm = nullptr;
    // SDG_FU_OCOLS=1: columns the fused matcher reads only to emit stay in arrival order (the bucket pass does not
    // move them; ChainArgs::ocols). Not with view positions (orig is then not an arrival row) or nulls. Off by
    // default: on C2 the scatter gains 0.31 ms and the matcher's dependent gathers cost 0.28 ms (r5x)
    uint32_t eo_mask = 0;
    // fused sub-batches (round 6; SDG_FU_SUB = own rows per sub-batch, a multiple of the bucket tile, 0 = off): the
    // flush's bucket pass and matcher run per time sub-batch whose view (own rows + a halo past their window) stays
    // in the Infinity Cache between the scatter that writes it and the matcher that reads it
    int64_t sub_S = 0, sub_H = 0, sub_J = 0;
    KeyGroupArgs sub_kg;
    std::memset(&sub_kg, 0, sizeof sub_kg);
    uint32_t* b_own = nullptr;
    const char* oc_env = getenv("SDG_FU_OCOLS");  // (read per flush: the tests switch it)
    const bool move_all = !(oc_env && atoi(oc_env) == 1);
    if (fused && partitioned && !d_vpos && !move_all && !getenv("SDG_FU_WIDE")) {
        ChainArgs ta;
        std::memset(&ta, 0, sizeof ta);
        for (int k = 0; k < nc; ++k) ta.nulls[k] = d_nulls[k];
        chain_staging(h, ta, q.carry_nullable);
        auto filt = [&](int k) {
            for (int i = 0; i < std::min(P.n_states, 2); ++i) {
                const FastPred& f = P.fast[i];
                if ((f.kind == FP_CONST || f.kind == FP_SLOT) && f.ca == k) return true;
                if (f.kind == FP_SLOT && f.cb == k) return true;
            }
            return false;
        };
        for (int k = 0; k < nc && k < 32 && chain_fused_ocols_ok(ta); ++k)
            if (!d_nulls[k] && !filt(k) && k != ta.sp.scan_col && !(ta.sp.scan_mode == SCAN_E1 && k == ta.sp.e1_col))
                eo_mask |= 1u << k;
    }
    if (partitioned && nrows > 0) {
        KeyGroupArgs a;
        std::memset(&a, 0, sizeof a);
        a.ts32_col = -1;
        a.n = nv;
        a.K = (int32_t)K;
        a.keys = d_key;
        a.key_flag = zero_copy ? flags + 4 : nullptr;  // caller-supplied device ids: range-check against K
        a.orig_in = d_vpos;                            // orig_sorted: view rows (+ pos_off), or positions
        int c = 0;
        // the register sequence kernel reads ts only for its output rows: gathered through orig (view rows) from the
        // arrival-order column instead of moved by every radix pass (a quarter of C3's sort traffic)
        const bool ts_by_orig = q.seq3 && !fused && !d_vpos && !P.has_within;
        if (ts_by_orig) {
            v_ts = nullptr;
        } else {
            a.src[c] = d_ts; a.dst[c] = q.so_ts.ensure(nv * 8); a.width[c] = 8; v_ts = (const int64_t*)a.dst[c]; ++c;
        }
        if (d_qs) { a.src[c] = d_qs; a.dst[c] = q.so_qs.ensure(nrows); a.width[c] = 1; v_qs = (const uint8_t*)a.dst[c]; ++c; }
        if (d_vrank) { a.src[c] = d_vrank; a.dst[c] = q.so_vrank.ensure(nrows * 4); a.width[c] = 4; v_vrank = (const uint32_t*)a.dst[c]; ++c; }
        for (int k = 0; k < nc; ++k) {
            if ((eo_mask >> k) & 1u) continue;  // stays in arrival order (v_cols[k] = d_cols[k])
            if (c >= MAX_COLS + 2) throw CompileError(SDG_ERR_UNSUPPORTED, "too many columns");
            int w = width_of(P.col_kind[k]);
            a.src[c] = d_cols[k]; a.dst[c] = q.so_cols[k].ensure(nv * w); a.width[c] = (uint8_t)w;
            v_cols[k] = a.dst[c];
            ++c;
            if (d_nulls[k]) {
                a.src[c] = d_nulls[k]; a.dst[c] = q.so_nulls[k].ensure(nrows); a.width[c] = 1;
                v_nulls[k] = (const uint8_t*)a.dst[c];
                ++c;
            }
        }
        a.ncols = c;
        if (sorted && q.carry[q.cur].n > 0) {  // the carried partials as prefix rows (ts, then each column's slots)
            const QueryRt::Carry& ci = q.carry[q.cur];
            a.pre_n = ci.n;
            a.pre_keys = ci.key.as<uint32_t>();
            a.pre_src[0] = ci.ts.p;
            for (int k = 0; k < nc; ++k) a.pre_src[1 + k] = ci.vals.as<int64_t>() + (size_t)k * ci.cap;
        }
        a.no_segments = sorted;
        // the sorted view moves ts as u32 offsets from ts[0] - 2^31 (a row outside that window sets flags[3]: the
        // batch reruns on the lane kernels); SDG_SV_WIDE keeps int64 ts (A/B)
        static const bool sv_wide = getenv("SDG_SV_WIDE") != nullptr;
        const bool sv32 = sorted && !sv_wide && !ts_by_orig;
        if (sv32) {
            int64_t* base = (int64_t*)q.sv_tsbase.ensure(8);
            ts_window_base(d_ts, base, st);
            a.ts32_col = 0;  // (ts is payload column 0)
            a.ts_base = base;
            a.ts32_flag = flags + 3;
            v_tsbase = base;
        }
        keygroup_bind(a, q.kg_counts.ensure(keygroup_workspace(nv, (int32_t)K, a.ncols, a.width)));
        a.keys_sorted = (uint32_t*)q.so_key.ensure(nv * 4);
        a.orig_sorted = (uint32_t*)q.so_orig.ensure(nv * 4);
        a.seg_start = (uint32_t*)q.seg.ensure((size_t)K * 4);
        a.seg_end = (uint32_t*)q.kg_gsum.ensure((size_t)K * 4);
        if (fused) {
            bbits = std::max(1, std::min(8, kbits));
            b_start = (uint32_t*)q.bk_plan.ensure(2 * 257 * 4);
            b_seg = b_start + 257;
            HIPCHECK(hipMemsetAsync(flags, 0, 32, st));
            // the slim bucket view: ts as u32 offsets from the batch's first ts, keys as u8 local keys (the matcher
            // regroups by them; the bucket is the range a row lies in)
            static const bool wide = getenv("SDG_FU_WIDE") != nullptr;  // A/B: int64 ts + u32 keys
            if (!wide) {
                a.ts32_col = 0;
                a.ts_base = d_ts;
                a.lkey_out = (uint8_t*)q.so_lkey.ensure(nrows);
            }
            // time-major block order (SDG_FU_BMAJOR: bucket-major, A/B)
            static const bool bmajor = getenv("SDG_FU_BMAJOR") != nullptr;
            const int64_t tm_cap = chain_fused_grid(nrows, 1 << bbits) + 2;
            if (!bmajor && eo_mask) b_tm = (uint32_t*)q.bk_tm.ensure((size_t)tm_cap * 4);
            // sub-batches: the own rows per sub-batch (a multiple of the bucket tile) and a halo sized from the
            // batch's mean event rate (1.25 x the rows of one window + 2 tiles; checked on the device: a too short
            // halo reruns the flush without sub-batches)
            const char* sub_env = getenv("SDG_FU_SUB");  // (read per flush: the tests switch it)
            const int64_t tile = bucket_tile();
            int64_t S = sub_env ? atoll(sub_env) : 0;
            S = S > 0 ? (S + tile - 1) / tile * tile : 0;
            if (S > 0 && !q.no_sub && !sub_retry && !wide && !eo_mask && !d_vpos && !d_qs && !d_vrank && P.has_within &&
                nrows > S && !sorted) {
                int64_t te[2];
                HIPCHECK(hipMemcpyAsync(&te[0], d_ts, 8, hipMemcpyDeviceToHost, st));
                HIPCHECK(hipMemcpyAsync(&te[1], d_ts + nrows - 1, 8, hipMemcpyDeviceToHost, st));
                HIPCHECK(hipStreamSynchronize(st));
                const double span = (double)std::max<int64_t>(te[1] - te[0], 1);
                const double win_rows = (double)nrows / span * (double)(P.within_ms + 1);
                int64_t H = (int64_t)(win_rows * 1.25) + 2 * tile;
                H = (H + tile - 1) / tile * tile;
                if (te[1] >= te[0] && H <= S / 2) {
                    sub_S = S;
                    sub_H = H;
                    sub_J = (nrows + S - 1) / S;
                }
            }
            if (sub_J > 1) {  // the view holds one sub-batch: S + H rows (the buffers above are reused from row 0)
                sub_kg = a;
                b_own = (uint32_t*)q.bk_own.ensure(257 * 4);
                sub_halo_check(d_ts, nrows, sub_S, sub_H, P.within_ms, flags, st);
            } else {
                bucketize(a, bbits, 0 /* ts is payload column 0 */, flags + 3, b_start, b_seg, FU_OWN, st,
                          g_no_events ? nullptr : &e->ev[4], b_tm, b_tm ? tm_cap : 0);
            }
            if (!wide) {
                v_ts32 = (const uint32_t*)a.dst[0];
                v_lkey = a.lkey_out;
                v_ts = nullptr;
            }
            if (getenv("SDG_DEBUG")) {  // validate the bucket plan on the host before the matcher reads it
                std::vector<uint32_t> hp(2 * 257);
                HIPCHECK(hipMemcpyAsync(hp.data(), b_start, 2 * 257 * 4, hipMemcpyDeviceToHost, st));
                HIPCHECK(hipStreamSynchronize(st));
                const int nbk = 1 << bbits;
                bool okp = hp[nbk] == (uint32_t)nrows && hp[257 + nbk] <= (uint32_t)chain_fused_grid(nrows, nbk);
                for (int d = 0; d < nbk; ++d) okp = okp && hp[d] <= hp[d + 1] && hp[257 + d] <= hp[257 + d + 1];
                if (!okp) throw DeviceError("fused bucket plan inconsistent (n=" + std::to_string(nrows) + ")");
            }
        } else {
            HIPCHECK(hipMemsetAsync(flags, 0, 32, st));
            keygroup(a, st, g_no_events ? nullptr : &e->ev[4]);
            if (a.ts32_col >= 0) {
                v_ts32 = (const uint32_t*)a.dst[0];
                v_ts = nullptr;
            }
        }
        v_key = v_lkey ? nullptr : a.keys_sorted;
        v_seg = a.seg_start;
        v_segend = a.seg_end;
        v_orig = a.orig_sorted;
        e->stats.keygroup_launches += 1;
    } else if (partitioned) {
        v_seg = (const uint32_t*)q.seg.ensure((size_t)K * 4);
        v_segend = (const uint32_t*)q.kg_gsum.ensure((size_t)K * 4);
        HIPCHECK(hipMemsetAsync((void*)v_seg, 0, (size_t)K * 4, st));
        HIPCHECK(hipMemsetAsync((void*)v_segend, 0, (size_t)K * 4, st));
    } else if (fused && nrows > 0) {  // one key: the batch is one bucket in arrival order; its segment plan here
        bbits = 0;
        b_start = (uint32_t*)q.bk_plan.ensure(2 * 257 * 4);
        b_seg = b_start + 257;
        uint32_t* hp2 = (uint32_t*)q.h_ret.ensure(64);
        hp2[0] = 0;
        hp2[1] = (uint32_t)nrows;
        hp2[2] = 0;
        hp2[3] = (uint32_t)((nrows + FU_ROWS / 2 - 1) / (FU_ROWS / 2));
        HIPCHECK(hipMemcpyAsync(b_start, hp2, 8, hipMemcpyHostToDevice, st));
        HIPCHECK(hipMemcpyAsync(b_seg, hp2 + 2, 8, hipMemcpyHostToDevice, st));
        HIPCHECK(hipMemsetAsync(flags, 0, 32, st));
        HIPCHECK(hipStreamSynchronize(st));  // (hp2 is reused for the run's read-backs)
    }
    hp.mark("keygroup_enqueue");
    ev_record(e->ev[1], st);
    if (!P.chain && q.seq3) {
        // ---- register sequence kernel (seq3.hip): per-key state grows to K keys (zeros: no partial) -------------
        const int64_t KK = partitioned ? (int64_t)K : 1;
        const int s3nc = q.s3.nc;
        if (q.s3_kcap < KK) {
            const int64_t nk = std::max<int64_t>(KK, q.s3_kcap + q.s3_kcap / 2);
            auto grow = [&](DevBuf& buf, int64_t per, int groups) {  // SoA: each of `groups` fields re-strided
                DevBuf nb;
                nb.ensure((size_t)(nk * per * groups));
                HIPCHECK(hipMemsetAsync(nb.p, 0, (size_t)(nk * per * groups), st));
                for (int g = 0; g < groups && q.s3_kcap > 0; ++g)
                    HIPCHECK(hipMemcpyAsync((uint8_t*)nb.p + g * nk * per, (const uint8_t*)buf.p + g * q.s3_kcap * per,
                                            (size_t)(q.s3_kcap * per), hipMemcpyDeviceToDevice, st));
                HIPCHECK(hipStreamSynchronize(st));
                std::swap(nb.p, buf.p);
                std::swap(nb.cap, buf.cap);
            };
            grow(q.s3_hdr, 4, 1);
            grow(q.s3_pn, 4, 1);
            grow(q.s3_qn, 4, 1);
            grow(q.s3_vals, 8, 6 * s3nc);
            grow(q.s3_ts, 8, 2);
            q.s3_kcap = nk;
        }
        Seq3Args a;
        std::memset(&a, 0, sizeof a);
        a.sp = q.s3;
        a.n = nrows;
        a.ts = v_ts;
        a.ts_view = d_ts;  // v_ts == nullptr: output ts = ts_view[orig[r]]
        a.seg_start = partitioned ? v_seg : nullptr;
        a.seg_end = partitioned ? v_segend : nullptr;
        a.K = (int32_t)KK;
        // emission position = seq_base + (orig ? orig[r] : r): orig holds view rows unless d_vpos mapped them
        a.orig = v_orig;
        a.pos_off = 0;
        a.seq_base = e->seq + (d_vpos ? 0 : pos_off);
        for (int k = 0; k < nc; ++k) { a.cols[k] = v_cols[k]; a.nulls[k] = v_nulls[k]; }
        a.st_hdr = q.s3_hdr.as<uint32_t>();
        a.st_pn = q.s3_pn.as<uint32_t>();
        a.st_qn = q.s3_qn.as<uint32_t>();
        a.st_vals = q.s3_vals.as<int64_t>();
        a.st_ts = q.s3_ts.as<int64_t>();
        a.kcap = q.s3_kcap;
        // at most one match per event: nrows records never overflow (no rerun, so the state updates in place)
        const int64_t cap = std::max<int64_t>(q.out_cap, nrows + 64);
        q.out_cap = cap;
        a.out_cap = cap;
        unsigned long long* counters = (unsigned long long*)q.counters.ensure(16);
        HIPCHECK(hipMemsetAsync(counters, 0, 16, st));
        if (!(partitioned && nrows > 0)) HIPCHECK(hipMemsetAsync(flags, 0, 32, st));
        a.out_count = counters;
        a.flags = flags;
        a.out_ts = (int64_t*)q.o_ts.ensure(cap * 8);
        a.out_key = (uint32_t*)q.o_key.ensure(cap * 4);
        a.out_vals = (int64_t*)q.o_vals.ensure((size_t)std::max(P.n_out, 1) * cap * 8);
        a.out_nulls = (uint32_t*)q.o_nulls.ensure(cap * 4);
        a.out_emit_seq = (int64_t*)q.o_emit.ensure(cap * 8);
        a.out_sub = (int64_t*)q.o_first.ensure(cap * 8);
        Seq3Args* h_a = (Seq3Args*)q.h_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));
        Seq3Args* d_a = (Seq3Args*)q.d_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));
        static_assert(sizeof(Seq3Args) <= 2 * sizeof(ChainArgs), "seq3 arguments fit the argument staging");
        *h_a = a;
        HIPCHECK(hipMemcpyAsync(d_a, h_a, sizeof(Seq3Args), hipMemcpyHostToDevice, st));
        ev_record(e->ev[8], st);
        seq3_run(a, d_a, st);
        ev_record(e->ev[2], st);
        unsigned long long hc = 0;
        int hf[8];
        HIPCHECK(hipMemcpyAsync(&hc, counters, 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(hf, flags, 32, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        if (hf[4]) throw CompileError(SDG_ERR_ARG, "device-resident partition key ids out of range (not from sdg_intern)");
        if (hf[0] || (int64_t)hc > cap) throw DeviceError("seq3: more matches than events (internal error)");
        e->stats.match_launches += 1;
        q.last_timers = false;
        q.last_rank.clear();
        q.taken.clear();
        q.reordered.clear();
        q.runs.clear();
        q.last_seq_base = e->seq;
        q.emit_base = e->seq;
        q.emit_span = e->flush_G;
        q.sub_is_seq = false;
        float ms_kg = 0, ms_m = 0, t;
        ev_elapsed(&ms_kg, e->ev[0], e->ev[1]);
        ev_elapsed(&ms_m, e->ev[1], e->ev[2]);
        e->stats.ms_keygroup += ms_kg;
        e->stats.ms_match += ms_m;
        if (partitioned && nrows > 0) {
            ev_elapsed(&t, e->ev[4], e->ev[5]);
            e->stats.ms_kg_hist += t;
            ev_elapsed(&t, e->ev[6], e->ev[7]);
            e->stats.ms_kg_prefix += t;
            ev_elapsed(&t, e->ev[5], e->ev[6]);
            e->stats.ms_kg_scatter += t;
        }
        ev_elapsed(&t, e->ev[8], e->ev[2]);
        e->stats.ms_nfa += t;
        e->stats.ms_nfa_kernel += t;
        e->stats.events += nrows;
        q.out_n = (int64_t)hc;
        q.polled = false;
        q.nulls_valid = true;
        e->stats.matches += q.out_n;
        e->stats.path = 2;
        return true;
    }
    if (!P.chain) {
        NfaArgs a;
        std::memset(&a, 0, sizeof a);
        a.plan = q.d_plan.as<Plan>();
        a.code = q.d_code.as<Instr>();
        a.consts = q.d_consts.as<int64_t>();
        a.n = nrows;
        a.ts = v_ts;
        a.qstream = multi_stream ? v_qs : nullptr;
        a.vrank = v_vrank;
        a.seg_start = partitioned ? v_seg : nullptr;
        a.seg_end = partitioned ? v_segend : nullptr;
        a.K = partitioned ? (int32_t)K : 1;
        a.orig = v_orig;
        a.pos_off = d_vpos ? 0 : pos_off;
        for (int k = 0; k < nc; ++k) { a.cols[k] = v_cols[k]; a.nulls[k] = v_nulls[k]; }
        a.seq_base = e->seq;
        const bool timers = P.n_sched > 0;
        // arenas: grow to K keys keeping the existing keys' state, new keys zeroed (= not yet initialised); two
        // copies + the per-key committed-copy bit, so a key can be rerun from its batch-start state (scheduler
        // reruns, arena growth)
        const int64_t kb = q.L.bytes;
        const int ib = nfa::idle_bytes(P.n_states);
        auto slot_pool = [&]() {
            SlotPool sp;
            sp.slot_of = q.slot_of.as<int32_t>();
            sp.idle_rec = q.idle_rec.as<uint8_t>();
            sp.slot_key = q.slot_key.as<int32_t>();
            sp.init_from = q.init_from.as<uint8_t>();
            sp.releasable = q.releasable.as<uint8_t>();
            sp.idle_out = q.idle_out.as<uint8_t>();
            sp.free_slots = q.free_slots.as<int32_t>();
            sp.counters = (unsigned int*)q.pool_ctr.ensure(16);
            sp.idle_bytes = ib;
            return sp;
        };
        auto regrow = [&](DevBuf& buf, int64_t old_n, int64_t new_n, int64_t per, int fill) {
            DevBuf nb;
            nb.ensure((size_t)std::max<int64_t>(new_n * per, 8));
            HIPCHECK(hipMemsetAsync(nb.p, fill, (size_t)(new_n * per), st));
            if (old_n) HIPCHECK(hipMemcpyAsync(nb.p, buf.p, (size_t)(old_n * per), hipMemcpyDeviceToDevice, st));
            HIPCHECK(hipStreamSynchronize(st));
            std::swap(nb.p, buf.p);
            std::swap(nb.cap, buf.cap);
        };
        if (q.reclaim) {
            // the key map covers every key; slots go to the keys with rows in this batch that have none
            if (q.map_keys < a.K) {
                const int64_t nk = std::max<int64_t>(a.K, q.map_keys + q.map_keys / 2);
                regrow(q.slot_of, q.map_keys, nk, 4, 0xFF);  // -1: never seen
                regrow(q.idle_rec, q.map_keys, nk, ib, 0);
                q.map_keys = nk;
            }
            SlotPool sp = slot_pool();
            if (q.arena_keys == 0) HIPCHECK(hipMemsetAsync(sp.counters, 0, 16, st));
            HIPCHECK(hipMemsetAsync(sp.counters + 1, 0, 4, st));
            nfa_slots_need(sp, partitioned ? v_seg : nullptr, partitioned ? v_segend : nullptr, a.K, st);
            unsigned int* hc2 = (unsigned int*)q.pool_ret.ensure(16);
            HIPCHECK(hipMemcpyAsync(hc2, sp.counters, 8, hipMemcpyDeviceToHost, st));
            HIPCHECK(hipStreamSynchronize(st));
            const int64_t top = hc2[0], need = hc2[1];
            if (need > top) {  // grow the pool: the new slots onto the free stack
                const int64_t old_n = q.arena_keys;
                const int64_t nn = std::max<int64_t>(2 * old_n, old_n + (need - top) + (need - top) / 4 + 1024);
                regrow(q.arena, old_n, nn, kb, 0);
                regrow(q.arena2, old_n, nn, kb, 0);
                regrow(q.cur_bits, old_n, nn, 1, 0);
                regrow(q.ran_bits, old_n, nn, 1, 0);
                regrow(q.init_from, old_n, nn, 1, 0);
                regrow(q.releasable, old_n, nn, 1, 0);
                regrow(q.slot_key, old_n, nn, 4, 0);
                regrow(q.free_slots, old_n, nn, 4, 0);
                q.idle_out.ensure((size_t)nn * ib);
                std::vector<int32_t> ids(nn - old_n);
                for (int64_t i = 0; i < nn - old_n; ++i) ids[i] = (int32_t)(old_n + i);
                HIPCHECK(hipMemcpy(q.free_slots.as<int32_t>() + top, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
                const unsigned int ntop = (unsigned int)(top + (nn - old_n));
                HIPCHECK(hipMemcpy(sp.counters, &ntop, 4, hipMemcpyHostToDevice));
                q.arena_keys = nn;
                sp = slot_pool();
            }
            nfa_slots_assign(sp, partitioned ? v_seg : nullptr, partitioned ? v_segend : nullptr, a.K, st);
            a.slot_of = sp.slot_of;
            a.init_from = sp.init_from;
            a.idle_rec = sp.idle_rec;
            a.idle_out = sp.idle_out;
            a.releasable = sp.releasable;
            a.idle_bytes = ib;
        } else if (q.arena_keys < a.K) {
            int64_t nk = std::max<int64_t>(a.K, q.arena_keys + q.arena_keys / 2);
            auto grow = [&](DevBuf& buf, int64_t per) {
                DevBuf nb;
                nb.ensure((size_t)(nk * per));
                HIPCHECK(hipMemsetAsync(nb.p, 0, (size_t)(nk * per), st));
                if (q.arena_keys) HIPCHECK(hipMemcpyAsync(nb.p, buf.p, (size_t)(q.arena_keys * per), hipMemcpyDeviceToDevice, st));
                HIPCHECK(hipStreamSynchronize(st));
                std::swap(nb.p, buf.p);
                std::swap(nb.cap, buf.cap);
            };
            grow(q.arena, kb);
            grow(q.arena2, kb);
            grow(q.cur_bits, 1);
            grow(q.ran_bits, 1);
            if (P.purge) grow(q.last_seen, 8);
            q.arena_keys = nk;
        }
        a.arena = q.arena.as<uint8_t>();
        a.arena2 = q.arena2.as<uint8_t>();
        a.cur = q.cur_bits.as<uint8_t>();
        a.ran = q.ran_bits.as<uint8_t>();
        // a key ran out of partial-match slots: every key's committed state into a layout with twice the slots
        // (the batch then reruns from its start)
        auto grow_slots = [&]() {
            const nfa::Layout Ln = nfa::make_layout(P.n_states, std::max(P.n_cols, 1), std::min(2 * q.L.ns, 4096), P.n_sched);
            DevBuf na, na2;
            na.ensure((size_t)(q.arena_keys * Ln.bytes));
            na2.ensure((size_t)(q.arena_keys * Ln.bytes));
            nfa_migrate(q.d_plan.as<Plan>(), q.arena.as<uint8_t>(), q.arena2.as<uint8_t>(), q.cur_bits.as<uint8_t>(), q.L,
                        na.as<uint8_t>(), Ln, q.arena_keys, st);
            HIPCHECK(hipMemsetAsync(q.cur_bits.p, 0, (size_t)q.arena_keys, st));
            HIPCHECK(hipMemsetAsync(q.ran_bits.p, 0, (size_t)q.arena_keys, st));
            HIPCHECK(hipStreamSynchronize(st));
            std::swap(na.p, q.arena.p);
            std::swap(na.cap, q.arena.cap);
            std::swap(na2.p, q.arena2.p);
            std::swap(na2.cap, q.arena2.cap);
            q.L = Ln;
            a.L = Ln;
            a.arena = q.arena.as<uint8_t>();
            a.arena2 = q.arena2.as<uint8_t>();
            e->stats.arena_growths += 1;
        };
        if (timers) {
            a.T.G = e->bc.G;
            a.T.clk = e->d_clk.as<int64_t>();
            a.T.nadv = e->d_nadv.as<uint32_t>();
            a.T.clock0 = e->bc.clock0;
            a.T.live = !P.playback;
            if (q.log_cap < 1024) q.log_cap = std::max<int64_t>(1024, 4 * nrows + 1024);
            a.T.log = (nfa::SchedLog*)q.d_log.ensure((size_t)q.log_cap * sizeof(nfa::SchedLog));
            a.T.log_cap = q.log_cap;
        }
        a.L = q.L;
        if (P.purge) {  // every run (first, reruns) reads the batch-start readings and writes the run's
            a.last_seen = q.last_seen.as<int64_t>();
            a.purge_clk = e->d_clk.as<int64_t>();
            a.purge_from = q.purge_first == INT64_MIN ? INT64_MAX : q.purge_first + P.purge_interval_ms;
            a.purge_idle = P.purge_idle_ms;
            HIPCHECK(hipMemcpyAsync(q.last_seen_bak.ensure((size_t)q.arena_keys * 8), q.last_seen.p, (size_t)q.arena_keys * 8,
                                    hipMemcpyDeviceToDevice, st));
            a.last_seen_in = q.last_seen_bak.as<int64_t>();
        }
        q.purge_agg = P.purge && P.n_agg > 0;
        if (q.purge_agg) a.agg_reset = (uint8_t*)q.agg_reset_flags.ensure((size_t)q.arena_keys);
        if (q.replay_carries) replay_carries(e, q, a, multi_stream);
        int64_t cap = std::max<int64_t>(q.out_cap, 2 * nrows + 4096);
        unsigned long long* counters = (unsigned long long*)q.counters.ensure(16);
        if (timers) a.T.log_count = counters + 1;
        a.flags = flags;
        a.out_count = counters;
        NfaArgs* h_na = (NfaArgs*)q.h_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));
        NfaArgs* d_na = (NfaArgs*)q.d_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));
        auto bind_out = [&]() {
            q.out_cap = cap;
            a.out_cap = cap;
            a.out_ts = (int64_t*)q.o_ts.ensure(cap * 8);
            a.out_key = (uint32_t*)q.o_key.ensure(cap * 4);
            a.out_vals = (int64_t*)q.o_vals.ensure((size_t)std::max(P.n_out, 1) * cap * 8);
            a.out_nulls = (uint32_t*)q.o_nulls.ensure(cap * 4);
            a.out_emit_seq = (int64_t*)q.o_emit.ensure(cap * 8);
            a.out_sub = (int64_t*)q.o_first.ensure(cap * 8);
            a.out_round = timers ? (uint8_t*)q.o_round.ensure(cap) : nullptr;
            a.out_flags = q.purge_agg ? (uint8_t*)q.o_flags.ensure(cap) : nullptr;
        };
        int hf[8];
        unsigned long long hc[2];
        // keys past the largest device layout go on on the host (QueryRt::spill); queries with timers (the
        // scheduler simulation owns their host runs) or @purge aggregators (per-record reset flags) still refuse
        const bool can_spill = !timers && !q.purge_agg;
        constexpr int32_t OVF_CAP = 4096;
        std::vector<uint32_t> spill_new;  // keys whose run overflowed the largest layout in this flush (sorted)
        if (can_spill) {
            uint32_t* ob = (uint32_t*)q.d_ovf.ensure((size_t)(OVF_CAP + 1) * 4);
            a.ovf_count = (unsigned int*)ob;
            a.ovf_keys = ob + 1;
            a.ovf_cap = OVF_CAP;
        }
        // one launch; returns false when a growable buffer (outputs, scheduler log) overflowed
        auto launch = [&](bool first) -> bool {
            if (a.ovf_count) HIPCHECK(hipMemsetAsync(a.ovf_count, 0, 4, st));
            if (first && q.purge_agg) HIPCHECK(hipMemsetAsync(a.agg_reset, 0, (size_t)q.arena_keys, st));
            if (first) {
                HIPCHECK(hipMemsetAsync(counters, 0, 16, st));
                if (!(partitioned && nrows > 0)) HIPCHECK(hipMemsetAsync(flags, 0, 32, st));
                else HIPCHECK(hipMemsetAsync(flags + 5, 0, 4, st));
            } else {
                HIPCHECK(hipMemsetAsync(counters + 1, 0, 8, st));  // log records of this rerun only
            }
            *h_na = a;
            HIPCHECK(hipMemcpyAsync(d_na, h_na, sizeof(NfaArgs), hipMemcpyHostToDevice, st));
            ev_record(e->ev[10], st);
            nfa_run(a, d_na, st);
            ev_record(e->ev[11], st);
            HIPCHECK(hipMemcpyAsync(hc, counters, 16, hipMemcpyDeviceToHost, st));
            HIPCHECK(hipMemcpyAsync(hf, flags, 32, hipMemcpyDeviceToHost, st));
            HIPCHECK(hipStreamSynchronize(st));
            float kms = 0;
            ev_elapsed(&kms, e->ev[10], e->ev[11]);
            e->stats.ms_nfa_kernel += kms;
            if (hf[4]) throw CompileError(SDG_ERR_ARG, "device-resident partition key ids out of range (not from sdg_intern)");
            if (hf[2] && q.L.ns < 4096) {  // grow the arenas and rerun (state is double-buffered)
                grow_slots();
                HIPCHECK(hipMemsetAsync(flags, 0, 32, st));
                return false;
            }
            spill_new.clear();
            if (hf[2] && can_spill) {  // the keys that overflowed: the host takes them over (spill_keys below)
                unsigned int no = 0;
                HIPCHECK(hipMemcpy(&no, a.ovf_count, 4, hipMemcpyDeviceToHost));
                if (no == 0 || no > (unsigned)OVF_CAP)
                    throw CompileError(SDG_ERR_CAPACITY, "query '" + h.name + "': " + std::to_string(no) + " partition keys "
                                                             "exceeded " + std::to_string(q.L.ns) + " live partial matches "
                                                             "in one flush (at most " + std::to_string(OVF_CAP) +
                                                             " can move to the host at once)");
                spill_new.resize(no);
                HIPCHECK(hipMemcpy(spill_new.data(), a.ovf_keys, (size_t)no * 4, hipMemcpyDeviceToHost));
                std::sort(spill_new.begin(), spill_new.end());
                spill_new.erase(std::unique(spill_new.begin(), spill_new.end()), spill_new.end());
                HIPCHECK(hipMemsetAsync(flags + 2, 0, 4, st));
            } else if (hf[2]) {
                e->stats.overflow += 1;
                throw CompileError(SDG_ERR_CAPACITY, "query '" + h.name + "': a partition key exceeded max_partials (" +
                                                         std::to_string(q.L.ns) + " live partial matches, or as many queued "
                                                         "timers); raise sdg_opts.max_partials");
            }
            bool ok = true;
            if (hf[0] || (int64_t)hc[0] > cap) {  // outputs: grow to what was asked for, run the batch again
                cap = std::max<int64_t>(2 * cap, (int64_t)hc[0] + 4096);
                ok = false;
            }
            if (timers && (hf[5] || (int64_t)hc[1] > q.log_cap)) {
                q.log_cap = std::max<int64_t>(2 * q.log_cap, (int64_t)hc[1] + 1024);
                a.T.log = (nfa::SchedLog*)q.d_log.ensure((size_t)q.log_cap * sizeof(nfa::SchedLog));
                a.T.log_cap = q.log_cap;
                ok = false;
            }
            if (!ok) {
                bind_out();
                HIPCHECK(hipMemsetAsync(flags, 0, 4, st));
                HIPCHECK(hipMemsetAsync(flags + 5, 0, 4, st));
            }
            return ok;
        };
        bind_out();
        ev_record(e->ev[8], st);
        auto first_run = [&]() {
            a.list = nullptr;
            a.nlist = 0;
            a.round = 0;
            for (int tries = 0; !launch(true); ++tries)  // state is double-buffered: a retry starts from the batch start
                if (tries > 24) throw CompileError(SDG_ERR_CAPACITY, "query '" + h.name + "': output buffers keep overflowing");
            e->stats.match_launches += 1;
        };
        first_run();
        q.last_timers = timers;
        q.last_rank.clear();
        q.taken.clear();
        q.reordered.clear();
        q.runs.clear();
        q.last_seq_base = e->seq;
        q.emit_base = e->seq;
        q.emit_span = e->flush_G;
        q.sub_is_seq = false;
        q.spill_runs.clear();
        if (can_spill && (!spill_new.empty() || !q.spill.empty())) {
            spill_keys(e, q, spill_new, SpillView{v_ts, multi_stream ? v_qs : nullptr, v_vrank, v_orig, a.pos_off,
                                                  partitioned ? v_seg : nullptr, partitioned ? v_segend : nullptr,
                                                  partitioned ? (int64_t)K : 1, nrows, v_cols, v_nulls, nc},
                       a.T, a.purge_from, a.purge_idle);
            q.taken = spill_new;  // their device records of this flush are void (the host runs replace them)
        }
        if (timers) {
            const auto t_sched = std::chrono::steady_clock::now();
            double k_before = e->stats.ms_nfa_kernel;
            // the global scheduler (sched.h) over the runs' logs, in two passes: an optimistic one lists the keys
            // whose fires it orders differently from their own runs, which rerun on the device with its fire order
            // (round 1); the exact pass then checks every key and replays on the host, from its batch-start state,
            // what still differs (their results replace the device's)
            std::vector<nfa::SchedLog> logs;
            auto read_logs = [&](bool keep_unlisted) {
                std::vector<nfa::SchedLog> nl(hc[1]);
                if (hc[1]) HIPCHECK(hipMemcpy(nl.data(), a.T.log, hc[1] * sizeof(nfa::SchedLog), hipMemcpyDeviceToHost));
                if (keep_unlisted) {  // the first run's records of the keys that were not rerun
                    uint32_t km = 0;
                    for (uint32_t k : q.reordered) km = std::max(km, k);
                    std::vector<uint8_t> rerun((size_t)km + 1, 0);  // (a flag per key, not a search per record)
                    for (uint32_t k : q.reordered) rerun[k] = 1;
                    nl.reserve(nl.size() + logs.size());
                    for (const nfa::SchedLog& r : logs)
                        if (r.key > km || !rerun[r.key]) nl.push_back(r);
                }
                // by (key, kseq): a stable counting sort by key (a lane appends its key's records in order); a key
                // whose records came out of order is sorted by kseq
                uint32_t kmax = 0;
                for (const nfa::SchedLog& r : nl) kmax = std::max(kmax, r.key);
                std::vector<uint32_t> cnt(nl.empty() ? 1 : (size_t)kmax + 2, 0);
                for (const nfa::SchedLog& r : nl) ++cnt[r.key + 1];
                for (size_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
                logs.resize(nl.size());
                for (const nfa::SchedLog& r : nl) logs[cnt[r.key]++] = r;
                for (size_t i = 0; i < logs.size();) {
                    size_t j = i + 1;
                    bool sorted = true;
                    for (; j < logs.size() && logs[j].key == logs[i].key; ++j) sorted &= logs[j - 1].kseq < logs[j].kseq;
                    if (!sorted)
                        std::sort(logs.begin() + i, logs.begin() + j,
                                  [](const nfa::SchedLog& x, const nfa::SchedLog& y) { return x.kseq < y.kseq; });
                    i = j;
                }
            };
            hp.mark("sched_first_run");
            read_logs(false);
            hp.mark("sched_read_logs");
            while ((int64_t)q.key_hash.size() < (int64_t)K) {  // HashMap hash of each key's toString
                const size_t k = q.key_hash.size();
                const std::string& ks = q.string_keys ? e->strings.strs[k] : q.keystr[k];
                q.key_hash.push_back(java_spread_hash(ks));
            }
            // the batch's rows by key, on the host: segments + positions (sorted view)
            const int64_t KR = partitioned ? (int64_t)K : 1;
            std::vector<uint32_t> hseg_b(KR, 0), hseg_e(KR, 0), horig;
            if (partitioned && nrows > 0) {
                HIPCHECK(hipMemcpy(hseg_b.data(), v_seg, KR * 4, hipMemcpyDeviceToHost));
                HIPCHECK(hipMemcpy(hseg_e.data(), v_segend, KR * 4, hipMemcpyDeviceToHost));
            } else if (!partitioned) {
                hseg_e[0] = (uint32_t)nrows;
            }
            if (v_orig && nrows > 0) {
                horig.resize(nrows);
                HIPCHECK(hipMemcpy(horig.data(), v_orig, nrows * 4, hipMemcpyDeviceToHost));
            }
            hp.mark("sched_key_hash+segments");
            KeyRows kr;
            kr.seg_b = hseg_b.data();
            kr.seg_e = hseg_e.data();
            kr.K = KR;
            kr.orig = v_orig ? horig.data() : nullptr;
            kr.pos_off = a.pos_off;
            kr.n = nrows;
            nfa::TimerIn T = a.T;  // host copy of the clock for the host runs
            T.clk = e->bc.clk.data();
            T.nadv = e->bc.nadv.data();
            q.runs.clear();
            auto take = [&](uint32_t k) -> KeyRun* {
                q.runs.emplace_back(new KeyRun());
                KeyRun* r = q.runs.back().get();
                r->key = k;
                uint8_t cur = 0;
                HIPCHECK(hipMemcpy(&cur, q.cur_bits.as<uint8_t>() + k, 1, hipMemcpyDeviceToHost));
                const int64_t kbn = q.L.bytes;  // (the layout may have grown during the run)
                r->arena.resize(kbn);
                const uint8_t* committed = (cur ? q.arena2.as<uint8_t>() : q.arena.as<uint8_t>()) + (int64_t)k * kbn;
                HIPCHECK(hipMemcpy(r->arena.data(), committed, kbn, hipMemcpyDeviceToHost));
                const int64_t b = k < (uint32_t)KR ? hseg_b[k] : 0, en = k < (uint32_t)KR ? hseg_e[k] : 0, m = en - b;
                r->ts.resize(m);
                r->pos.resize(m);
                for (int64_t p = 0; p < m; ++p) r->pos[p] = (uint32_t)kr.pos(b + p);
                if (m) HIPCHECK(hipMemcpy(r->ts.data(), v_ts + b, m * 8, hipMemcpyDeviceToHost));
                if (v_vrank) {
                    r->vrank.resize(m);
                    if (m) HIPCHECK(hipMemcpy(r->vrank.data(), v_vrank + b, m * 4, hipMemcpyDeviceToHost));
                }
                r->has_qs = multi_stream;
                if (multi_stream) {
                    r->qs.resize(m);
                    if (m) HIPCHECK(hipMemcpy(r->qs.data(), v_qs + b, m, hipMemcpyDeviceToHost));
                }
                r->cols.resize(nc);
                r->nulls.resize(nc);
                for (int c = 0; c < nc; ++c) {
                    const int w = width_of(P.col_kind[c]);
                    r->cols[c].resize((size_t)std::max<int64_t>(m, 1) * w);
                    if (m) HIPCHECK(hipMemcpy(r->cols[c].data(), (const uint8_t*)v_cols[c] + b * w, m * w, hipMemcpyDeviceToHost));
                    if (v_nulls[c]) {
                        r->nulls[c].resize(std::max<int64_t>(m, 1));
                        if (m) HIPCHECK(hipMemcpy(r->nulls[c].data(), v_nulls[c] + b, m, hipMemcpyDeviceToHost));
                    }
                }
                if (P.purge) {  // the key's batch-start reading of its last activity
                    int64_t ls = 0;
                    HIPCHECK(hipMemcpy(&ls, q.last_seen_bak.as<int64_t>() + k, 8, hipMemcpyDeviceToHost));
                    const nfa::PurgeIn pin{e->bc.clk.data(), a.purge_from, a.purge_idle, ls ^ INT64_MIN};
                    r->start(&P, h.code.data(), h.consts.data(), q.L, T, e->seq, &pin);
                } else {
                    r->start(&P, h.code.data(), h.consts.data(), q.L, T, e->seq);
                }
                return r;
            };
            SchedSim::Result res;
            for (int tries = 0; !e->sched_host; ++tries) {
                q.sim.simulate(e->bc, logs, q.key_hash, kr, take, res, true);
                hp.mark("sched_simulate_optimistic");
                q.reordered = res.reordered;
                if (q.reordered.empty()) break;
                const int64_t nl = (int64_t)q.reordered.size();
                a.list = (const uint32_t*)q.d_list.ensure(nl * 4);
                a.fire_off = (const uint32_t*)q.d_foff.ensure((nl + 1) * 4);
                a.fires = (const nfa::TimerFire*)q.d_fires.ensure(std::max<size_t>(1, res.fires.size()) * sizeof(nfa::TimerFire));
                HIPCHECK(hipMemcpyAsync((void*)a.list, q.reordered.data(), nl * 4, hipMemcpyHostToDevice, st));
                HIPCHECK(hipMemcpyAsync((void*)a.fire_off, res.fire_off.data(), (nl + 1) * 4, hipMemcpyHostToDevice, st));
                if (!res.fires.empty())
                    HIPCHECK(hipMemcpyAsync((void*)a.fires, res.fires.data(), res.fires.size() * sizeof(nfa::TimerFire),
                                            hipMemcpyHostToDevice, st));
                a.nlist = (int32_t)nl;
                a.round = 1;
                e->stats.match_launches += 1;
                if (launch(false)) {
                    hp.mark("sched_rerun_launch");
                    read_logs(true);
                    hp.mark("sched_rerun_logs");
                    break;
                }
                // outputs or logs overflowed in the rerun (buffers grown): everything again from the batch start
                if (tries > 8) throw CompileError(SDG_ERR_CAPACITY, "query '" + h.name + "': output buffers keep overflowing");
                first_run();
                q.reordered.clear();
                read_logs(false);
            }
            q.runs.clear();
            // the exact pass only when the reruns did not reproduce the optimistic pass's model changes
            // (SDG_SCHED_EXACT: always; SDG_SCHED_HOST: no optimistic pass, so always)
            if (e->sched_exact || e->sched_host || !q.sim.confirm(logs, res)) {
                q.sim.simulate(e->bc, logs, q.key_hash, kr, take, res);
                e->stats.sched_exact_passes += 1;
            }
            hp.mark("sched_simulate_exact");
            for (auto& r : q.runs) {
                if (r->overflow())
                    throw CompileError(SDG_ERR_CAPACITY, "query '" + h.name + "': a partition key exceeded max_partials "
                                                         "(host replay of a key the scheduler reordered)");
                e->stats.host_rows += (int64_t)r->ts.size();
                uint8_t cur = 0;  // its state goes where the device run's went (nfa_commit makes it current)
                HIPCHECK(hipMemcpy(&cur, q.cur_bits.as<uint8_t>() + r->key, 1, hipMemcpyDeviceToHost));
                uint8_t* work = (cur ? q.arena.as<uint8_t>() : q.arena2.as<uint8_t>()) + (int64_t)r->key * q.L.bytes;
                HIPCHECK(hipMemcpy(work, r->arena.data(), q.L.bytes, hipMemcpyHostToDevice));
                if (P.purge) {
                    const int64_t ls = r->purge_last() ^ INT64_MIN;
                    HIPCHECK(hipMemcpy(q.last_seen.as<int64_t>() + r->key, &ls, 8, hipMemcpyHostToDevice));
                }
            }
            q.sim.commit();
            q.last_rank = std::move(res.rank);
            q.taken.assign(res.taken.begin(), res.taken.end());
            e->stats.sched_fires += res.n_fires;
            e->stats.sched_shifted += res.n_shifted;
            e->stats.sched_host_keys += (int64_t)res.taken.size();
            e->stats.sched_rerun_keys += (int64_t)q.reordered.size();
            e->stats.ms_sched_host += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_sched).count() -
                                      (e->stats.ms_nfa_kernel - k_before);
        }
        if (q.reclaim) nfa_commit_slots(slot_pool(), q.cur_bits.as<uint8_t>(), q.ran_bits.as<uint8_t>(), q.arena_keys, st);
        else nfa_commit(q.cur_bits.as<uint8_t>(), q.ran_bits.as<uint8_t>(), q.arena_keys, st);
        if (!spill_new.empty()) mark_spilled(e, q, spill_new, slot_pool());
        e->stats.arena_slots += q.arena_keys;
        ev_record(e->ev[2], st);
        HIPCHECK(hipStreamSynchronize(st));
        float ms_kg = 0, ms_m = 0, t;
        ev_elapsed(&ms_kg, e->ev[0], e->ev[1]);
        ev_elapsed(&ms_m, e->ev[1], e->ev[2]);
        e->stats.ms_keygroup += ms_kg;
        e->stats.ms_match += ms_m;
        if (partitioned && nrows > 0) {
            ev_elapsed(&t, e->ev[4], e->ev[5]);
            e->stats.ms_kg_hist += t;
            ev_elapsed(&t, e->ev[6], e->ev[7]);
            e->stats.ms_kg_prefix += t;
            ev_elapsed(&t, e->ev[5], e->ev[6]);
            e->stats.ms_kg_scatter += t;
        }
        ev_elapsed(&t, e->ev[8], e->ev[2]);
        e->stats.ms_nfa += t;
        e->stats.events += nrows;
        q.out_n = (int64_t)hc[0];
        q.polled = false;
        q.nulls_valid = true;  // (a chain query that moved here may have left it false)
        e->stats.matches += q.out_n;
        e->stats.path = 1;
        return true;
    }
    // ---- 3. chain matcher -------------------------------------------------------------------------------
    QueryRt::Carry& cin = q.carry[q.cur];
    QueryRt::Carry& cout = q.carry[q.cur ^ 1];
    // output / carry capacity with slack: a buffer that grows inside a timed flush costs a hipFree (device sync)
    // plus a multi-GB hipMalloc, so round up once instead of growing with every larger carry-in count
    // (carried partials: at least n/8 of headroom from the first batch on, so the batch after it -- the first with
    // carries -- does not reallocate every output and carry buffer)
    int64_t cap = nrows + nrows / 8 + std::max(cin.n, nrows / 8) + 4096;
    q.out_cap = cap;
    ChainArgs a;
    std::memset(&a, 0, sizeof a);
    a.xcds = g_xcds;
    a.plan = q.d_plan.as<Plan>();
    a.code = q.d_code.as<Instr>();
    a.consts = q.d_consts.as<int64_t>();
    a.n = nv;
    a.fold = sorted;
    a.ts = v_ts;
    a.ts32 = v_ts32;
    a.ts_base = v_ts32 ? v_tsbase : nullptr;
    a.lkey = v_lkey;
    a.qstream = multi_stream ? v_qs : nullptr;
    a.key = partitioned ? v_key : nullptr;
    a.seg_start = partitioned ? v_seg : nullptr;
    a.seg_end = partitioned ? v_segend : nullptr;
    a.K = (int32_t)K;
    a.orig = v_orig;
    for (int k = 0; k < nc; ++k) { a.cols[k] = v_cols[k]; a.nulls[k] = v_nulls[k]; }
    if (fused) {
        a.ocol_mask = eo_mask;
        for (int k = 0; k < nc; ++k)
            if ((eo_mask >> k) & 1u) a.ocols[k] = d_cols[k];
        a.tm = b_tm;
    }
    a.seq_base = e->seq + (d_vpos ? 0 : pos_off);  // emission seq = seq_base + orig (view row or position)
    a.s0 = h.stream_pos(P.st[0].stream);
    a.s1 = P.n_states > 1 ? h.stream_pos(P.st[1].stream) : a.s0;
    a.out_cap = cap;
    unsigned long long* counters = (unsigned long long*)q.counters.ensure(16);
    HIPCHECK(hipMemsetAsync(counters, 0, 16, st));
    if (!(partitioned && nrows > 0)) HIPCHECK(hipMemsetAsync(flags, 0, 32, st));  // else cleared before grouping
    a.out_count = counters;
    a.carry_count = counters + 1;
    a.flags = flags;
    a.out_ts = (int64_t*)q.o_ts.ensure(cap * 8);
    a.out_key = nullptr;  // not read back
    a.out_vals = (int64_t*)q.o_vals.ensure((size_t)std::max(P.n_out, 1) * cap * 8);
    a.out_nulls = (uint32_t*)q.o_nulls.ensure(cap * 4);
    a.out_emit_seq = (int64_t*)q.o_emit.ensure(cap * 8);
    a.out_first_seq = (int64_t*)q.o_first.ensure(cap * 8);
    cout.cap = cap;
    a.carry_cap = cap;
    a.carry_key = (uint32_t*)cout.key.ensure(cap * 4);
    a.carry_ts = (int64_t*)cout.ts.ensure(cap * 8);
    a.carry_seq = (int64_t*)cout.seq.ensure(cap * 8);
    a.carry_vals = (int64_t*)cout.vals.ensure((size_t)std::max(nc, 1) * cap * 8);
    a.carry_nulls = (uint32_t*)cout.nulls.ensure(cap * 4);
    a.cin_n = cin.n;
    a.cin_key = cin.key.as<uint32_t>();
    a.cin_ts = cin.ts.as<int64_t>();
    a.cin_seq = cin.seq.as<int64_t>();
    a.cin_vals = cin.vals.as<int64_t>();
    a.cin_nulls = cin.nulls.as<uint32_t>();
    a.cin_cap = cin.cap;
    chain_staging(h, a, q.carry_nullable);
    q.nulls_valid = a.write_nulls;
    q.carry_nullable = false;
    for (int k = 0; k < nc; ++k) q.carry_nullable |= a.nulls[k] != nullptr;
    if (fused) {
        static const char* skip = getenv("SDG_FU_SKIP");
        a.fu_skip = skip ? atoi(skip) : 0;
        static const bool old_dq = getenv("SDG_FU_OLDDQ") != nullptr;  // A/B: the monotone-deque pass
        if (old_dq) a.fu_skip |= 64;
        static const bool no_cskip = getenv("SDG_FU_NOSKIP") != nullptr;  // A/B: chunk-summary skipping in the deque
        if (no_cskip) a.fu_skip |= 128;
        a.fu_mode = getenv("SDG_FU_NODEQUE") ? DQ_OFF : a.deque_mode;
        // A/B: the round-4 match passes (chunked deque; SDG_FU_NODEQUE: fixed per-lane forward scans) instead of
        // the wave work queue
        static const bool old_match = getenv("SDG_FU_DEQUE") != nullptr || getenv("SDG_FU_NODEQUE") != nullptr;
        if (old_match) a.fu_skip |= 256;
        a.deque_mode = DQ_OFF;
        a.bstart = b_start;
        a.bseg = b_seg;
        a.nb = 1 << bbits;
        a.bbits = bbits;
        a.lbits = std::max(0, kbits - bbits);
        a.seg_start = a.seg_end = nullptr;
        // one key: half the staged rows are halo (its window spans ~all of a batch's rate, C1: 1000 rows per
        // second), and the staging checks time order itself (no bucket pass did)
        a.fu_own = partitioned ? FU_OWN : FU_ROWS / 2;
        a.fu_check_ts = partitioned ? 0 : 1;
    }
    if (sorted) {  // chain_sorted_k: deque / forward scans in LDS blocks, the rest of a cut run in chain_sovf_k
        static const char* skip = getenv("SDG_FU_SKIP");  // A/B: 512 = the deque step's loops; phase timing (results
        a.fu_skip = (skip ? atoi(skip) : 0) & (512 | 2 | 8 | 16);  // invalid): 8 staging only, 16 no matching, 2 no emission
        // round 6: the wave work queue (C5 shard: matcher 11.16 -> 7.45 ms, flush 28.1 -> 24.4-25.2 ms, r6t).
        // A/B: SDG_SV_DEQUE=1 the round-4 chunked deque + carried-partial scans, SDG_SV_NODEQUE=1 per-lane forward
        // scans for every candidate (8.23 ms, r6s)
        static const bool sv_nodq = getenv("SDG_SV_NODEQUE") != nullptr;
        static const bool sv_dq = getenv("SDG_SV_DEQUE") != nullptr;
        if (!sv_dq && !sv_nodq) a.fu_skip |= 1024;
        a.fu_mode = sv_nodq ? DQ_OFF : a.deque_mode;
        a.deque_mode = DQ_OFF;
        a.seg_start = a.seg_end = nullptr;
    }
    if ((a.deque_mode != DQ_OFF || fused || sorted) && nrows > 0) {
        a.mq = (uint32_t*)q.o_mq.ensure((size_t)nrows * 4);
        a.ovf_rows = (uint32_t*)q.o_ovf.ensure((size_t)nv * 4);
        a.ovf_count = (unsigned long long*)q.o_ovfc.ensure(8);
        HIPCHECK(hipMemsetAsync(a.ovf_count, 0, 8, st));
    }
    // one-key batch on the deque path: 64-row chunk summaries let a lane's continuation skip the chunks that cannot
    // complete its deque's top (ordering comparisons on a numeric scan column only; chain_dq_summ_k)
    const bool numeric = a.sp.scan_t == VK_I32 || a.sp.scan_t == VK_I64 || a.sp.scan_t == VK_F32 || a.sp.scan_t == VK_F64;
    const bool ord_op = a.sp.scan_op == CMP_GT || a.sp.scan_op == CMP_GE || a.sp.scan_op == CMP_LT || a.sp.scan_op == CMP_LE;
    static const bool summ_all = getenv("SDG_DQ_SUMM_ALL") != nullptr;  // A/B: summaries on keyed batches too
    if (a.deque_mode != DQ_OFF && !fused && nrows > 0 && (!a.key || summ_all) && numeric && ord_op &&
        a.sp.scan_mode != SCAN_TRUE && !getenv("SDG_DQ_NOSKIP")) {
        const int64_t nch = (nrows + DQ_CHUNK - 1) / DQ_CHUNK, ngr = nch * (DQ_CHUNK / DQ_GROUP);
        uint8_t* b = (uint8_t*)q.o_dqs.ensure((size_t)(nch + ngr) * 17);
        a.dq_hi = (int64_t*)b;
        a.dq_lo = a.dq_hi + nch;
        a.dq_hi8 = a.dq_lo + nch;
        a.dq_lo8 = a.dq_hi8 + ngr;
        a.dq_any = (uint8_t*)(a.dq_lo8 + ngr);
        a.dq_any8 = a.dq_any + nch;
        // with skipping, a lane's own rows are most of its serial work: fewer per lane, more lanes (C1: 244 waves
        // of 64 rows left 3/4 of the SIMDs idle)
        static const char* lane = getenv("SDG_DQ_LANE");
        a.dq_lane = lane ? atoi(lane) : 16;
        if (a.dq_lane < DQ_GROUP || a.dq_lane % DQ_GROUP) a.dq_lane = DQ_CHUNK;
    }
    ChainArgs* d_a = (ChainArgs*)q.d_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));
    ChainArgs* h_a = (ChainArgs*)q.h_args.ensure(std::max(sizeof(NfaArgs), 2 * sizeof(ChainArgs)));  // pinned
    h_a[0] = a;
    h_a[1] = a;  // emit-only pass over mq
    h_a[1].mq_in = a.mq;
    HIPCHECK(hipMemcpyAsync(d_a, h_a, 2 * sizeof(ChainArgs), hipMemcpyHostToDevice, st));
    static const bool dbg = getenv("SDG_DEBUG") != nullptr;
    auto dbg_sync = [&](const char* what) {  // SDG_DEBUG: name the kernel an asynchronous fault came from
        if (!dbg) return;
        hipError_t err = hipStreamSynchronize(st);
        if (err != hipSuccess) throw DeviceError(std::string(what) + ": " + hipGetErrorString(err));
    };
    dbg_sync("bucketize / staging");
    ev_record(e->ev[3], st);  // after the buffer (re)allocations above: they stall the stream, not the kernels
    // fused path: the carried partials' pass is independent of the matcher's (both only reserve output / carry slots
    // atomically; delivery order comes from the export's sort), so SDG_CARRY_SIDE=1 runs it on a second stream beside
    // it (the stream joins before anything reads the counters). Off by default: C2 step 3.695 -> 3.673 ms, but the
    // matcher's own time grows 2.04 -> 2.10 ms beside it (r5c1)
    const char* cside_env = getenv("SDG_CARRY_SIDE");  // (read per flush: the tests switch it)
    const bool carry_serial = !(cside_env && atoi(cside_env) == 1);
    const bool carry_side = fused && !sorted && a.cin_n > 0 && !carry_serial && !dbg && sub_J <= 1;
    if (carry_side) {
        HIPCHECK(hipEventRecord(e->fork, st));
        HIPCHECK(hipStreamWaitEvent(e->stream2, e->fork, 0));
        chain_carry(a, d_a, e->stream2);
        HIPCHECK(hipEventRecord(e->join, e->stream2));
    } else if (!sorted && sub_J <= 1) {
        chain_carry(a, d_a, st);  // (sorted: the carried partials are rows of the view; sub-batches: below)
    }
    dbg_sync("chain_carry_k");
    ev_record(e->ev[8], st);
    if (fused && sub_J > 1) {
        // per sub-batch: its bucket pass (view + plan), [the carried partials, on the first view], the matcher and
        // its HBM scans. Two argument blocks: every sub-batch but the last ends dead (sub_dead), the last carries
        ChainArgs* d_sub = (ChainArgs*)q.d_sub_args.ensure(2 * sizeof(ChainArgs));
        ChainArgs* h_sub = (ChainArgs*)q.h_sub_args.ensure(2 * sizeof(ChainArgs));  // pinned
        h_sub[0] = a;
        h_sub[0].bown = b_own;
        h_sub[0].sub_dead = 1;
        h_sub[1] = h_sub[0];
        h_sub[1].sub_dead = 0;
        HIPCHECK(hipMemcpyAsync(d_sub, h_sub, 2 * sizeof(ChainArgs), hipMemcpyHostToDevice, st));
        const int64_t tile = bucket_tile();
        if (q.sub_ev.size() < (size_t)(4 * sub_J + 2)) {
            const size_t old_n = q.sub_ev.size();
            q.sub_ev.resize((size_t)(4 * sub_J + 2));
            for (size_t i = old_n; i < q.sub_ev.size(); ++i) HIPCHECK(hipEventCreate(&q.sub_ev[i]));
        }
        hp.mark("chain_setup+carry");
        for (int64_t j = 0; j < sub_J; ++j) {
            const bool last = j + 1 == sub_J;
            const int64_t row0 = j * sub_S;
            const int64_t rows = last ? nrows - row0 : std::min(sub_S + sub_H, nrows - row0);
            const int64_t own = last ? (rows + tile - 1) / tile * tile : sub_S;
            ChainArgs* dj = d_sub + (last ? 1 : 0);
            const ChainArgs& hj = h_sub[last ? 1 : 0];
            ev_record(q.sub_ev[4 * j], st);
            bucketize_sub(sub_kg, bbits, 0, flags + 3, row0, rows, own, b_start, b_seg, b_own, FU_OWN, st);
            ev_record(q.sub_ev[4 * j + 1], st);
            if (j == 0) chain_carry(hj, dj, st);
            ev_record(q.sub_ev[4 * j + 2], st);
            if (j > 0) HIPCHECK(hipMemsetAsync(a.ovf_count, 0, 8, st));  // (the HBM-scan list is per view)
            chain_fused(hj, dj, chain_fused_grid(rows, a.nb, a.fu_own), st);
            ev_record(q.sub_ev[4 * j + 3], st);
            chain_fovf(hj, dj, st);
            dbg_sync("fused sub-batch");
        }
        ev_record(e->ev[9], st);
    } else if (fused) {
        const int64_t grid = chain_fused_grid(nrows, a.nb, a.fu_own);
        static int64_t* trace = nullptr;
        static int64_t trace_n = 0;
        if (dbg) {  // host-mapped progress trace, readable after a device fault
            if (trace_n < grid * 4) {
                if (trace) (void)hipHostFree(trace);
                HIPCHECK(hipHostMalloc((void**)&trace, (size_t)(grid * 4 + 64) * 8, hipHostMallocMapped));
                trace_n = grid * 4;
            }
            for (int64_t i = 0; i < grid * 4 + 64; ++i) trace[i] = -1;
            void* dp = nullptr;
            HIPCHECK(hipHostGetDevicePointer(&dp, trace, 0));
            a.dbg = (volatile int64_t*)dp;
            HIPCHECK(hipMemcpyAsync(d_a, &a, sizeof a, hipMemcpyHostToDevice, st));
        }
        hp.mark("chain_setup+carry");
        try {
            chain_fused(a, d_a, grid, st);
        } catch (...) {  // stream2 may still write carry / output buffers: join it before anything reuses them
            if (carry_side) (void)hipStreamSynchronize(e->stream2);
            throw;
        }
        if (carry_side) HIPCHECK(hipStreamWaitEvent(st, e->join, 0));
        hp.mark("fused_enqueue");
        if (dbg) {
            hipError_t err = hipStreamSynchronize(st);
            if (err != hipSuccess) {
                std::string m = "chain_fused_k: " + std::string(hipGetErrorString(err)) + "; grid " + std::to_string(grid) +
                                " nb " + std::to_string(a.nb) + " bbits " + std::to_string(a.bbits) + " lbits " +
                                std::to_string(a.lbits) + " n " + std::to_string(nrows) + "; unfinished waves:";
                for (int i = 0; i < 16; ++i) m += (i % 8 ? "," : " | ") + std::to_string(trace[grid * 4 + i]);
                char pb[64];
                for (int k = 0; k < nc; ++k) { snprintf(pb, sizeof pb, " col%d=%p", k, a.cols[k]); m += pb; }
                snprintf(pb, sizeof pb, " out_vals=%p", (void*)a.out_vals); m += pb;
                int shown = 0;
                for (int64_t i = 0; i < grid * 4 && shown < 40; ++i)
                    if (trace[i] != 100 && trace[i] != 99) {
                        m += " [" + std::to_string(i / 4) + "." + std::to_string(i % 4) + "]=" + std::to_string(trace[i]);
                        ++shown;
                    }
                fprintf(stderr, "%s\n", m.c_str());
                throw DeviceError(m);
            }
        }
        ev_record(e->ev[9], st);
        chain_fovf(a, d_a, st);
        dbg_sync("chain_fovf_k");
    } else if (sorted) {
        chain_sorted(a, d_a, st);
        dbg_sync("chain_sorted_k");
        ev_record(e->ev[9], st);
        chain_sovf(a, d_a, st);
        dbg_sync("chain_sovf_k");
    } else if (a.deque_mode != DQ_OFF && nrows > 0) {
        chain_deque(a, d_a, st);
        ev_record(e->ev[9], st);
        chain_match(h_a[1], d_a + 1, st);
    } else {
        ev_record(e->ev[9], st);
        chain_match(a, d_a, st);
    }
    e->stats.match_launches += (cin.n > 0) + (nrows > 0);
    ev_record(e->ev[2], st);
    uint8_t* ret = (uint8_t*)q.h_ret.ensure(56);
    unsigned long long* hc = (unsigned long long*)ret;
    int* hf = (int*)(ret + 16);
    unsigned long long& hovf = *(unsigned long long*)(ret + 48);
    hovf = 0;
    HIPCHECK(hipMemcpyAsync(hc, counters, 16, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(hf, flags, 32, hipMemcpyDeviceToHost, st));
    if (fused || sorted) HIPCHECK(hipMemcpyAsync(&hovf, a.ovf_count, 8, hipMemcpyDeviceToHost, st));
    hp.mark("tail_enqueue");
    HIPCHECK(hipStreamSynchronize(st));
    hp.mark("sync_wait");
    if (hf[4]) throw CompileError(SDG_ERR_ARG, "device-resident partition key ids out of range (not from sdg_intern)");
    if (fused && hf[2]) throw DeviceError("fused matcher bounds check failed: bits " + std::to_string(hf[2]));
    if (fused && sub_J > 1 && hf[5]) {  // a sub-batch's halo did not reach past its window: rerun without sub-batches
        q.no_sub = true;
        sub_retry = true;
        q.carry_nullable = carry_nullable0;
        return false;
    }
    if (fused && hf[3]) {  // batch timestamps not in arrival order (or a block's span over 2^32 ms): radix / lane path
        e->stats.fused = 2;
        q.carry_nullable = carry_nullable0;
        return false;
    }
    if (sorted && hf[3]) {  // a block's staged span over 2^32 ms: the lane deque kernels
        sorted_now = false;
        q.carry_nullable = carry_nullable0;
        return false;
    }
    e->stats.fused = fused ? 1 : e->stats.fused;
    e->stats.sorted_view = sorted ? 1 : 0;
    e->stats.fused_ovf += (int64_t)hovf;
    float ms_kg = 0, ms_m = 0;
    ev_elapsed(&ms_kg, e->ev[0], e->ev[1]);
    ev_elapsed(&ms_m, e->ev[1], e->ev[2]);
    e->stats.ms_keygroup += ms_kg;
    e->stats.ms_match += ms_m;
    float t;
    if (fused && sub_J > 1) {  // sub-batches: bucket passes (hist + prefix + scatter + plan), carry, matcher, HBM scans
        for (int64_t j = 0; j < sub_J; ++j) {
            ev_elapsed(&t, q.sub_ev[4 * j], q.sub_ev[4 * j + 1]);
            e->stats.ms_kg_scatter += t;
            ev_elapsed(&t, q.sub_ev[4 * j + 1], q.sub_ev[4 * j + 2]);
            e->stats.ms_chain_carry += t;
            ev_elapsed(&t, q.sub_ev[4 * j + 2], q.sub_ev[4 * j + 3]);
            e->stats.ms_chain_match += t;
            ev_elapsed(&t, q.sub_ev[4 * j + 3], j + 1 < sub_J ? q.sub_ev[4 * j + 4] : e->ev[9]);
            e->stats.ms_chain_emit += t;
        }
        e->stats.sub_batches = (int32_t)sub_J;
    } else if (partitioned && nrows > 0) {
        // radix: [4]..[5] first hist+prefix, [5]..[6] scatter passes (+ later hist/prefix), [6]..[7] segments
        ev_elapsed(&t, e->ev[4], e->ev[5]);
        e->stats.ms_kg_hist += t;
        ev_elapsed(&t, e->ev[6], e->ev[7]);
        e->stats.ms_kg_prefix += t;
        ev_elapsed(&t, e->ev[5], e->ev[6]);
        e->stats.ms_kg_scatter += t;
    }
    e->stats.carry_in += cin.n;
    e->stats.carry_out += (int64_t)hc[1];
    if (!(fused && sub_J > 1)) {
        ev_elapsed(&t, e->ev[3], e->ev[8]);
        e->stats.ms_chain_carry += t;
        ev_elapsed(&t, e->ev[8], e->ev[9]);
        e->stats.ms_chain_match += t;
        ev_elapsed(&t, e->ev[9], e->ev[2]);
        e->stats.ms_chain_emit += t;
    }
    e->stats.deque = sorted ? a.fu_mode : a.deque_mode;
    e->stats.events += nrows;
    if (hf[0]) {
        e->stats.overflow += 1;
        throw CompileError(SDG_ERR_CAPACITY, "match/carry buffer overflow in query '" + h.name + "'");
    }
    if (hf[1]) {
        // timestamps decrease within a partition key: the chain path's exactness argument needs them
        // non-decreasing. From this batch on the query runs on the generic NFA (nothing of this run is committed:
        // the carries stay in cin and are replayed into the arenas first).
        P.chain = 0;
        q.replay_carries = cin.n > 0;
        q.carry_nullable = carry_nullable0;
        e->stats.path = 1;
        return false;
    }
    cout.n = (int64_t)hc[1];
    cin.n = 0;
    q.cur ^= 1;
    q.out_n = (int64_t)hc[0];
    q.polled = false;
    e->stats.matches += q.out_n;
    e->stats.path = 0;
    q.last_timers = false;
    q.emit_base = e->seq;
    q.emit_span = e->flush_G;
    q.sub_is_seq = true;
    hp.mark("post_sync");
    return true;
    };
    // rerun on the radix path (fused precondition broken), or on the generic NFA (chain precondition broken)
    for (int attempt = 0; !run(try_fused && (attempt == 0 || (attempt == 1 && sub_retry))); ++attempt)
        if (attempt >= 3) throw DeviceError("query '" + h.name + "': no matcher path accepted the batch");
}

// read the last flush's match records back (pinned staging) and append them to the query's delivery backlog in
// the reference's delivery order: by emitting event, then by the partial's position in the pending list
// (StateMultiProcessStreamReceiver.processAndClear :47-68, QuerySelector.processNoGroupBy :161-205)
// a pinned delivery batch (QueryRt::del_buf) not polled yet joins the host backlog (acc_*) before more records do
void del_to_backlog(QueryRt& q) {
    if (q.del_n < 0) return;
    const int64_t n = q.del_n;
    const int nu = q.del_nu;
    const uint8_t* base = (const uint8_t*)q.del_buf[q.del_cur ^ 1].p;
    const int64_t* ts = (const int64_t*)base;
    const int64_t* emit = ts + n;
    const int64_t* vals = emit + n;
    const uint8_t* nb = (const uint8_t*)(vals + (size_t)nu * n);
    const size_t b = q.acc_ts.size();
    q.acc_ts.resize(b + n);
    q.acc_seq.resize(b + n);
    par_memcpy(q.acc_ts.data() + b, ts, (size_t)n * 8);
    par_memcpy(q.acc_seq.data() + b, emit, (size_t)n * 8);
    q.acc_vals.resize(nu);
    q.acc_nulls.resize(nu);
    for (int j = 0; j < nu; ++j) {
        q.acc_vals[j].resize(b + n);
        par_memcpy(q.acc_vals[j].data() + b, vals + (size_t)j * n, (size_t)n * 8);
        q.acc_nulls[j].resize(b + n);
        if (q.del_nulls) par_memcpy(q.acc_nulls[j].data() + b, nb + (size_t)j * n, (size_t)n);
        else std::memset(q.acc_nulls[j].data() + b, 0, (size_t)n);
    }
    q.del_n = -1;
}

void drain(sdg_engine* e, QueryRt& q) {
    if (q.polled) return;
    q.polled = true;
    HostProf hp;  // SDG_HOST_PROF: the drain's phases (ordering enqueue, read-back, null bytes)
    del_to_backlog(q);
    hp.mark("drain_backlog");
    const int64_t n = q.out_n;
    // @purge with aggregators: keys purged after their last record restart their aggregator states -- after this
    // flush's records went through the post pass
    struct TailReset {
        sdg_engine* e;
        QueryRt& q;
        ~TailReset() {
            if (!q.purge_agg || q.agg_keys <= 0 || !q.agg_reset_flags.p) return;
            agg_reset((int64_t*)q.agg_state.p, q.hq.plan.n_agg, q.agg_reset_flags.as<uint8_t>(),
                      std::min<int64_t>(q.agg_keys, q.arena_keys), e->stream);
            (void)hipStreamSynchronize(e->stream);
        }
    } tail_reset{e, q};
    // host runs whose records join the device's: scheduler replays (timers) and spilled keys
    std::vector<const KeyOut*> hruns;
    for (auto& r : q.runs) hruns.push_back(r.get());
    for (auto& r : q.spill_runs) hruns.push_back(r.get());
    if (n <= 0 && hruns.empty()) return;
    const int na = q.hq.plan.n_out;  // every column of the records (hidden selector columns included)
    const bool post = q.hq.plan.has_post;
    uint8_t* hb = (uint8_t*)q.h_rb.ensure((size_t)n * (28 + 8 * (size_t)na));
    int64_t* ts = (int64_t*)hb;
    int64_t* emit = ts + n;
    int64_t* first = emit + n;
    int64_t* vals = first + n;
    uint32_t* nulls = (uint32_t*)(vals + (size_t)na * n);
    hipStream_t st = e->stream;
    // records of queries without timers are put in delivery order on the device and read back in that order
    const void* src_ts = q.o_ts.p;
    const void* src_emit = q.o_emit.p;
    const void* src_first = q.o_first.p;
    const int64_t* src_vals = (const int64_t*)q.o_vals.p;
    int64_t vstride = q.out_cap;
    const void* src_nulls = q.o_nulls.p;
    const void* src_key = q.o_key.p;
    const void* src_flags = q.o_flags.p;
    const bool dev_order = !q.last_timers && n > 1 && hruns.empty();
    if (dev_order) {
        const size_t wb = order_workspace(n);
        void* work = q.ord_ws.ensure_slack(wb);  // (slack: a slightly larger flush must not reallocate -- a
                                                     // hipFree + hipMalloc of GBs costs more than the ordering)
        uint32_t* perm = nullptr;
        order_records((const int64_t*)q.o_emit.p, (const int64_t*)q.o_first.p, n, q.emit_base, q.emit_span,
                      q.sub_is_seq ? q.emit_base - (1ll << 40) : 0, q.sub_bits(), work, wb, &perm, st);
        const size_t ns = (size_t)n;  // (slack: ensure_slack, as the workspaces)
        int64_t* gts = (int64_t*)q.g_ts.ensure_slack(ns * 8);
        int64_t* gem = (int64_t*)q.g_emit.ensure_slack(ns * 8);
        int64_t* gv = (int64_t*)q.g_vals.ensure_slack((size_t)std::max(na, 1) * ns * 8);
        {
            std::vector<const int64_t*> src{(const int64_t*)q.o_ts.p, (const int64_t*)q.o_emit.p};
            std::vector<int64_t*> dst{gts, gem};
            for (int j = 0; j < na; ++j) {
                src.push_back((const int64_t*)q.o_vals.p + (size_t)j * q.out_cap);
                dst.push_back(gv + (size_t)j * n);
            }
            gather_cols_i64(src.data(), dst.data(), (int)src.size(), perm, n,
                            q.gather_ws.ensure_slack(gather_cols_workspace(n, std::min((int)src.size(), GATHER_MAX_COLS))), st);
        }
        if (q.nulls_valid) {
            uint32_t* gn = (uint32_t*)q.g_nulls.ensure((size_t)n * 4);
            gather_u32((const uint32_t*)q.o_nulls.p, perm, n, gn, st);
            src_nulls = gn;
        }
        if (post) {
            uint32_t* gk = (uint32_t*)q.g_key.ensure((size_t)n * 4);
            gather_u32((const uint32_t*)q.o_key.p, perm, n, gk, st);
            src_key = gk;
        }
        if (q.purge_agg) {
            uint8_t* gf = (uint8_t*)q.g_flags.ensure((size_t)n);
            gather_u8((const uint8_t*)q.o_flags.p, perm, n, gf, st);
            src_flags = gf;
        }
        src_ts = gts;
        src_emit = gem;
        src_first = nullptr;
        src_vals = gv;
        vstride = n;
        if (hp.on) {
            HIPCHECK(hipStreamSynchronize(st));
            hp.mark("drain_order");
        }
    }
    // pinned delivery: read the ordered columns straight into the next delivery buffer (layout ts | emit | vals[nu]
    // | null bytes[nu]); sdg_poll hands it out as it is
    const int nu_out = q.hq.plan.n_user_out + q.hq.plan.n_list_cols;
    bool direct = dev_order && !post && q.acc_ts.empty() && nu_out <= na && !getenv("SDG_POLL_COPY");
    for (int j = 0; j < q.hq.plan.n_user_out && direct; ++j) direct = !q.hq.plan.out_multi[j];
    if (direct) {
        const size_t bytes = (size_t)n * (16 + 8 * (size_t)nu_out) + (q.nulls_valid ? (size_t)n * nu_out : 0);
        uint8_t* db = (uint8_t*)q.del_buf[q.del_cur ^ 1].ensure_slack(bytes);  // (slack: flush sizes vary)
        int64_t* dts = (int64_t*)db;
        int64_t* dem = dts + n;
        int64_t* dv = dem + n;
        uint8_t* dnb = (uint8_t*)(dv + (size_t)nu_out * n);
        HIPCHECK(hipMemcpyAsync(dts, src_ts, n * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(dem, src_emit, n * 8, hipMemcpyDeviceToHost, st));
        for (int j = 0; j < nu_out; ++j)
            HIPCHECK(hipMemcpyAsync(dv + (size_t)j * n, src_vals + (size_t)j * vstride, n * 8, hipMemcpyDeviceToHost, st));
        if (q.nulls_valid) HIPCHECK(hipMemcpyAsync(nulls, src_nulls, n * 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        hp.mark("drain_d2h_direct");
        if (q.nulls_valid)
            for (int j = 0; j < nu_out; ++j) {
                uint8_t* dn = dnb + (size_t)j * n;
                par_range(n, 1 << 20, [&](int64_t lo, int64_t hi) {
                    for (int64_t i = lo; i < hi; ++i) dn[i] = (nulls[i] >> j) & 1u;
                });
            }
        std::vector<uint8_t>& z = q.del_zero[q.del_cur ^ 1];
        if (z.size() < (size_t)n) z.assign((size_t)n + (size_t)n / 8, 0);
        q.del_n = n;
        q.del_nu = nu_out;
        q.del_nulls = q.nulls_valid;
        hp.mark("drain_nulls");
        return;
    }
    std::vector<uint32_t> okey;
    std::vector<uint8_t> oround, oflags;
    if (n > 0) {  // (a flush whose records all come from host runs reads nothing back)
        if (q.purge_agg) {  // (no timers: purge with aggregators excludes absent states, so no host replay records)
            oflags.resize(n);
            HIPCHECK(hipMemcpyAsync(oflags.data(), src_flags, n, hipMemcpyDeviceToHost, st));
        }
        if (q.last_timers || post || !q.taken.empty()) {  // keys: the aggregators' state, the records of keys the
            okey.resize(n);                                 // host replayed (dropped), timer matches' fire order
            HIPCHECK(hipMemcpyAsync(okey.data(), src_key, n * 4, hipMemcpyDeviceToHost, st));
        }
        if (q.last_timers) {
            if (!q.reordered.empty()) {  // and the first run's records of the keys rerun with the scheduler's order
                oround.resize(n);
                HIPCHECK(hipMemcpyAsync(oround.data(), q.o_round.p, n, hipMemcpyDeviceToHost, st));
            }
        }
        HIPCHECK(hipMemcpyAsync(ts, src_ts, n * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(emit, src_emit, n * 8, hipMemcpyDeviceToHost, st));
        if (src_first) HIPCHECK(hipMemcpyAsync(first, src_first, n * 8, hipMemcpyDeviceToHost, st));
        if (q.nulls_valid) HIPCHECK(hipMemcpyAsync(nulls, src_nulls, n * 4, hipMemcpyDeviceToHost, st));
        for (int j = 0; j < na; ++j)
            HIPCHECK(hipMemcpyAsync(vals + (size_t)j * n, src_vals + (size_t)j * vstride, n * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
    }
    // records already in delivery order on the device, nothing to drop, rank or aggregate: the columns join the
    // backlog as they are (a memcpy per column instead of a per-record walk)
    if (dev_order && !post) {
        const int nu = q.hq.plan.n_user_out + q.hq.plan.n_list_cols;
        const size_t b = q.acc_ts.size();
        q.acc_ts.resize(b + n);
        q.acc_seq.resize(b + n);
        par_memcpy(q.acc_ts.data() + b, ts, (size_t)n * 8);
        par_memcpy(q.acc_seq.data() + b, emit, (size_t)n * 8);
        q.acc_vals.resize(nu);
        q.acc_nulls.resize(nu);
        for (int j = 0; j < nu; ++j) {
            q.acc_vals[j].resize(b + n);
            par_memcpy(q.acc_vals[j].data() + b, vals + (size_t)j * n, (size_t)n * 8);
            q.acc_nulls[j].resize(b + n);
            uint8_t* dn = q.acc_nulls[j].data() + b;
            if (q.nulls_valid)
                par_range(n, 1 << 20, [&](int64_t lo, int64_t hi) {
                    for (int64_t i = lo; i < hi; ++i) dn[i] = (nulls[i] >> j) & 1u;
                });
            else
                par_range(n, 16 << 20, [&](int64_t lo, int64_t hi) { std::memset(dn + lo, 0, (size_t)(hi - lo)); });
        }
        for (int j = 0; j < q.hq.plan.n_user_out; ++j)  // OP_SLOTLEN counted to cap + 1: a longer chain
            if (q.hq.plan.out_multi[j])
                for (int64_t i = 0; i < n; ++i)
                    if (q.acc_vals[j][b + i] > q.hq.plan.out_list_cap[j])
                        throw CompileError(SDG_ERR_CAPACITY, "query '" + q.hq.name + "': a multi-value selection holds "
                                                             "more than " + std::to_string(q.hq.plan.out_list_cap[j]) +
                                                             " events");
        return;
    }
    if (!q.nulls_valid) std::memset(nulls, 0, (size_t)n * 4);
    // the host replays' records join the device's (same layout, after them)
    int64_t nh = 0;
    for (const KeyOut* r : hruns) nh += (int64_t)r->count;
    std::vector<int64_t> hts, hemit, hfirst, hvals;
    std::vector<uint32_t> hnulls, hkey;
    if (nh) {
        hts.reserve(nh); hemit.reserve(nh); hfirst.reserve(nh); hnulls.reserve(nh); hkey.reserve(nh);
        hvals.resize((size_t)na * nh);
        int64_t x = 0;
        for (const KeyOut* r : hruns) {
            const int64_t cap = (int64_t)r->o_ts.size();
            for (unsigned long long i = 0; i < r->count; ++i, ++x) {
                hts.push_back(r->o_ts[i]);
                hemit.push_back(r->o_seq[i]);
                hfirst.push_back(r->o_sub[i]);
                hnulls.push_back(r->o_nulls[i]);
                hkey.push_back(r->key);
                for (int j = 0; j < na; ++j) hvals[(size_t)j * nh + x] = r->o_vals[(size_t)j * cap + i];
            }
        }
    }
    auto slot = [&](int64_t& em, int64_t& fs, uint32_t key) {  // a timer match: its fire's slot (position, rank)
        if (fs >= 0) return;
        const int sch = (int)((fs >> 48) & 0x7F);
        const SchedSim::Slot* it = q.last_rank.find(SchedSim::rank_key((uint32_t)(em - q.last_seq_base), sch, key));
        if (!it) return;
        em = q.last_seq_base + it->g;
        fs = INT64_MIN | ((int64_t)it->rank << 24) | (fs & 0xFFFFFF);
    };
    std::vector<int64_t> ord;  // < n: device record, >= n: host record n + i
    ord.reserve(n + nh);
    for (int64_t i = 0; i < n; ++i) {
        if (!q.taken.empty() && std::binary_search(q.taken.begin(), q.taken.end(), okey[i])) continue;
        if (q.last_timers) {
            if (!oround.empty() && oround[i] == 0 && std::binary_search(q.reordered.begin(), q.reordered.end(), okey[i]))
                continue;
            slot(emit[i], first[i], okey[i]);
        }
        ord.push_back(i);
    }
    for (int64_t i = 0; i < nh; ++i) {
        slot(hemit[i], hfirst[i], hkey[i]);
        ord.push_back(n + i);
    }
    auto EM = [&](int64_t x) { return x < n ? emit[x] : hemit[x - n]; };
    auto FI = [&](int64_t x) { return x < n ? first[x] : hfirst[x - n]; };
    const int64_t nk = (int64_t)ord.size();
    if (!dev_order)
        std::sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) {
            return EM(x) != EM(y) ? EM(x) < EM(y) : FI(x) < FI(y);
        });
    // the selector's post pass on the device over the records in delivery order (aggregators per key, select items
    // over them, having), then the user's columns of the records that pass join the backlog
    std::vector<int64_t> fv;
    std::vector<uint32_t> fn;
    std::vector<uint8_t> fpass;
    if (post && nk > 0) {
        const Plan& P = q.hq.plan;
        std::vector<uint32_t> fk(nk);
        fv.resize((size_t)na * nk);
        fn.resize(nk);
        uint32_t kmax = 0;
        std::vector<uint8_t> fr(q.purge_agg ? nk : 0);
        for (int64_t i = 0; i < nk; ++i) {
            const int64_t s = ord[i];
            const bool dev = s < n;
            if (q.purge_agg) fr[i] = dev ? oflags[s] : 0;
            fk[i] = dev ? okey[s] : hkey[s - n];
            kmax = std::max(kmax, fk[i]);
            fn[i] = dev ? nulls[s] : hnulls[s - n];
            for (int j = 0; j < na; ++j) fv[(size_t)j * nk + i] = dev ? vals[(size_t)j * n + s] : hvals[(size_t)j * nh + (s - n)];
        }
        const int64_t K = (int64_t)kmax + 1;
        const size_t per = (size_t)std::max(P.n_agg, 1) * 16;
        if (K > q.agg_keys) {  // grow the per-key aggregator state, keeping the existing keys' states
            const int64_t nkeys = std::max<int64_t>(K, q.agg_keys * 2);
            void* nb = nullptr;
            HIPCHECK(hipMalloc(&nb, (size_t)nkeys * per));
            HIPCHECK(hipMemsetAsync(nb, 0, (size_t)nkeys * per, st));
            if (q.agg_keys) HIPCHECK(hipMemcpyAsync(nb, q.agg_state.p, (size_t)q.agg_keys * per, hipMemcpyDeviceToDevice, st));
            HIPCHECK(hipStreamSynchronize(st));
            if (q.agg_state.p) HIPCHECK(hipFree(q.agg_state.p));
            q.agg_state.p = nb;
            q.agg_state.cap = (size_t)nkeys * per;
            q.agg_keys = nkeys;
        }
        int kbits = 0;
        while ((1ll << kbits) < K) ++kbits;
        uint32_t* dk = (uint32_t*)q.ps_key.ensure((size_t)nk * 4);
        int64_t* dv = (int64_t*)q.ps_vals.ensure((size_t)na * nk * 8);
        uint32_t* dn = (uint32_t*)q.ps_nulls.ensure((size_t)nk * 4);
        uint8_t* dp = (uint8_t*)q.ps_pass.ensure((size_t)nk);
        HIPCHECK(hipMemcpyAsync(dk, fk.data(), (size_t)nk * 4, hipMemcpyHostToDevice, st));
        HIPCHECK(hipMemcpyAsync(dv, fv.data(), (size_t)na * nk * 8, hipMemcpyHostToDevice, st));
        HIPCHECK(hipMemcpyAsync(dn, fn.data(), (size_t)nk * 4, hipMemcpyHostToDevice, st));
        SelPostArgs pa;
        std::memset(&pa, 0, sizeof pa);
        pa.plan = q.d_plan.as<Plan>();
        pa.code = q.d_code.as<Instr>();
        pa.consts = q.d_consts.as<int64_t>();
        pa.n = nk;
        pa.vals = dv;
        pa.vstride = nk;
        pa.nulls = dn;
        pa.pass = dp;
        pa.agg_state = (int64_t*)q.agg_state.p;
        if (q.purge_agg) {
            uint8_t* dr = (uint8_t*)q.ps_reset.ensure((size_t)nk);
            HIPCHECK(hipMemcpyAsync(dr, fr.data(), (size_t)nk, hipMemcpyHostToDevice, st));
            pa.reset = dr;
        }
        select_post(pa, q.hq.plan.partitioned ? dk : nullptr, kbits, q.ps_ws.ensure(select_post_workspace(nk)), st);
        fpass.resize(nk);
        HIPCHECK(hipMemcpyAsync(fv.data(), dv, (size_t)(P.n_user_out + P.n_list_cols) * nk * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(fn.data(), dn, (size_t)nk * 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(fpass.data(), dp, (size_t)nk, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
    }
    const int nu = q.hq.plan.n_user_out + q.hq.plan.n_list_cols;  // the select list, then list elements
    int64_t keep = nk;
    if (post) keep = (int64_t)std::count(fpass.begin(), fpass.end(), (uint8_t)1);
    const size_t b = q.acc_ts.size();
    q.acc_ts.resize(b + keep);
    q.acc_seq.resize(b + keep);
    q.acc_vals.resize(nu);
    q.acc_nulls.resize(nu);
    for (int j = 0; j < nu; ++j) {
        q.acc_vals[j].resize(b + keep);
        q.acc_nulls[j].resize(b + keep);
    }
    for (int64_t i = 0, o = (int64_t)b; i < nk; ++i) {
        if (post && !fpass[i]) continue;
        const int64_t s = ord[i];
        const bool dev = s < n;
        const int64_t hs = s - n;
        q.acc_ts[o] = dev ? ts[s] : hts[hs];
        q.acc_seq[o] = EM(s);
        const uint32_t nm = post ? fn[i] : dev ? nulls[s] : hnulls[hs];
        for (int j = 0; j < nu; ++j) {
            q.acc_vals[j][o] = post ? fv[(size_t)j * nk + i] : dev ? vals[(size_t)j * n + s] : hvals[(size_t)j * nh + hs];
            q.acc_nulls[j][o] = (nm >> j) & 1u;
        }
        for (int j = 0; j < q.hq.plan.n_user_out; ++j)  // OP_SLOTLEN counted to cap + 1: a longer chain
            if (q.hq.plan.out_multi[j] && q.acc_vals[j][o] > q.hq.plan.out_list_cap[j])
                throw CompileError(SDG_ERR_CAPACITY, "query '" + q.hq.name + "': a multi-value selection holds more than " +
                                                         std::to_string(q.hq.plan.out_list_cap[j]) + " events");
        ++o;
    }
    q.runs.clear();
    q.spill_runs.clear();
}

// the batch clock (sched.h BatchClock): playback = TimestampGeneratorImpl.setCurrentTimestamp per position (an
// event or advance_time with ts >= clock advances it and runs the TimeChangeListeners); live = only advance_time
// points move the modelled wall clock, each running live_fire_until
void build_clock(sdg_engine* e, int64_t G) {
    BatchClock& bc = e->bc;
    const bool playback = e->app.playback;
    bc.G = G;
    bc.clock0 = e->clock;
    bc.clk.resize(G);
    bc.adv.resize(G);
    bc.nadv.resize(G + 1);
    int64_t c = e->clock, g = 0;
    std::vector<int64_t> tmp;
    for (const PushChunk& ch : e->pending) {
        const int64_t* ts = ch.ts.data();
        if (ch.device) {  // device-resident timestamps: read back (only apps with absent states build a clock)
            tmp.resize(ch.n);
            if (ch.n) HIPCHECK(hipMemcpy(tmp.data(), ch.d_ts, ch.n * 8, hipMemcpyDeviceToHost));
            ts = tmp.data();
        }
        for (int64_t r = 0; r < ch.n; ++r, ++g) {
            const int64_t t = ts[r];
            if (playback) {
                bc.adv[g] = !ch.no_adv && t >= c;
                if (bc.adv[g]) c = t;
            } else {
                bc.adv[g] = ch.stream == -1;  // advance_time points only
                if (ch.stream == -1 && t > c) c = t;
            }
            bc.clk[g] = c;
        }
    }
    bc.nadv[G] = (uint32_t)G;
    for (int64_t x = G - 1; x >= 0; --x) bc.nadv[x] = bc.adv[x] ? (uint32_t)x : bc.nadv[x + 1];
    int64_t* dc = (int64_t*)e->d_clk.ensure((size_t)std::max<int64_t>(G, 1) * 8);
    uint32_t* dn = (uint32_t*)e->d_nadv.ensure((size_t)(G + 1) * 4);
    if (G) HIPCHECK(hipMemcpyAsync(dc, bc.clk.data(), G * 8, hipMemcpyHostToDevice, e->stream));
    HIPCHECK(hipMemcpyAsync(dn, bc.nadv.data(), (G + 1) * 4, hipMemcpyHostToDevice, e->stream));
}

void resolve_staged(sdg_engine* e);

int do_flush(sdg_engine* e) {
    if (e->compile_only) throw DeviceError("engine was compiled with SDG_COMPILE_ONLY");
    HIPCHECK(hipSetDevice(e->device));
    e->stats.events = e->stats.matches = 0;
    e->stats.ms_keygroup = e->stats.ms_match = e->stats.ms_total = 0;
    e->stats.keygroup_launches = e->stats.match_launches = 0;
    e->stats.overflow = 0;
    e->stats.ms_kg_hist = e->stats.ms_kg_prefix = e->stats.ms_kg_scatter = 0;
    e->stats.ms_chain_carry = e->stats.ms_chain_match = e->stats.ms_chain_emit = 0;
    e->stats.ms_nfa = e->stats.ms_nfa_kernel = e->stats.ms_sched_host = 0;
    e->stats.arena_growths = 0;
    e->stats.carry_in = e->stats.carry_out = 0;
    e->stats.arena_slots = 0;
    e->stats.fused_ovf = 0;
    e->stats.sched_fires = e->stats.sched_shifted = e->stats.sched_host_keys = e->stats.sched_rerun_keys = 0;
    e->stats.sched_exact_passes = 0;
    e->stats.sorted_view = 0;
    e->stats.sub_batches = 0;
    e->stats.spilled_keys = 0;
    e->stats.host_rows = 0;
    // a flush consumes its batch whether or not it succeeds: a failing query must not make the next flush
    // replay the events onto the queries that already committed them. The batch's positions and its clock are
    // consumed with it: queries that committed before a failing one hold carries, arenas and scheduler state
    // stamped with positions [seq, seq + G) and the batch's clock, so the next flush starts after them
    struct Consume {
        sdg_engine* e;
        int64_t G = 0;
        bool clock_built = false;
        ~Consume() {
            if (clock_built && G > 0) e->clock = e->bc.clk[G - 1];
            e->seq += G;
            e->pending.clear();
            e->pending_n = 0;
            for (Stage& S : e->stage) {
                S.n = 0;
                std::fill(S.has_nulls.begin(), S.has_nulls.end(), 0);
            }
            std::fill(e->host_pending.begin(), e->host_pending.end(), 0);
        }
    } consume{e};
    resolve_staged(e);
    int64_t G = 0;
    for (auto& c : e->pending) G += c.n;
    consume.G = G;
    e->flush_G = G;
    if (G >= (int64_t)0xFFFFFFF0) throw CompileError(SDG_ERR_CAPACITY, "a flush holds more than 2^32 - 16 events");
    if (e->any_sched || e->any_purge) {
        build_clock(e, G);
        consume.clock_built = true;
    }
    for (auto& q : e->qs) {
        drain(e, *q);  // earlier unpolled results go to the backlog first
        if (q->hq.plan.purge && q->purge_first == INT64_MIN) {  // the partition's first event: its clock reading
            int64_t g = 0;
            for (const PushChunk& ch : e->pending) {
                const auto& ss = q->hq.streams;
                if (ch.stream >= 0 && std::find(ss.begin(), ss.end(), ch.stream) != ss.end() && ch.n > 0) {
                    q->purge_first = e->bc.clk[g];
                    break;
                }
                if (ch.stream == -2) {
                    int64_t r = 0;
                    while (r < ch.n && std::find(ss.begin(), ss.end(), ch.rstream[r]) == ss.end()) ++r;
                    if (r < ch.n) {
                        q->purge_first = e->bc.clk[g + r];
                        break;
                    }
                }
                g += ch.n;
            }
        }
        flush_query(e, *q);
    }
    e->stats.ms_total = e->stats.ms_keygroup + e->stats.ms_match;
    return SDG_OK;
}

// ---- snapshot / restore ------------------------------------------------------------------------------------
// SiddhiAppRuntime.snapshot() / restore(byte[]) (core/SiddhiAppRuntimeImpl.java:677-737) collect every
// StateHolder's state (StreamPreStateProcessor.java:450-469, CountPreStateProcessor.java:206-219,
// AbsentStreamPreStateProcessor.java:328-341, the schedulers, the selector's aggregators). Here that state is what
// outlives a flush: the chain queries' carried partials, the generic NFA's per-key arenas (the StreamPreStates,
// committed copies), the scheduler model, the per-key aggregator states, the key dictionaries, the string table,
// the position counter and the clock. The format is this engine's own (the reference's is Java serialisation);
// restore is behavioural: the restored engine continues exactly as the one snapshotted would have.
struct SnapW {
    std::vector<uint8_t>& o;
    template <class T>
    void put(const T& v) {
        const uint8_t* b = (const uint8_t*)&v;
        o.insert(o.end(), b, b + sizeof(T));
    }
    void bytes(const void* p, size_t n) {
        put<uint64_t>(n);
        o.insert(o.end(), (const uint8_t*)p, (const uint8_t*)p + n);
    }
    template <class T>
    void vec(const std::vector<T>& v) { bytes(v.data(), v.size() * sizeof(T)); }
    void str(const std::string& s) { bytes(s.data(), s.size()); }
    void dev(const void* d, size_t n, hipStream_t st) {  // a device buffer's first n bytes
        put<uint64_t>(n);
        const size_t at = o.size();
        o.resize(at + n);
        if (n) HIPCHECK(hipMemcpyAsync(o.data() + at, d, n, hipMemcpyDeviceToHost, st));
        if (n) HIPCHECK(hipStreamSynchronize(st));
    }
};
struct SnapR {
    const uint8_t* p;
    const uint8_t* end;
    template <class T>
    T get() {
        if (p + sizeof(T) > end) throw CompileError(SDG_ERR_ARG, "snapshot is truncated");
        T v;
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    const uint8_t* bytes(size_t* n) {
        *n = get<uint64_t>();
        if (*n > (size_t)(end - p)) throw CompileError(SDG_ERR_ARG, "snapshot is truncated");
        const uint8_t* r = p;
        p += *n;
        return r;
    }
    template <class T>
    void vec(std::vector<T>& v) {
        size_t n;
        const uint8_t* b = bytes(&n);
        v.resize(n / sizeof(T));
        std::memcpy(v.data(), b, v.size() * sizeof(T));
    }
    std::string str() {
        size_t n;
        const uint8_t* b = bytes(&n);
        return std::string((const char*)b, n);
    }
    void dev(DevBuf& d, hipStream_t st) {  // into a device buffer (allocated to at least the size)
        size_t n;
        const uint8_t* b = bytes(&n);
        void* x = d.ensure(n);
        if (n) HIPCHECK(hipMemcpyAsync(x, b, n, hipMemcpyHostToDevice, st));
        if (n) HIPCHECK(hipStreamSynchronize(st));
    }
};
// "SSDGSNP2": format 2 (round 4 on: spilled-key host arenas and the broadcast PartitionKeyOrder per query). Blobs of
// format 1 (earlier builds) are rejected with a version error instead of being misread
constexpr uint64_t SNAP_MAGIC = 0x32504e5347445353ull;      // "SSDGSNP2"
constexpr uint64_t SNAP_MAGIC_V1 = 0x31504e5347445353ull;   // "SSDGSNP1"
}  // namespace
void sdg::PartitionKeyOrder::throw_corrupt() { throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (partition keys)"); }
namespace {

void snapshot(sdg_engine* e, std::vector<uint8_t>& out) {
    out.clear();
    SnapW w{out};
    hipStream_t st = e->stream;
    w.put(SNAP_MAGIC);
    w.put(e->app_hash);
    w.put(e->seq);
    w.put(e->clock);
    w.put<uint64_t>(e->strings.strs.size());
    for (auto& x : e->strings.strs) w.str(x);
    w.put<uint32_t>((uint32_t)e->qs.size());
    for (auto& qp : e->qs) {
        QueryRt& q = *qp;
        const Plan& P = q.hq.plan;
        w.put<int32_t>(P.chain);
        w.put<uint8_t>(q.replay_carries);
        w.put<uint8_t>(q.carry_nullable);
        // carried partials (chain path): the committed buffer's n records, SoA
        const QueryRt::Carry& c = q.carry[q.cur];
        const int nc = std::max(P.n_cols, 1);
        w.put<int64_t>(c.n);
        if (c.n > 0) {
            w.dev(c.key.p, (size_t)c.n * 4, st);
            w.dev(c.ts.p, (size_t)c.n * 8, st);
            w.dev(c.seq.p, (size_t)c.n * 8, st);
            for (int k = 0; k < nc; ++k) w.dev((const int64_t*)c.vals.p + (size_t)k * c.cap, (size_t)c.n * 8, st);
            w.dev(c.nulls.p, (size_t)c.n * 4, st);
        }
        // key dictionaries (numeric partition values; string keys use the string table)
        w.vec(q.intkeys.k);
        w.vec(q.intkeys.v);
        w.put<uint64_t>(q.intkeys.n);
        w.put<uint64_t>(q.keystr.size());
        for (auto& x : q.keystr) w.str(x);
        w.vec(q.key_hash);
        if (q.broadcast) q.korder.save(w);
        // generic NFA: layout + both arena copies + the committed-copy bits
        w.put(q.L);
        w.put<int64_t>(q.arena_keys);
        if (q.arena_keys > 0) {
            w.dev(q.arena.p, (size_t)(q.arena_keys * q.L.bytes), st);
            w.dev(q.arena2.p, (size_t)(q.arena_keys * q.L.bytes), st);
            w.dev(q.cur_bits.p, (size_t)q.arena_keys, st);
        }
        // reclaiming queries: the key -> slot map, idle records, the slots' keys and the free stack
        w.put<uint8_t>(q.reclaim);
        if (q.reclaim) {
            const size_t ib = (size_t)nfa::idle_bytes(P.n_states);
            w.put<int64_t>(q.map_keys);
            if (q.map_keys > 0) {
                w.dev(q.slot_of.p, (size_t)q.map_keys * 4, st);
                w.dev(q.idle_rec.p, (size_t)q.map_keys * ib, st);
            }
            if (q.arena_keys > 0) {
                w.dev(q.slot_key.p, (size_t)q.arena_keys * 4, st);
                w.dev(q.free_slots.p, (size_t)q.arena_keys * 4, st);
                w.dev(q.pool_ctr.p, 4, st);
            }
        }
        // spilled keys: their host arenas (32-bit layouts)
        w.put<uint64_t>(q.spill.size());
        for (const auto& kv : q.spill) {
            w.put<uint32_t>(kv.first);
            w.put<int32_t>(kv.second.L.ns);
            w.put<int64_t>(kv.second.purge_last);
            w.vec(kv.second.arena);
        }
        w.put<int64_t>(q.purge_first);
        if (P.purge && q.arena_keys > 0) w.dev(q.last_seen.p, (size_t)q.arena_keys * 8, st);
        // selector aggregators per key
        w.put<int64_t>(q.agg_keys);
        if (q.agg_keys > 0) w.dev(q.agg_state.p, (size_t)q.agg_keys * (size_t)std::max(P.n_agg, 1) * 16, st);
        // register sequence kernel: the per-key partials (SoA, stride s3_kcap)
        w.put<int64_t>(q.s3_kcap);
        if (q.s3_kcap > 0) {
            w.dev(q.s3_hdr.p, (size_t)q.s3_kcap * 4, st);
            w.dev(q.s3_pn.p, (size_t)q.s3_kcap * 4, st);
            w.dev(q.s3_qn.p, (size_t)q.s3_kcap * 4, st);
            w.dev(q.s3_vals.p, (size_t)q.s3_kcap * 8 * 6 * q.s3.nc, st);
            w.dev(q.s3_ts.p, (size_t)q.s3_kcap * 16, st);
        }
        q.sim.save(out);
    }
}

// restore in two phases, like the reference (which deserialises the whole snapshot before touching a state): the
// blob is parsed and validated completely first (device payloads stay as views into it), then applied. A truncated
// or corrupt blob throws before any engine state changed.
struct SnapView {
    const uint8_t* p = nullptr;
    size_t n = 0;
};
struct SnapStage {
    int32_t chain = 0;
    bool replay = false, nullable = false;
    int64_t cn = 0;
    SnapView ckey, cts, cseq, cnulls;
    std::vector<SnapView> cvals;
    std::vector<int64_t> ik;
    std::vector<uint32_t> iv;
    uint64_t in = 0;
    std::vector<std::string> keystr;
    std::vector<int32_t> key_hash;
    PartitionKeyOrder korder;
    nfa::Layout L{};
    int64_t arena_keys = 0;
    SnapView arena, arena2, cur_bits, last_seen, agg;
    bool reclaim = false;
    int64_t map_keys = 0;
    SnapView slot_of, idle_rec, slot_key, free_slots, pool_ctr;
    int64_t purge_first = INT64_MIN, agg_keys = 0;
    int64_t s3_kcap = 0;
    SnapView s3_hdr, s3_pn, s3_qn, s3_vals, s3_ts;
    SchedSim sim;
    std::map<uint32_t, QueryRt::Spilled> spill;
};
struct SnapParsed {
    int64_t seq = 0, clock = 0;
    Interner strings;
    std::vector<SnapStage> stg;  // per query (device payloads are views into the blob)
};

void parse_snapshot(sdg_engine* e, const uint8_t* data, size_t len, SnapParsed& out) {
    SnapR r{data, data + len};
    const uint64_t magic = r.get<uint64_t>();
    if (magic == SNAP_MAGIC_V1)
        throw CompileError(SDG_ERR_ARG, "snapshot format 1 (written by an earlier engine build) cannot be restored by "
                                        "this build (format 2)");
    if (magic != SNAP_MAGIC) throw CompileError(SDG_ERR_ARG, "not an engine snapshot");
    if (r.get<uint64_t>() != e->app_hash)
        throw CompileError(SDG_ERR_ARG, "the snapshot was taken from a different Siddhi app");  // CannotRestoreSiddhiAppStateException
    using View = SnapView;
    auto view = [&]() {
        View v;
        v.p = r.bytes(&v.n);
        return v;
    };
    using Stage = SnapStage;
    out.seq = r.get<int64_t>();
    out.clock = r.get<int64_t>();
    const uint64_t ns = r.get<uint64_t>();
    for (uint64_t i = 0; i < ns; ++i) out.strings.get(r.str());
    if (r.get<uint32_t>() != e->qs.size()) throw CompileError(SDG_ERR_ARG, "snapshot query count differs");
    std::vector<Stage>& stg = out.stg;
    stg.resize(e->qs.size());
    for (size_t qi = 0; qi < e->qs.size(); ++qi) {
        const Plan& P = e->qs[qi]->hq.plan;
        Stage& g = stg[qi];
        g.chain = r.get<int32_t>();
        g.replay = r.get<uint8_t>() != 0;
        g.nullable = r.get<uint8_t>() != 0;
        const int nc = std::max(P.n_cols, 1);
        g.cn = r.get<int64_t>();
        if (g.cn < 0) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (carry count)");
        if (g.cn > 0) {
            g.ckey = view();
            g.cts = view();
            g.cseq = view();
            for (int k = 0; k < nc; ++k) g.cvals.push_back(view());
            g.cnulls = view();
            bool ok = g.ckey.n == (size_t)g.cn * 4 && g.cts.n == (size_t)g.cn * 8 && g.cseq.n == (size_t)g.cn * 8 &&
                      g.cnulls.n == (size_t)g.cn * 4;
            for (const View& v : g.cvals) ok = ok && v.n == (size_t)g.cn * 8;
            if (!ok) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (carried partials)");
        }
        r.vec(g.ik);
        r.vec(g.iv);
        g.in = r.get<uint64_t>();
        const uint64_t nks = r.get<uint64_t>();
        if (nks > (uint64_t)(r.end - r.p) / 8) throw CompileError(SDG_ERR_ARG, "snapshot is truncated");
        g.keystr.resize(nks);
        for (auto& x : g.keystr) x = r.str();
        r.vec(g.key_hash);
        if (e->qs[qi]->broadcast) g.korder.load(r);
        g.L = r.get<nfa::Layout>();
        g.arena_keys = r.get<int64_t>();
        if (g.arena_keys < 0) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (arena keys)");
        if (g.arena_keys > 0) {
            g.arena = view();
            g.arena2 = view();
            g.cur_bits = view();
            if (g.arena.n != (size_t)(g.arena_keys * g.L.bytes) || g.arena2.n != g.arena.n || g.cur_bits.n != (size_t)g.arena_keys)
                throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (arenas)");
        }
        g.reclaim = r.get<uint8_t>() != 0;
        if (g.reclaim != e->qs[qi]->reclaim) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (arena mode)");
        if (g.reclaim) {
            const size_t ib = (size_t)nfa::idle_bytes(P.n_states);
            g.map_keys = r.get<int64_t>();
            if (g.map_keys < 0) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (key map)");
            if (g.map_keys > 0) {
                g.slot_of = view();
                g.idle_rec = view();
                if (g.slot_of.n != (size_t)g.map_keys * 4 || g.idle_rec.n != (size_t)g.map_keys * ib)
                    throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (key map)");
            }
            if (g.arena_keys > 0) {
                g.slot_key = view();
                g.free_slots = view();
                g.pool_ctr = view();
                if (g.slot_key.n != (size_t)g.arena_keys * 4 || g.free_slots.n != g.slot_key.n || g.pool_ctr.n != 4)
                    throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (arena slots)");
            }
        }
        const uint64_t nsp = r.get<uint64_t>();
        if (nsp > (uint64_t)(r.end - r.p) / 16) throw CompileError(SDG_ERR_ARG, "snapshot is truncated");
        for (uint64_t i = 0; i < nsp; ++i) {
            const uint32_t k = r.get<uint32_t>();
            const int32_t sns = r.get<int32_t>();
            if (sns <= 0 || sns > (1 << 22)) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (spilled key)");
            QueryRt::Spilled& sp = g.spill[k];
            sp.L = nfa::make_layout<int32_t>(P.n_states, std::max(P.n_cols, 1), sns, P.n_sched);
            sp.purge_last = r.get<int64_t>();
            r.vec(sp.arena);
            if ((int64_t)sp.arena.size() != sp.L.bytes) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (spilled key)");
        }
        g.purge_first = r.get<int64_t>();
        if (P.purge && g.arena_keys > 0) g.last_seen = view();
        g.agg_keys = r.get<int64_t>();
        if (g.agg_keys > 0) g.agg = view();
        g.s3_kcap = r.get<int64_t>();
        if (g.s3_kcap < 0 || (g.s3_kcap > 0 && !e->qs[qi]->seq3)) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (sequence state)");
        if (g.s3_kcap > 0) {
            g.s3_hdr = view();
            g.s3_pn = view();
            g.s3_qn = view();
            g.s3_vals = view();
            g.s3_ts = view();
            const size_t kc = (size_t)g.s3_kcap;
            if (g.s3_hdr.n != kc * 4 || g.s3_pn.n != kc * 4 || g.s3_qn.n != kc * 4 ||
                g.s3_vals.n != kc * 8 * 6 * (size_t)e->qs[qi]->s3.nc || g.s3_ts.n != kc * 16)
                throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (sequence state)");
        }
        g.sim.setup(P.n_sched, P.partitioned, !P.playback);
        r.p = g.sim.load(r.p, r.end);
    }
    if (r.p != r.end) throw CompileError(SDG_ERR_ARG, "snapshot has trailing bytes");
}

void restore(sdg_engine* e, const uint8_t* data, size_t len) {
    SnapParsed parsed;
    parse_snapshot(e, data, len, parsed);
    std::vector<SnapStage>& stg = parsed.stg;
    using Stage = SnapStage;
    // ---- apply ------------------------------------------------------------------------------------------
    hipStream_t st = e->stream;
    auto up = [&](DevBuf& d, const SnapView& v) {
        void* x = d.ensure(v.n);
        if (v.n) HIPCHECK(hipMemcpyAsync(x, v.p, v.n, hipMemcpyHostToDevice, st));
    };
    for (size_t qi = 0; qi < e->qs.size(); ++qi) {
        QueryRt& q = *e->qs[qi];
        Plan& P = q.hq.plan;
        Stage& g = stg[qi];
        P.chain = g.chain;
        q.spill.swap(g.spill);
        q.spill_runs.clear();
        q.replay_carries = g.replay;
        q.carry_nullable = g.nullable;
        const int nc = std::max(P.n_cols, 1);
        q.cur = 0;
        q.carry[1].n = 0;
        QueryRt::Carry& c = q.carry[0];
        c.n = g.cn;
        if (c.n > 0) {
            c.cap = c.n;
            up(c.key, g.ckey);
            up(c.ts, g.cts);
            up(c.seq, g.cseq);
            c.vals.ensure((size_t)nc * c.n * 8);
            for (int k = 0; k < nc; ++k)
                HIPCHECK(hipMemcpyAsync((int64_t*)c.vals.p + (size_t)k * c.cap, g.cvals[k].p, g.cvals[k].n,
                                        hipMemcpyHostToDevice, st));
            up(c.nulls, g.cnulls);
        }
        q.intkeys.k = std::move(g.ik);
        q.intkeys.v = std::move(g.iv);
        q.intkeys.n = (size_t)g.in;
        q.keystr = std::move(g.keystr);
        q.keydict.clear();
        q.kt_cap = 0;  // the device key table is rebuilt from the dictionary on the next device-resident batch
        q.kt_synced = 0;
        if (q.key_class != KC_INT)
            for (size_t i = 0; i < q.keystr.size(); ++i) q.keydict[q.keystr[i]] = (uint32_t)i;
        q.key_hash = std::move(g.key_hash);
        q.korder = std::move(g.korder);
        q.L = g.L;
        q.arena_keys = g.arena_keys;
        if (q.arena_keys > 0) {
            up(q.arena, g.arena);
            up(q.arena2, g.arena2);
            up(q.cur_bits, g.cur_bits);
            q.ran_bits.ensure((size_t)q.arena_keys);
            HIPCHECK(hipMemsetAsync(q.ran_bits.p, 0, (size_t)q.arena_keys, st));
        }
        if (q.reclaim) {
            q.map_keys = g.map_keys;
            if (q.map_keys > 0) {
                up(q.slot_of, g.slot_of);
                up(q.idle_rec, g.idle_rec);
            }
            if (q.arena_keys > 0) {
                up(q.slot_key, g.slot_key);
                up(q.free_slots, g.free_slots);
                q.pool_ctr.ensure(16);
                HIPCHECK(hipMemsetAsync(q.pool_ctr.p, 0, 16, st));
                HIPCHECK(hipMemcpyAsync(q.pool_ctr.p, g.pool_ctr.p, 4, hipMemcpyHostToDevice, st));
                HIPCHECK(hipMemsetAsync(q.init_from.ensure((size_t)q.arena_keys), 0, (size_t)q.arena_keys, st));
                HIPCHECK(hipMemsetAsync(q.releasable.ensure((size_t)q.arena_keys), 0, (size_t)q.arena_keys, st));
                q.idle_out.ensure((size_t)q.arena_keys * nfa::idle_bytes(P.n_states));
            }
        }
        q.purge_first = g.purge_first;
        if (P.purge && q.arena_keys > 0) up(q.last_seen, g.last_seen);
        q.agg_keys = g.agg_keys;
        if (q.agg_keys > 0) up(q.agg_state, g.agg);
        q.s3_kcap = g.s3_kcap;
        if (q.s3_kcap > 0) {
            up(q.s3_hdr, g.s3_hdr);
            up(q.s3_pn, g.s3_pn);
            up(q.s3_qn, g.s3_qn);
            up(q.s3_vals, g.s3_vals);
            up(q.s3_ts, g.s3_ts);
        }
        q.sim = std::move(g.sim);
        HIPCHECK(hipStreamSynchronize(st));  // the views point into the caller's blob
    }
    e->seq = parsed.seq;
    e->clock = parsed.clock;
    e->strings = std::move(parsed.strings);
}

// ---- snapshot -> the reference's state maps ------------------------------------------------------------------
// A snapshot blob decoded into what SnapshotService would collect from the pattern processors of the same app:
// per query, per partition key, per processor (stateId) the StreamPreState.snapshot() map
// (StreamPreStateProcessor.java:450-459: FirstEvent, PendingStateEventList, NewAndEveryStateEventList,
// Initialized, Started) plus the subclass fields (CountPreStateProcessor.java:206-212, AbsentStreamPreStateProcessor
// .java:328-334, AbsentLogicalPreStateProcessor.java:407-413). JSON, in the layout of the oracle's orc_state_dump:
//   {"queries":[{"name":..,"form":..,"states":{"<key>":{"<stateId>":{..map..}}}}]}
//   StateEvent = {"ts":..,"type":..,"events":[null | [{"ts":..,"data":{"<attribute index>":v}} ..] per position]}
// A StreamEvent holds the attributes the query reads (the arena keeps no others). States a holder would destroy
// (canDestroy) and keys left with none are omitted. "form" says how exact the map is:
//   "arena"     the generic NFA's arenas ARE these maps (nfa.h PState = StreamPreState, SE = StateEvent, the
//               Node chain = the StreamEvent chain of a position): exact;
//   "chain"     the fused path keeps only the pending partials (e1 events, in arrival order): the map is given as
//               the next event's updateState() sees it -- NewAndEvery merged into Pending, the start state's seed
//               with timestamp -1 -- and only for the keys holding partials (a key whose only state is the seed
//               equals a fresh key);
// A query on the sequence register kernel (seq3.hip) is refused with SDG_ERR_UNSUPPORTED (its registers keep
// e2[0] / e2[last] only; SDG_NO_SEQ3 runs the query on the arenas).
struct StateJson {
    std::string o;
    void str(const std::string& s) {
        o += '"';
        for (unsigned char c : s) {
            if (c == '"' || c == '\\') {
                o += '\\';
                o += (char)c;
            } else if (c < 0x20) {
                char b[8];
                std::snprintf(b, sizeof b, "\\u%04x", c);
                o += b;
            } else {
                o += (char)c;
            }
        }
        o += '"';
    }
    void real(double x) {
        if (x != x) { o += "\"NaN\""; return; }
        if (std::isinf(x)) { o += x > 0 ? "\"Infinity\"" : "\"-Infinity\""; return; }
        char b[40];
        std::snprintf(b, sizeof b, "%.17g", x);
        o += b;
    }
    void val(uint8_t kind, int64_t v, bool null, const Interner& S) {
        if (null) { o += "null"; return; }
        switch (kind) {
            case VK_I32: o += std::to_string((int32_t)v); break;
            case VK_I64: o += std::to_string(v); break;
            case VK_F32: {
                const uint32_t u = (uint32_t)v;
                float f;
                std::memcpy(&f, &u, 4);
                real((double)f);
                break;
            }
            case VK_F64: {
                double d;
                std::memcpy(&d, &v, 8);
                real(d);
                break;
            }
            case VK_BOOL: o += v ? "true" : "false"; break;
            default: {
                const uint32_t id = (uint32_t)v;
                str(id < S.strs.size() ? S.strs[id] : std::string());
            }
        }
    }
    void flag(const char* name, bool b) { o += std::string(",\"") + name + "\":" + (b ? "true" : "false"); }
};

// one stream event of position p: the query's columns of that position's stream, by attribute index
void state_event_data(StateJson& J, const HostQuery& h, int p, const int64_t* vals, uint32_t nullmask,
                      const Interner& S) {
    const Plan& P = h.plan;
    const int qp = h.stream_pos(P.st[p].stream);
    J.o += "{";
    bool first = true;
    for (int c = 0; c < P.n_cols; ++c) {
        const int ai = qp >= 0 && qp < (int)h.col_attr.size() && c < (int)h.col_attr[qp].size() ? h.col_attr[qp][c] : -1;
        if (ai < 0) continue;
        if (!first) J.o += ',';
        first = false;
        J.o += '"' + std::to_string(ai) + "\":";
        J.val(P.col_kind[c], vals[c], (nullmask >> c) & 1u, S);
    }
    J.o += "}";
}

template <class IX>
void state_maps_of_key(StateJson& J, const HostQuery& h, const nfa::Layout& L, uint8_t* base, const Interner& S) {
    const Plan& P = h.plan;
    nfa::CtxT<true, IX> c;
    c.P = &P;
    c.L = L;
    c.base = base;
    auto se_json = [&](IX s) {
        const auto& e = c.se(s);
        J.o += "{\"ts\":" + std::to_string(e.ts) + ",\"type\":" + std::to_string((int)e.type) + ",\"events\":[";
        const IX* sl = c.slots(s);
        for (int p = 0; p < L.n_states; ++p) {
            if (p) J.o += ',';
            if (sl[p] == (IX)nfa::NIL) {
                J.o += "null";
                continue;
            }
            J.o += '[';
            int guard = 0;
            for (IX n = sl[p]; n != (IX)nfa::NIL; n = c.nd(n).next) {
                if (guard++ > L.nn) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (event chain)");
                if (guard > 1) J.o += ',';
                const IX r = c.nd(n).rec;
                J.o += "{\"ts\":" + std::to_string(c.rc(r).ts) + ",\"data\":";
                state_event_data(J, h, p, c.vals(r), c.rc(r).nullmask, S);
                J.o += '}';
            }
            J.o += ']';
        }
        J.o += "]}";
    };
    bool first = true;
    for (int p = 0; p < L.n_states; ++p) {
        const auto& st = c.ps(p);
        if (st.pn == 0 && st.nw == 0 && !st.initialized && st.last_arrival == 0) continue;  // canDestroy
        if (!first) J.o += ',';
        first = false;
        J.o += '"' + std::to_string(p) + "\":{\"FirstEvent\":null,\"PendingStateEventList\":[";
        for (int j = 0; j < st.pn; ++j) {
            if (j) J.o += ',';
            se_json(c.pend(p)[j]);
        }
        J.o += "],\"NewAndEveryStateEventList\":[";
        for (int j = 0; j < st.nw; ++j) {
            if (j) J.o += ',';
            se_json(c.newe(p)[j]);
        }
        J.o += ']';
        const StateRow& row = P.st[p];
        J.flag("Initialized", st.initialized);
        // partitionCreated() sets `started` on every startup processor, but a non-start one's state is empty then
        // and its holder destroys it on return (canDestroy), so the reference never holds started == true there;
        // the arena keeps the bit (nothing reads it again)
        J.flag("Started", st.started && row.is_start);
        if (row.kind == PK_COUNT) {
            J.flag("SuccessCondition", st.success);
            J.flag("StartStateReset", st.start_reset);
        } else if (row.kind == PK_LOGICAL && row.absent) {
            J.flag("IsActive", st.active);
            J.o += ",\"LastArrivalTime\":" + std::to_string(st.last_arrival);
        } else if (row.kind == PK_ABSENT) {
            J.flag("IsActive", st.active);
            J.o += ",\"LastScheduledTime\":" + std::to_string(st.last_sched);
        }
        J.o += '}';
    }
}

void snapshot_states(sdg_engine* e, const SnapParsed& sp, std::string& out) {
    StateJson J;
    const Interner& S = sp.strings;
    J.o = "{\"queries\":[";
    for (size_t qi = 0; qi < e->qs.size(); ++qi) {
        const QueryRt& q = *e->qs[qi];
        const HostQuery& h = q.hq;
        const Plan& P = h.plan;
        const SnapStage& g = sp.stg[qi];
        if (qi) J.o += ',';
        J.o += "{\"name\":";
        J.str(h.name);
        // the register sequence kernel keeps a partial's e2[0] / e2[last] only, not the reference's count chain
        // (CountPreStateProcessor.java:206-219 + every pending StateEvent's chain, StreamPreStateProcessor.java:
        // 450-469): refused rather than decoded into a map that would differ
        if (q.seq3)
            throw CompileError(SDG_ERR_UNSUPPORTED, "query '" + h.name + "' runs on the register sequence kernel, whose "
                               "state keeps e2[0] / e2[last] of a count chain only; its StreamPreState maps cannot be "
                               "decoded (compile with SDG_NO_SEQ3 to keep the query on the arenas)");
        const char* form = (g.chain || g.cn > 0) ? "chain" : "arena";
        J.o += std::string(",\"form\":\"") + form + "\",\"states\":{";
        // key ids: the string table's ids for string partition values, else the query's own dictionary
        const int64_t K = !P.partitioned ? 1 : q.string_keys ? (int64_t)S.strs.size() : (int64_t)g.keystr.size();
        auto key_name = [&](int64_t k) {
            return !P.partitioned ? std::string() : q.string_keys ? S.strs[(size_t)k] : g.keystr[(size_t)k];
        };
        // per key JSON of its processors (keys sorted by name: the maps are unordered)
        std::map<std::string, std::string> keys;
        if (!q.seq3 && (g.chain || g.cn > 0)) {
            // carried partials per key, arrival order
            std::vector<std::vector<int64_t>> per(K);
            const int nc = std::max(P.n_cols, 1);
            for (int64_t i = 0; i < g.cn; ++i) {
                uint32_t k;
                std::memcpy(&k, g.ckey.p + i * 4, 4);
                if (!P.partitioned) k = 0;
                if ((int64_t)k >= K) throw CompileError(SDG_ERR_ARG, "snapshot is corrupt (carried partial key)");
                per[k].push_back(i);
            }
            auto rd = [](const SnapView& v, int64_t i) {
                int64_t x;
                std::memcpy(&x, v.p + i * 8, 8);
                return x;
            };
            for (int64_t k = 0; k < K; ++k) {
                // (a key without carried partials holds only the start state's seed, as a fresh key would: the
                // fused path keeps no record of it, so it is left out -- see "chain" above)
                if (per[k].empty()) continue;
                std::sort(per[k].begin(), per[k].end(), [&](int64_t a, int64_t b) { return rd(g.cseq, a) < rd(g.cseq, b); });
                StateJson kj;
                kj.o = "\"0\":{\"FirstEvent\":null,\"PendingStateEventList\":[],\"NewAndEveryStateEventList\":[{\"ts\":-1,"
                       "\"type\":0,\"events\":[";
                for (int p = 0; p < P.n_states; ++p) kj.o += p ? ",null" : "null";
                kj.o += "]}],\"Initialized\":true,\"Started\":false}";
                if (!per[k].empty()) {
                    kj.o += ",\"1\":{\"FirstEvent\":null,\"PendingStateEventList\":[";
                    std::vector<int64_t> vals(nc);
                    for (size_t j = 0; j < per[k].size(); ++j) {
                        const int64_t i = per[k][j];
                        const int64_t ts = rd(g.cts, i);
                        for (int cidx = 0; cidx < nc; ++cidx) vals[cidx] = rd(g.cvals[cidx], i);
                        uint32_t nm;
                        std::memcpy(&nm, g.cnulls.p + i * 4, 4);
                        if (j) kj.o += ',';
                        kj.o += "{\"ts\":" + std::to_string(ts) + ",\"type\":0,\"events\":[[{\"ts\":" + std::to_string(ts) +
                                ",\"data\":";
                        state_event_data(kj, h, 0, vals.data(), nm, S);
                        kj.o += "}]";
                        for (int p = 1; p < P.n_states; ++p) kj.o += ",null";
                        kj.o += "]}";
                    }
                    kj.o += "],\"NewAndEveryStateEventList\":[],\"Initialized\":false,\"Started\":false}";
                }
                keys[key_name(k)] = std::move(kj.o);
            }
        } else if (!q.seq3) {
            const nfa::Layout& L = g.L;
            std::vector<uint8_t> scratch;
            const int ib = nfa::idle_bytes(P.n_states);
            auto slot_of = [&](int64_t k) {
                int32_t so;
                std::memcpy(&so, g.slot_of.p + k * 4, 4);
                return so;
            };
            for (int64_t k = 0; k < K; ++k) {
                StateJson kj;
                auto sit = g.spill.find((uint32_t)k);
                if (sit != g.spill.end()) {  // spilled: its host arena (32-bit indices)
                    scratch.assign(sit->second.arena.begin(), sit->second.arena.end());
                    state_maps_of_key<int32_t>(kj, h, sit->second.L, scratch.data(), S);
                } else {
                    int64_t s = k;
                    bool idle = false;
                    if (g.reclaim) {
                        if (k >= g.map_keys) continue;
                        const int32_t so = slot_of(k);
                        if (so == -1 || so == -3) continue;
                        if (so == -2) idle = true;
                        else s = so;
                    }
                    if (!idle && s >= g.arena_keys) continue;
                    scratch.assign((size_t)L.bytes, 0);
                    if (idle) {
                        nfa::CtxT<true> c;
                        c.P = &P;
                        c.L = L;
                        c.base = scratch.data();
                        nfa::from_idle(c, g.idle_rec.p + k * ib);
                    } else {
                        const uint8_t cur = g.cur_bits.p[s];
                        std::memcpy(scratch.data(), (cur ? g.arena2.p : g.arena.p) + s * L.bytes, (size_t)L.bytes);
                    }
                    const nfa::KHead& kh = *(const nfa::KHead*)scratch.data();
                    if (!(kh.flags & 2)) continue;  // never initialised
                    state_maps_of_key<int16_t>(kj, h, L, scratch.data(), S);
                }
                if (!kj.o.empty()) keys[key_name(k)] = std::move(kj.o);
            }
        }
        bool first = true;
        for (auto& kv : keys) {
            if (!first) J.o += ',';
            first = false;
            J.str(kv.first);
            J.o += ":{" + kv.second + '}';
        }
        J.o += "}}";
    }
    J.o += "]}";
    out.swap(J.o);
}

template <class F>
int guarded(F f) {
    try {
        return f();
    } catch (const CompileError& ex) {
        return fail(ex.code, ex.what());
    } catch (const sql::Unsupported& ex) {
        return fail(SDG_ERR_UNSUPPORTED, ex.what());
    } catch (const sql::ParseError& ex) {
        return fail(SDG_ERR_PARSE, ex.what());
    } catch (const DeviceError& ex) {
        return fail(SDG_ERR_DEVICE, ex.what());
    } catch (const std::exception& ex) {
        return fail(SDG_ERR_ARG, ex.what());
    }
}

}  // namespace

extern "C" {

const char* sdg_last_error(void) { return g_err.c_str(); }

int sdg_compile(const char* text, const sdg_opts* opts, sdg_engine** out) {
    if (!text || !out) return fail(SDG_ERR_ARG, "null argument");
    *out = nullptr;
    return guarded([&]() {
        auto e = std::make_unique<sdg_engine>();
        e->app = sql::parse_app(text);
        e->app_hash = 1469598103934665603ull;
        for (const char* c = text; *c; ++c) e->app_hash = (e->app_hash ^ (uint8_t)*c) * 1099511628211ull;
        if (opts) {
            e->device = opts->device;
            if (opts->batch_capacity > 0) e->capacity = opts->batch_capacity;
            e->compile_only = (opts->flags & SDG_COMPILE_ONLY) != 0;
            e->force_generic = (opts->flags & SDG_FORCE_GENERIC) != 0;
            e->no_fused = (opts->flags & SDG_NO_FUSED) != 0;
            e->no_seq3 = (opts->flags & (SDG_NO_SEQ3 | SDG_FORCE_GENERIC)) != 0;
            e->sched_exact = (opts->flags & SDG_SCHED_EXACT) != 0 || getenv("SDG_SCHED_EXACT") != nullptr;
            e->sched_host = (opts->flags & SDG_SCHED_HOST) != 0;
            e->no_sorted = (opts->flags & SDG_NO_SORTED) != 0 || getenv("SDG_NO_SORTED") != nullptr;
        }
        if (opts && opts->max_partials > 0) {
            if (opts->max_partials > 4096) throw CompileError(SDG_ERR_ARG, "max_partials must be <= 4096");
            e->max_partials = opts->max_partials;
        }
        auto hqs = compile_app(e->app, e->strings);
        if (!e->compile_only) {
            int ndev = 0;
            if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
                throw DeviceError("no HIP device visible (the engine has no CPU fallback)");
            HIPCHECK(hipSetDevice(e->device));
            hipDeviceProp_t prop;
            HIPCHECK(hipGetDeviceProperties(&prop, e->device));
            if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
                throw DeviceError(std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
            int xccs = 0;  // the XCD-aware block remaps follow the device's XCD count (partition mode)
            if (hipDeviceGetAttribute(&xccs, hipDeviceAttributeNumberOfXccs, e->device) != hipSuccess) xccs = 1;
            if (const char* x = getenv("SDG_XCDS")) xccs = atoi(x);  // override (A/B)
            g_xcds = std::max(1, xccs);
            g_cus = std::max(1, prop.multiProcessorCount);
            if (getenv("SDG_VERBOSE"))
                fprintf(stderr, "[sdg] device %d: %s, %d CUs, %d XCDs\n", e->device, prop.gcnArchName,
                        prop.multiProcessorCount, g_xcds);
            HIPCHECK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
            HIPCHECK(hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking));
            for (auto& ev : e->ev) HIPCHECK(hipEventCreate(&ev));
            HIPCHECK(hipEventCreateWithFlags(&e->fork, hipEventDisableTiming));
            HIPCHECK(hipEventCreateWithFlags(&e->join, hipEventDisableTiming));
        }
        for (auto& h : hqs) {
            auto q = std::make_unique<QueryRt>();
            q->hq = std::move(h);
            if (e->force_generic) q->hq.plan.chain = 0;
            const Plan& P = q->hq.plan;
            q->broadcast = std::find(q->hq.key_attr.begin(), q->hq.key_attr.end(), -3) != q->hq.key_attr.end();
            q->ranked = q->broadcast || std::find(q->hq.key_attr.begin(), q->hq.key_attr.end(), -2) != q->hq.key_attr.end();
            q->L = nfa::make_layout(P.n_states, std::max(P.n_cols, 1), e->max_partials, P.n_sched);
            q->sim.setup(P.n_sched, P.partitioned, !P.playback);
            e->any_sched |= P.n_sched > 0;
            e->any_purge |= P.purge != 0;
            for (size_t i = 0; i < q->hq.key_kind.size(); ++i)
                if (q->hq.key_attr[i] >= 0 && q->hq.key_kind[i] != VK_STR) q->string_keys = false;
            q->key_class = P.partitioned && !q->hq.key_kind.empty() ? key_class_of(q->hq.key_kind[0]) : KC_NONE;
            for (size_t i = 0; i < q->hq.key_kind.size(); ++i)
                if (q->hq.key_attr[i] < 0 || key_class_of(q->hq.key_kind[i]) != q->key_class) q->key_class = KC_NONE;
            // arenas sized by live keys (nfa.h to_idle): partitioned generic-NFA queries without timers or @purge
            q->seq3 = !e->no_seq3 && !getenv("SDG_NO_SEQ3") && seq3_spec(q->hq, q->s3);
            q->reclaim = P.partitioned && !P.chain && !q->seq3 && P.n_sched == 0 && !P.purge && !getenv("SDG_NO_RECLAIM");
            if (!e->compile_only) upload_plan(e.get(), *q);
            e->qs.push_back(std::move(q));
        }
        for (auto& s : e->app.streams) {
            std::vector<int32_t> t;
            for (auto& a : s.attrs) t.push_back((int32_t)a.type);
            e->stream_types.push_back(t);
        }
        // streams whose host pushes go to HBM at push time: every query reading them takes device-resident batches
        // (one stream; no range partition; string keys or one class of value keys)
        e->stage.resize(e->stream_types.size());
        e->stage_ok.assign(e->stream_types.size(), 1);
        e->host_pending.assign(e->stream_types.size(), 0);
        for (auto& q : e->qs) {
            const HostQuery& h = q->hq;
            const bool ranged = std::find(h.key_attr.begin(), h.key_attr.end(), -2) != h.key_attr.end();
            const bool ok = h.streams.size() == 1 && !ranged && !q->broadcast &&
                            (!h.plan.partitioned || q->string_keys || q->key_class != KC_NONE);
            if (!ok)
                for (int s2 : h.streams) e->stage_ok[s2] = 0;
        }
        for (auto& q : e->qs) {
            e->out_types.push_back(q->hq.out_types);
            std::vector<const char*> nm;
            for (auto& s : q->hq.out_names) nm.push_back(s.c_str());
            e->out_names.push_back(nm);
        }
        *out = e.release();
        return SDG_OK;
    });
}

void sdg_destroy(sdg_engine* e) {
    if (!e) return;
    if (e->compile_only) {
        delete e;
        return;
    }
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    e->qs.clear();
    for (auto& ev : e->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : e->bounce_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->stream2) (void)hipStreamDestroy(e->stream2);
    if (e->fork) (void)hipEventDestroy(e->fork);
    if (e->join) (void)hipEventDestroy(e->join);
    delete e;
}

int sdg_snapshot(sdg_engine* e, const uint8_t** data, int64_t* len) {
    if (!e || !data || !len) return fail(SDG_ERR_ARG, "bad snapshot arguments");
    return guarded([&]() {
        if (e->compile_only) throw DeviceError("engine was compiled with SDG_COMPILE_ONLY");
        HIPCHECK(hipSetDevice(e->device));
        if (!e->pending.empty()) do_flush(e);  // persist(): what was sent before is processed first
        for (auto& q : e->qs) drain(e, *q);     // results produced so far stay queued for sdg_poll
        snapshot(e, e->snap);
        *data = e->snap.data();
        *len = (int64_t)e->snap.size();
        return (int)SDG_OK;
    });
}

int sdg_restore(sdg_engine* e, const uint8_t* data, int64_t len) {
    if (!e || !data || len < 0) return fail(SDG_ERR_ARG, "bad restore arguments");
    return guarded([&]() {
        if (e->compile_only) throw DeviceError("engine was compiled with SDG_COMPILE_ONLY");
        if (!e->pending.empty()) throw CompileError(SDG_ERR_ARG, "events are pending: flush before restoring");
        HIPCHECK(hipSetDevice(e->device));
        restore(e, data, (size_t)len);
        return (int)SDG_OK;
    });
}

int sdg_snapshot_states(sdg_engine* e, const uint8_t* data, int64_t len, const char** json, int64_t* json_len) {
    if (!e || !data || len < 0 || !json || !json_len) return fail(SDG_ERR_ARG, "bad snapshot_states arguments");
    return guarded([&]() {
        SnapParsed parsed;
        parse_snapshot(e, data, (size_t)len, parsed);
        snapshot_states(e, parsed, e->states_json);
        *json = e->states_json.c_str();
        *json_len = (int64_t)e->states_json.size();
        return (int)SDG_OK;
    });
}

int sdg_stream_index(sdg_engine* e, const char* sid) { return e && sid ? e->app.stream_index(sid) : -1; }

int sdg_stream_schema(sdg_engine* e, int s, int32_t* n, const int32_t** types) {
    if (!e || s < 0 || s >= (int)e->stream_types.size()) return fail(SDG_ERR_ARG, "bad stream index");
    *n = (int32_t)e->stream_types[s].size();
    *types = e->stream_types[s].data();
    return SDG_OK;
}

int sdg_num_queries(sdg_engine* e) { return e ? (int)e->qs.size() : 0; }
int sdg_query_flags(sdg_engine* e, int q) {
    if (!e || q < 0 || q >= (int)e->qs.size()) return -1;
    const Plan& P = e->qs[q]->hq.plan;
    return (P.partitioned ? SDG_Q_PARTITIONED : 0) | (P.n_sched > 0 ? SDG_Q_TIMERS : 0) |
           (e->qs[q]->broadcast ? SDG_Q_BROADCAST : 0);
}
int sdg_query_key_attr(sdg_engine* e, int q, int stream) {
    if (!e || q < 0 || q >= (int)e->qs.size()) return -1;
    const HostQuery& h = e->qs[q]->hq;
    const int qp = h.stream_pos(stream);
    if (qp < 0 || !h.plan.partitioned) return -1;
    return h.key_attr[qp];
}
int sdg_query_reads(sdg_engine* e, int q, int stream) {
    if (!e || q < 0 || q >= (int)e->qs.size()) return 0;
    return e->qs[q]->hq.stream_pos(stream) >= 0 ? 1 : 0;
}
int sdg_query_path(sdg_engine* e, int q) {
    if (!e || q < 0 || q >= (int)e->qs.size()) return -1;
    return e->qs[q]->hq.plan.chain ? 0 : e->qs[q]->seq3 ? 2 : 1;
}
const char* sdg_query_name(sdg_engine* e, int q) { return e->qs[q]->hq.name.c_str(); }
const char* sdg_query_target(sdg_engine* e, int q) { return e->qs[q]->hq.target.c_str(); }
int sdg_query_output_schema(sdg_engine* e, int q, int32_t* n, const int32_t** types, const char* const** names) {
    if (!e || q < 0 || q >= (int)e->qs.size()) return fail(SDG_ERR_ARG, "bad query index");
    *n = (int32_t)e->out_types[q].size();
    *types = e->out_types[q].data();
    *names = e->out_names[q].data();
    return SDG_OK;
}

uint32_t sdg_intern(sdg_engine* e, const char* s, size_t len) { return e->strings.get(std::string(s, len)); }
int sdg_intern_many(sdg_engine* e, int64_t n, const char* bytes, const int64_t* offsets, uint32_t* ids) {
    if (!e || n < 0 || (n > 0 && (!bytes || !offsets || !ids))) return fail(SDG_ERR_ARG, "bad intern arguments");
    return guarded([&]() {
        Interner& in = e->strings;
        in.strs.reserve(in.strs.size() + (size_t)n);
        in.ids.reserve(in.ids.size() + (size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            if (offsets[i + 1] < offsets[i]) throw std::invalid_argument("intern offsets decrease");
            ids[i] = in.get(std::string(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i])));
        }
        return (int)SDG_OK;
    });
}
const char* sdg_string(sdg_engine* e, uint32_t id) {
    return id < e->strings.strs.size() ? e->strings.strs[id].c_str() : nullptr;
}

namespace {
// a host push straight into HBM (the stream's staging columns): the flush then takes the zero-copy device path
// instead of re-assembling rows on the host (InputHandler.send -> pinned columnar batches, BASELINE north_star).
// Only when every query of the stream takes device-resident batches and the push has no null partition key.
// staged chunks back to host columns: a query's batch view is assembled on the host when a stream's rows mix staged
// and host pushes (a push with a null partition key, a mixed push)
void unstage(sdg_engine* e, int stream) {
    for (PushChunk& c : e->pending) {
        if (c.stage_off < 0 || (stream >= 0 && c.stream != stream)) continue;
        Stage& S = e->stage[c.stream];
        const auto& types = e->stream_types[c.stream];
        c.ts.resize(c.n);
        HIPCHECK(hipMemcpy(c.ts.data(), S.ts.as<int64_t>() + c.stage_off, (size_t)c.n * 8, hipMemcpyDeviceToHost));
        c.cols.assign(types.size(), {});
        c.nulls.assign(types.size(), {});
        for (size_t a = 0; a < types.size(); ++a) {
            const int w = width_of((uint8_t)types[a]);
            c.cols[a].resize((size_t)c.n * w);
            HIPCHECK(hipMemcpy(c.cols[a].data(), (const uint8_t*)S.cols[a].p + (size_t)c.stage_off * w, (size_t)c.n * w,
                               hipMemcpyDeviceToHost));
            if (S.has_nulls[a]) {
                c.nulls[a].resize((size_t)c.n);
                HIPCHECK(hipMemcpy(c.nulls[a].data(), (const uint8_t*)S.nulls[a].p + c.stage_off, (size_t)c.n,
                                   hipMemcpyDeviceToHost));
            }
        }
        c.device = false;
        c.stage_off = -1;
        e->host_pending[c.stream] = 1;
    }
}

// a pageable host buffer into HBM on the engine's stream: large ones through two pinned chunks, the threads' copy
// of chunk i+1 overlapping the DMA of chunk i (the runtime's pageable path copies on one thread). The source is
// free when the stream has caught up.
void h2d(sdg_engine* e, void* dst, const void* src, size_t bytes) {
    constexpr size_t CH = (size_t)32 << 20;
    static const bool direct = getenv("SDG_PAGEABLE") != nullptr;
    if (bytes < ((size_t)4 << 20) || direct) {
        HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream));
        return;
    }
    for (int k = 0; k < 2; ++k) {
        e->bounce[k].ensure(CH);
        if (!e->bounce_ev[k]) HIPCHECK(hipEventCreateWithFlags(&e->bounce_ev[k], hipEventDisableTiming));
    }
    size_t i = 0;
    for (size_t off = 0; off < bytes; off += CH, ++i) {
        const int k = (int)(i & 1);
        const size_t len = std::min(CH, bytes - off);
        HIPCHECK(hipEventSynchronize(e->bounce_ev[k]));  // the chunk's previous DMA has read it
        par_memcpy(e->bounce[k].p, (const uint8_t*)src + off, len);
        HIPCHECK(hipMemcpyAsync((uint8_t*)dst + off, e->bounce[k].p, len, hipMemcpyHostToDevice, e->stream));
        HIPCHECK(hipEventRecord(e->bounce_ev[k], e->stream));
    }
}

bool stage_push(sdg_engine* e, int stream, int64_t n, const int64_t* ts, const void* const* cols,
                const uint8_t* const* nulls, PushChunk& c) {
    if (e->compile_only || e->no_stage || getenv("SDG_NO_STAGE") || stream >= (int)e->stage_ok.size() ||
        !e->stage_ok[stream] || e->host_pending[stream])
        return false;
    const auto& types = e->stream_types[stream];
    for (auto& qp : e->qs) {  // null partition keys are dropped by the host path (PartitionStreamReceiver :262-272)
        const HostQuery& h = qp->hq;
        const int qpos = h.stream_pos(stream);
        if (qpos < 0 || !h.plan.partitioned) continue;
        const int ai = h.key_attr[qpos];
        if (ai >= 0 && nulls && nulls[ai])
            for (int64_t r = 0; r < n; ++r)
                if (nulls[ai][r]) {
                    unstage(e, stream);  // this push goes to the host: so do the stream's earlier ones
                    e->host_pending[stream] = 1;
                    return false;
                }
    }
    for (size_t a = 0; a < types.size(); ++a)
        if (!cols[a]) throw std::invalid_argument("missing column");
    Stage& S = e->stage[stream];
    if (S.cols.size() != types.size()) {
        S.cols = std::vector<DevBuf>(types.size());
        S.nulls = std::vector<DevBuf>(types.size());
        S.has_nulls.assign(types.size(), 0);
    }
    if (S.n + n > S.cap) {  // grow, keeping the rows staged so far
        const int64_t nc = std::max<int64_t>(S.n + n, 2 * S.cap);
        auto keep = [&](DevBuf& b, int w) {
            DevBuf nb;
            nb.ensure((size_t)nc * w);
            if (S.n) HIPCHECK(hipMemcpy(nb.p, b.p, (size_t)S.n * w, hipMemcpyDeviceToDevice));
            std::swap(nb.p, b.p);
            std::swap(nb.cap, b.cap);
        };
        keep(S.ts, 8);
        for (size_t a = 0; a < types.size(); ++a) {
            keep(S.cols[a], width_of((uint8_t)types[a]));
            if (S.has_nulls[a]) keep(S.nulls[a], 1);
        }
        S.cap = nc;
    }
    hipStream_t st = e->stream;
    h2d(e, S.ts.as<int64_t>() + S.n, ts, (size_t)n * 8);
    for (size_t a = 0; a < types.size(); ++a) {
        const int w = width_of((uint8_t)types[a]);
        h2d(e, (uint8_t*)S.cols[a].p + (size_t)S.n * w, cols[a], (size_t)n * w);
        bool any = false;
        if (nulls && nulls[a])
            for (int64_t r = 0; r < n && !any; ++r) any = nulls[a][r] != 0;
        if (any && !S.has_nulls[a]) {  // the first nulls of this attribute: earlier rows are not null
            S.nulls[a].ensure((size_t)S.cap);
            HIPCHECK(hipMemsetAsync(S.nulls[a].p, 0, (size_t)S.n, st));
            S.has_nulls[a] = 1;
        }
        if (any) h2d(e, (uint8_t*)S.nulls[a].p + S.n, nulls[a], (size_t)n);
        else if (S.has_nulls[a]) HIPCHECK(hipMemsetAsync((uint8_t*)S.nulls[a].p + S.n, 0, (size_t)n, st));
    }
    HIPCHECK(hipStreamSynchronize(st));  // the caller's buffers are free when the push returns
    c.device = true;
    c.stage_off = S.n;
    S.n += n;
    return true;
}

// staged chunks: their device pointers into the staging (stable from here to the end of the flush)
void resolve_staged(sdg_engine* e) {
    for (PushChunk& c : e->pending) {
        if (c.stage_off < 0) continue;
        Stage& S = e->stage[c.stream];
        c.d_ts = S.ts.as<int64_t>() + c.stage_off;
        const size_t na = S.cols.size();
        c.d_cols.assign(na, nullptr);
        c.d_nulls.assign(na, nullptr);
        for (size_t a = 0; a < na; ++a) {
            const int w = width_of((uint8_t)e->stream_types[c.stream][a]);
            c.d_cols[a] = (const uint8_t*)S.cols[a].p + (size_t)c.stage_off * w;
            if (S.has_nulls[a]) c.d_nulls[a] = (const uint8_t*)S.nulls[a].p + c.stage_off;
        }
    }
}

int push_host(sdg_engine* e, int stream, int64_t n, const int64_t* ts, const void* const* cols,
              const uint8_t* const* nulls, bool event_array) {
    if (!e || stream < 0 || stream >= (int)e->stream_types.size() || n < 0 || (n > 0 && !ts))
        return fail(SDG_ERR_ARG, "bad push arguments");
    return guarded([&]() {
        if (event_array && n > 1) {
            // PartitionStreamReceiver.receive(Event[]) (:176-188) of a stream with no partition key hands the WHOLE
            // chunk to each key in turn (key-major delivery); the engine's broadcast rows are event-major (one event
            // to every key, then the next), so a multi-event array on such a stream is refused, not reordered
            for (auto& qp : e->qs) {
                const int qpos = qp->hq.stream_pos(stream);
                if (qp->broadcast && qpos >= 0 && qp->hq.key_attr[qpos] == -3)
                    throw CompileError(SDG_ERR_UNSUPPORTED, "send(Event[]) of more than one event to stream '" +
                                                                e->app.streams[stream].id + "', which has no partition "
                                                                "key in partition query '" + qp->hq.name +
                                                                "' (key-major delivery of the chunk is not supported)");
            }
        }
        if (event_array && n > 0 && e->app.playback) {  // InputHandler.send(Event[]) :85-95: the clock first
            PushChunk a;                                  // moves to the last event's timestamp
            a.stream = -1;
            a.n = 1;
            a.device = false;
            a.ts.assign(1, ts[n - 1]);
            e->pending.push_back(std::move(a));
        }
        PushChunk c;
        c.stream = stream;
        c.n = n;
        c.device = false;
        c.no_adv = event_array;
        if (n > 0 && stage_push(e, stream, n, ts, cols, nulls, c)) {
            e->pending_n += n;
            e->pending.push_back(std::move(c));
            if (e->pending_n >= e->capacity) return do_flush(e);
            return (int)SDG_OK;
        }
        c.ts.assign(ts, ts + n);
        const auto& types = e->stream_types[stream];
        c.cols.resize(types.size());
        c.nulls.resize(types.size());
        for (size_t a = 0; a < types.size(); ++a) {
            int w = width_of((uint8_t)types[a]);
            if (n > 0 && !cols[a]) throw std::invalid_argument("missing column");
            c.cols[a].assign((const uint8_t*)cols[a], (const uint8_t*)cols[a] + n * w);
            if (nulls && nulls[a]) c.nulls[a].assign(nulls[a], nulls[a] + n);
        }
        e->pending_n += n;
        e->pending.push_back(std::move(c));
        if (e->pending_n >= e->capacity) return do_flush(e);
        return (int)SDG_OK;
    });
}
}  // namespace

int sdg_push(sdg_engine* e, int stream, int64_t n, const int64_t* ts, const void* const* cols,
             const uint8_t* const* nulls) {
    return push_host(e, stream, n, ts, cols, nulls, false);
}

int sdg_push_events(sdg_engine* e, int stream, int64_t n, const int64_t* ts, const void* const* cols,
                    const uint8_t* const* nulls) {
    return push_host(e, stream, n, ts, cols, nulls, true);
}

int sdg_push_mixed(sdg_engine* e, int64_t n, const int32_t* streams, const int64_t* ts, int32_t n_attrs,
                   const int64_t* const* slots, const uint8_t* const* nulls) {
    if (!e || n < 0 || (n > 0 && (!ts || !streams || !slots)) || n_attrs < 0) return fail(SDG_ERR_ARG, "bad push arguments");
    return guarded([&]() {
        if (!e->no_stage) {  // rows of several streams per push: host assembly from here on
            unstage(e, -1);
            e->no_stage = true;
        }
        PushChunk c;
        c.stream = -2;
        c.n = n;
        c.device = false;
        c.ts.assign(ts, ts + n);
        c.rstream.assign(streams, streams + n);
        int32_t na = 0;
        for (int64_t r = 0; r < n; ++r) {
            if (c.rstream[r] < 0 || c.rstream[r] >= (int)e->stream_types.size())
                throw std::invalid_argument("bad stream index in a mixed push");
            na = std::max<int32_t>(na, (int32_t)e->stream_types[c.rstream[r]].size());
        }
        if (na > n_attrs) throw std::invalid_argument("a row's stream has more attributes than n_attrs");
        c.cols.resize(na);
        c.nulls.resize(na);
        for (int32_t a = 0; a < na; ++a) {
            c.cols[a].assign((const uint8_t*)slots[a], (const uint8_t*)slots[a] + n * 8);
            if (nulls && nulls[a]) c.nulls[a].assign(nulls[a], nulls[a] + n);
        }
        e->pending_n += n;
        e->pending.push_back(std::move(c));
        if (e->pending_n >= e->capacity) return do_flush(e);
        return (int)SDG_OK;
    });
}

int sdg_push_device(sdg_engine* e, int stream, int64_t n, const int64_t* d_ts, const void* const* d_cols,
                    const uint8_t* const* d_nulls) {
    if (!e || stream < 0 || stream >= (int)e->stream_types.size() || n < 0)
        return fail(SDG_ERR_ARG, "bad push arguments");
    return guarded([&]() {
        if (e->compile_only) throw DeviceError("engine was compiled with SDG_COMPILE_ONLY");
        PushChunk c;
        c.stream = stream;
        c.n = n;
        c.device = true;
        c.d_ts = d_ts;
        size_t na = e->stream_types[stream].size();
        c.d_cols.assign(d_cols, d_cols + na);
        c.d_nulls.assign(na, nullptr);
        if (d_nulls)
            for (size_t a = 0; a < na; ++a) c.d_nulls[a] = d_nulls[a];
        e->pending_n += n;
        e->pending.push_back(std::move(c));
        return (int)SDG_OK;
    });
}

int64_t sdg_pending(sdg_engine* e) { return e ? e->pending_n : 0; }

int sdg_advance_time(sdg_engine* e, int64_t ts) {
    if (!e) return fail(SDG_ERR_ARG, "null engine");
    return guarded([&]() {
        PushChunk c;  // a position of its own in the next flush
        c.stream = -1;
        c.n = 1;
        c.device = false;
        c.ts.assign(1, ts);
        e->pending.push_back(std::move(c));
        return (int)SDG_OK;
    });
}

int sdg_start(sdg_engine* e, int64_t ts) {
    if (!e) return fail(SDG_ERR_ARG, "null engine");
    if (!e->app.playback && e->seq == 0 && e->pending.empty()) e->clock = ts;
    return SDG_OK;
}

int sdg_flush(sdg_engine* e) {
    if (!e) return fail(SDG_ERR_ARG, "null engine");
    return guarded([&]() { return do_flush(e); });
}

int sdg_sync(sdg_engine* e) {
    if (!e) return fail(SDG_ERR_ARG, "null engine");
    return guarded([&]() {
        HIPCHECK(hipStreamSynchronize(e->stream));
        return (int)SDG_OK;
    });
}

int sdg_poll(sdg_engine* e, int qi, sdg_out* out) {
    if (!e || qi < 0 || qi >= (int)e->qs.size() || !out) return fail(SDG_ERR_ARG, "bad poll arguments");
    return guarded([&]() {
        QueryRt& q = *e->qs[qi];
        const int na = q.hq.plan.n_user_out + q.hq.plan.n_list_cols;  // list elements kept for sdg_poll_list
        if (!e->compile_only) drain(e, q);
        if (q.del_n >= 0 && q.acc_ts.empty()) {  // pinned delivery: hand the buffer out as it is
            const int64_t n = q.del_n;
            const int nd = q.del_nu;
            q.del_cur ^= 1;
            q.del_n = -1;
            const uint8_t* base = (const uint8_t*)q.del_buf[q.del_cur].p;
            const int64_t* ts = (const int64_t*)base;
            const int64_t* vals = ts + 2 * n;
            const uint8_t* nb = (const uint8_t*)(vals + (size_t)nd * n);
            q.h_vptr.assign(na, nullptr);
            q.h_nptr.assign(na, nullptr);
            for (int j = 0; j < na && j < nd; ++j) {
                q.h_vptr[j] = vals + (size_t)j * n;
                q.h_nptr[j] = q.del_nulls ? nb + (size_t)j * n : q.del_zero[q.del_cur].data();
            }
            out->n = n;
            out->ts = ts;
            out->expired = q.del_zero[q.del_cur].data();
            out->n_attrs = q.hq.plan.n_user_out;
            out->types = e->out_types[qi].data();
            out->values = q.h_vptr.data();
            out->nulls = q.h_nptr.data();
            out->event_seq = ts + n;
            return (int)SDG_OK;
        }
        del_to_backlog(q);
        const int64_t n = (int64_t)q.acc_ts.size();
        q.h_ts.swap(q.acc_ts);
        q.h_seq.swap(q.acc_seq);
        q.h_vals.swap(q.acc_vals);
        q.h_nulls.swap(q.acc_nulls);
        q.acc_ts.clear();
        q.acc_seq.clear();
        for (auto& v : q.acc_vals) v.clear();
        for (auto& v : q.acc_nulls) v.clear();
        q.h_vals.resize(na);
        q.h_nulls.resize(na);
        q.h_expired.assign(n, 0);
        q.h_vptr.resize(na);
        q.h_nptr.resize(na);
        for (int j = 0; j < na; ++j) {
            q.h_vals[j].resize(n);
            q.h_nulls[j].resize(n);
            q.h_vptr[j] = q.h_vals[j].data();
            q.h_nptr[j] = q.h_nulls[j].data();
        }
        out->n = n;
        out->ts = q.h_ts.data();
        out->expired = q.h_expired.data();
        out->n_attrs = q.hq.plan.n_user_out;
        out->types = e->out_types[qi].data();
        out->values = q.h_vptr.data();
        out->nulls = q.h_nptr.data();
        out->event_seq = q.h_seq.data();
        return (int)SDG_OK;
    });
}

int sdg_discard(sdg_engine* e) {
    if (!e) return fail(SDG_ERR_ARG, "null engine");
    for (auto& q : e->qs) {
        q->polled = true;
        q->del_n = -1;
        q->acc_ts.clear();
        q->acc_seq.clear();
        q->acc_vals.clear();
        q->acc_nulls.clear();
    }
    return SDG_OK;
}

int sdg_poll_list(sdg_engine* e, int qi, int attr, int32_t* cap, int32_t* elem_type, const int64_t* const** items,
                  const uint8_t* const** item_nulls) {
    if (!e || qi < 0 || qi >= (int)e->qs.size() || !cap) return fail(SDG_ERR_ARG, "bad poll_list arguments");
    QueryRt& q = *e->qs[qi];
    const Plan& P = q.hq.plan;
    if (attr < 0 || attr >= P.n_user_out) return fail(SDG_ERR_ARG, "bad attribute index");
    *cap = P.out_multi[attr] ? P.out_list_cap[attr] : 0;
    if (elem_type) *elem_type = P.out_kind[attr];
    const size_t c0 = (size_t)P.out_list_col[attr];
    if (items) *items = *cap && q.h_vptr.size() >= c0 + *cap ? q.h_vptr.data() + c0 : nullptr;
    if (item_nulls) *item_nulls = *cap && q.h_nptr.size() >= c0 + *cap ? q.h_nptr.data() + c0 : nullptr;
    return SDG_OK;
}

namespace {
int export_records(sdg_engine* e, int qi, int64_t cap, int64_t* n_out, int64_t* d_ts, int64_t* d_seq, int64_t* d_sub,
                   int64_t* d_vals, bool ordered) {
    if (!e || qi < 0 || qi >= (int)e->qs.size() || !n_out) return fail(SDG_ERR_ARG, "bad export arguments");
    return guarded([&]() {
        QueryRt& q = *e->qs[qi];
        if (e->compile_only) throw DeviceError("engine was compiled with SDG_COMPILE_ONLY");
        if (!q.acc_ts.empty() || q.del_n >= 0)
            throw CompileError(SDG_ERR_ARG, "earlier results are still queued on the host: sdg_poll first");
        if (q.last_timers) throw CompileError(SDG_ERR_UNSUPPORTED, "device export of timer (absent-state) matches");
        if (!q.spill.empty())
            throw CompileError(SDG_ERR_UNSUPPORTED, "device export of a query with partition keys spilled to the host "
                                                    "(their records are host-side): use sdg_poll");
        if (q.hq.plan.has_post) throw CompileError(SDG_ERR_UNSUPPORTED, "device export of aggregated / having outputs");
        const int64_t n = q.polled ? 0 : q.out_n;
        *n_out = n;
        if (n > cap) throw CompileError(SDG_ERR_CAPACITY, "export buffers hold " + std::to_string(cap) + " of " +
                                                              std::to_string(n) + " records");
        hipStream_t st = e->stream;
        const int na = q.hq.plan.n_user_out;
        bool done = false;
        static const bool two_pass = getenv("SDG_EXPORT_TWO_PASS") != nullptr;  // A/B: order_records + gather
        if (n > 0 && ordered && !two_pass) {  // one sort, then ranks + gathers in one kernel (sub compared as int64)
            const size_t wb = order_workspace(n);
            void* work = q.ord_ws.ensure_slack(wb);
            std::vector<const int64_t*> src;
            std::vector<int64_t*> dst;
            auto col = [&](const void* from, int64_t* to) {
                if (!to) return;
                src.push_back((const int64_t*)from);
                dst.push_back(to);
            };
            col(q.o_ts.p, d_ts);
            col(q.o_first.p, d_sub);
            for (int j = 0; j < na && d_vals; ++j) col((const int64_t*)q.o_vals.p + (size_t)j * q.out_cap, d_vals + (size_t)j * cap);
            done = order_export((const int64_t*)q.o_emit.p, (const int64_t*)q.o_first.p, n, q.emit_base, q.emit_span,
                                src.data(), dst.data(), (int)src.size(), d_seq, work, st);
        }
        if (done) {
        } else if (n > 0 && ordered) {  // the delivery-order pass of drain(), gathering straight into the caller's buffers
            const size_t wb = order_workspace(n);
            void* work = q.ord_ws.ensure_slack(wb);
            uint32_t* perm = nullptr;
            order_records((const int64_t*)q.o_emit.p, (const int64_t*)q.o_first.p, n, q.emit_base, q.emit_span,
                          q.sub_is_seq ? q.emit_base - (1ll << 40) : 0, q.sub_bits(), work, wb, &perm, st);
            std::vector<const int64_t*> src;  // (a null destination column is not exported)
            std::vector<int64_t*> dst;
            auto col = [&](const void* from, int64_t* to) {
                if (!to) return;
                src.push_back((const int64_t*)from);
                dst.push_back(to);
            };
            col(q.o_ts.p, d_ts);
            col(q.o_emit.p, d_seq);
            col(q.o_first.p, d_sub);
            for (int j = 0; j < na && d_vals; ++j) col((const int64_t*)q.o_vals.p + (size_t)j * q.out_cap, d_vals + (size_t)j * cap);
            gather_cols_i64(src.data(), dst.data(), (int)src.size(), perm, n,
                            q.gather_ws.ensure_slack(gather_cols_workspace(n, std::min((int)src.size(), GATHER_MAX_COLS))), st);
            HIPCHECK(hipStreamSynchronize(st));
        } else if (n > 0) {
            if (d_ts) HIPCHECK(hipMemcpyAsync(d_ts, q.o_ts.p, n * 8, hipMemcpyDeviceToDevice, st));
            if (d_seq) HIPCHECK(hipMemcpyAsync(d_seq, q.o_emit.p, n * 8, hipMemcpyDeviceToDevice, st));
            if (d_sub) HIPCHECK(hipMemcpyAsync(d_sub, q.o_first.p, n * 8, hipMemcpyDeviceToDevice, st));
            for (int j = 0; j < na && d_vals; ++j)
                HIPCHECK(hipMemcpyAsync(d_vals + (size_t)j * cap, (const int64_t*)q.o_vals.p + (size_t)j * q.out_cap, n * 8,
                                        hipMemcpyDeviceToDevice, st));
            HIPCHECK(hipStreamSynchronize(st));
        }
        q.polled = true;
        return SDG_OK;
    });
}
}  // namespace

int sdg_export_device(sdg_engine* e, int qi, int64_t cap, int64_t* n_out, int64_t* d_ts, int64_t* d_seq,
                      int64_t* d_sub, int64_t* d_vals) {
    return export_records(e, qi, cap, n_out, d_ts, d_seq, d_sub, d_vals, false);
}
int sdg_export_ordered(sdg_engine* e, int qi, int64_t cap, int64_t* n_out, int64_t* d_ts, int64_t* d_seq,
                       int64_t* d_sub, int64_t* d_vals) {
    return export_records(e, qi, cap, n_out, d_ts, d_seq, d_sub, d_vals, true);
}

int sdg_last_stats(sdg_engine* e, sdg_stats* out) {
    if (!e || !out) return fail(SDG_ERR_ARG, "null argument");
    *out = e->stats;
    return SDG_OK;
}

int sdg_merge_runs(int32_t device, int32_t G, const int64_t* const* keys, const int64_t* lens, int32_t ncols,
                   const void* const* cols, const uint8_t* widths, int64_t* out_keys, void* const* out_cols) {
    if (G < 1 || !keys || !lens || !out_keys || (ncols > 0 && (!cols || !widths || !out_cols)))
        return fail(SDG_ERR_ARG, "null argument");
    if (G > MG_MAX_RUNS || ncols < 0 || ncols > MG_MAX_COLS) return fail(SDG_ERR_ARG, "too many runs or columns");
    return guarded([&]() {
        HIPCHECK(hipSetDevice(device));
        static hipStream_t st[64] = {};  // one stream per device, the merge's own (synchronous call)
        if (device < 0 || device >= 64) throw CompileError(SDG_ERR_ARG, "device ordinal out of range");
        if (!st[device]) HIPCHECK(hipStreamCreateWithFlags(&st[device], hipStreamNonBlocking));
        try {
            merge_runs_device(G, keys, lens, ncols, cols, widths, out_keys, out_cols, st[device]);
        } catch (const std::invalid_argument& x) {
            throw CompileError(SDG_ERR_ARG, x.what());
        } catch (const std::runtime_error& x) {
            throw DeviceError(x.what());
        }
        return SDG_OK;
    });
}

}  // extern "C"
