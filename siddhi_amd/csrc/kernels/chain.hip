// gfx950 chain matcher: PATTERN `every e1=S0[c0] -> e2=S1[c1] [within T]` (and `every e1=S0[c0]`), whose
// partials never interact. Over the key-sorted view, every event is a candidate e1; its e2 is
// the first later event of its key that passes c1 while the partial is alive (a forward scan).
//
//   reference: StreamPreStateProcessor.processAndReturn / isExpired / updateState
//              (core/query/input/stream/state/StreamPreStateProcessor.java:364-403, :118-129, :308-323),
//              PatternMultiProcessStreamReceiver (state/receiver/PatternMultiProcessStreamReceiver.java:27-51).
//
// chain_match_k: one block per tile of CM_TILE sorted events. The tile plus a halo of CM_HALO rows is staged in
// LDS (ts, the query-stream byte and the columns the e2 filter reads), so scans run out of LDS; a scan that
// leaves the halo continues in HBM. c1 of the common shapes (`e2.x OP const`, `e2.x OP e1.y`, none) is a typed
// loop with the e1 operand hoisted; anything else runs the bytecode. One global atomic per block reserves the
// block's match / carry ranges.
// chain_carry_k: partials carried in from the previous batch scan the new batch's key segment.
#include <hip/hip_runtime.h>

#include <limits>
#include <stdexcept>

#include "../engine/eval.h"
#include "kernels.h"
#include "wave.h"

namespace sdg {

extern __shared__ int64_t cm_lds[];

namespace {

// rows [lo, hi) of the sorted view mirrored in LDS (lo == hi: none). Offsets are in int64 words of cm_lds,
// oqs in bytes.
struct View {
    int64_t lo = 0, hi = 0;
    int32_t ots = 0, oc0 = 0, oc1 = 0, oqs = 0;
};

__device__ __forceinline__ bool in_view(const View& v, int64_t r) { return r >= v.lo && r < v.hi; }

// the fused path's slim bucket view (bucketize): ts as u32 offsets from the batch's first ts, keys as u8 local keys
__device__ __forceinline__ int64_t vts(const ChainArgs& a, int64_t r) {
    return a.ts32 ? *a.ts_base + (int64_t)a.ts32[r] : a.ts[r];
}
// row r of a bucket view belongs to key kf (the caller scans kf's bucket, so the local key decides)
__device__ __forceinline__ bool bkey_is(const ChainArgs& a, int64_t r, uint32_t kf) {
    return a.lkey ? a.lkey[r] == (uint8_t)(kf >> a.bbits) : (!a.key || a.key[r] == kf);  // (no key: one-key batch)
}
__device__ __forceinline__ int64_t orig_of(const ChainArgs& a, int64_t r) { return a.orig ? (int64_t)a.orig[r] : r; }
// column `col` of view row r: emission-only columns of the fused path stay in arrival order (ChainArgs::ocols)
__device__ __forceinline__ int64_t col_at(const ChainArgs& a, int col, uint8_t kind, int64_t r) {
    if ((a.ocol_mask >> col) & 1u) return load_col(a.ocols[col], kind, orig_of(a, r));
    return load_col(a.cols[col], kind, r);
}
__device__ __forceinline__ int64_t ts_row(const ChainArgs& a, const View& v, int64_t r) {
    return in_view(v, r) ? cm_lds[v.ots + (r - v.lo)] : vts(a, r);
}
__device__ __forceinline__ int qs_row(const ChainArgs& a, const View& v, int64_t r) {
    if (!a.qstream) return 0;
    return in_view(v, r) ? (int)((const uint8_t*)cm_lds)[v.oqs + (r - v.lo)] : (int)a.qstream[r];
}
__device__ __forceinline__ int64_t col_row(const ChainArgs& a, const View& v, int col, uint8_t kind, int64_t r) {
    const int s = a.stage_of[col];
    if (s >= 0 && in_view(v, r)) return cm_lds[(s == 0 ? v.oc0 : v.oc1) + (r - v.lo)];
    return col_at(a, col, kind, r);
}
__device__ __forceinline__ bool null_row(const ChainArgs& a, int col, int64_t r) {
    return a.nulls[col] ? a.nulls[col][r] != 0 : false;
}

// attribute access for the bytecode / FastPred evaluators (eval.h): slot 0 = e1 (a row, or a carried partial),
// slot 1 = e2 (the scanned row)
struct ChainAcc {
    const ChainArgs* A;
    View V;
    int64_t r0, c0, r1;
    __device__ void load(int slot, int col, int chain, uint8_t kind, int64_t* v, bool* null) {
        *v = 0;
        *null = true;
        if (!(chain == 0 || chain == -1)) return;  // a plain state's chain holds exactly one event
        int64_t row;
        if (slot == 0) {
            if (c0 >= 0) {
                *v = A->cin_vals[(int64_t)col * A->cin_cap + c0];
                *null = (A->cin_nulls[c0] >> col) & 1u;
                return;
            }
            row = r0;
        } else if (slot == 1) {
            row = r1;
        } else {
            return;
        }
        if (row < 0) return;
        *v = col_row(*A, V, col, kind, row);
        *null = null_row(*A, col, row);
    }
    __device__ void agg(int, int64_t* v, bool* n) { *v = 0; *n = true; }  // aggregators: the post pass only
    __device__ bool slot_empty(int slot, int chain) {
        if (!(chain == 0 || chain == -1)) return true;
        if (slot == 0) return !(c0 >= 0 || r0 >= 0);
        if (slot == 1) return r1 < 0;
        return true;
    }
};

// comparison kind -> C type (eval.h cmp(): bool compares as (v != 0), strings as dictionary ids)
template <int K> struct KT;
template <> struct KT<VK_I32> { using T = int32_t; static __device__ T get(int64_t v) { return (int32_t)v; } };
template <> struct KT<VK_I64> { using T = int64_t; static __device__ T get(int64_t v) { return v; } };
template <> struct KT<VK_F32> { using T = float; static __device__ T get(int64_t v) { return bits_f32(v); } };
template <> struct KT<VK_F64> { using T = double; static __device__ T get(int64_t v) { return bits_f64(v); } };
template <> struct KT<VK_BOOL> { using T = int; static __device__ T get(int64_t v) { return v != 0; } };
template <> struct KT<VK_STR> { using T = uint32_t; static __device__ T get(int64_t v) { return (uint32_t)v; } };

constexpr uint8_t OP_ALWAYS = 254, OP_NEVER = 255;

// a comparison operator as wave-uniform masks: x OP y == (lt && x<y) || (eq && x==y) || (gt && x>y) || (ne && x!=y)
// (NaN: <, ==, > all false, so only != holds -- Java's double/float semantics)
struct CmpMask {
    bool lt, eq, gt, ne;
};
__device__ __forceinline__ CmpMask cmp_mask(uint8_t op) {
    switch (op) {
        case CMP_EQ: return {false, true, false, false};
        case CMP_NE: return {false, false, false, true};
        case CMP_GT: return {false, false, true, false};
        case CMP_GE: return {false, true, true, false};
        case CMP_LT: return {true, false, false, false};
        case CMP_LE: return {true, true, false, false};
        case OP_ALWAYS: return {true, true, true, true};
        default: return {false, false, false, false};
    }
}
template <class T>
__device__ __forceinline__ bool cmp_m(const CmpMask& m, T x, T y) {
    return (m.lt && x < y) || (m.eq && x == y) || (m.gt && x > y) || (m.ne && !(x == y));
}

// typed scan: c1 == `e2.col OP k` (e2_left) or `k OP e2.col`, k uniform (a constant or the e1 operand)
// returns: >= 0 the matching row; -1 expired (dead); -2 reached the end of the segment (carry)
template <int K>
__device__ int64_t scan_typed(const ChainArgs& a, const View& v, int64_t from, int64_t end, int64_t ts0, int64_t k,
                              uint8_t op, uint32_t kf) {
    using C = KT<K>;
    const typename C::T y = C::get(k);
    const ChainSpec& sp = a.sp;
    const int col = sp.scan_col;
    const uint8_t kind = sp.scan_col_kind;
    const bool left = sp.scan_e2_left;
    const int32_t has_within = sp.has_within;
    const int64_t within = sp.within_ms;
    const CmpMask m = cmp_mask(op);
    const bool always = op == OP_ALWAYS;
    int64_t q = from;
    // LDS part: the scan column is staged and has no nulls
    if (a.scan_lds) {
        const int oc = a.stage_of[col] == 0 ? v.oc0 : v.oc1;
        const int64_t e = min(end, v.hi);
        const uint8_t* qs = (const uint8_t*)cm_lds + v.oqs;
        const bool multi = a.qstream != nullptr;
        for (; q < e; ++q) {
            const int i = (int)(q - v.lo);
            if (has_within) {
                int64_t d = ts0 - cm_lds[v.ots + i];
                if (d < 0) d = -d;
                if (d > within) return -1;
            }
            if (multi && qs[i] != a.s1) continue;
            if (always) return q;
            const typename C::T x = C::get(cvt(cm_lds[oc + i], kind, (uint8_t)K));
            if (left ? cmp_m(m, x, y) : cmp_m(m, y, x)) return q;
        }
    }
    const bool filt = a.bstart != nullptr;  // bucket view: other keys' rows are interleaved
    for (; q < end; ++q) {
        if (filt) {  // bucket view rows are time-ordered: past the window at any row, no later row can match
            if (has_within && ts_row(a, v, q) - ts0 > within) return -1;
            if (!bkey_is(a, q, kf)) continue;
            if (ts_row(a, v, q) < ts0) atomicOr(&a.flags[1], 1);  // the key's time went back across batches
        }
        // StreamPreStateProcessor.isExpired: |start.ts - now| > within, checked before the event is processed
        if (has_within) {
            int64_t d = ts0 - ts_row(a, v, q);
            if (d < 0) d = -d;
            if (d > within) return -1;
        }
        if (qs_row(a, v, q) != a.s1) continue;
        if (always) return q;
        if (null_row(a, col, q)) continue;  // compare with null -> false
        const typename C::T x = C::get(cvt(col_row(a, v, col, kind, q), kind, (uint8_t)K));
        if (left ? cmp_m(m, x, y) : cmp_m(m, y, x)) return q;
    }
    return -2;
}

// scan the key's events after `from` (exclusive) for the e2 of a partial whose e1 is at ts0.
// GEN = false: the query needs no bytecode (typed scan, FastPred / direct-load selects), so the interpreter is
// not compiled into the kernel (registers, code size).
template <bool GEN>
__device__ __forceinline__ int64_t chain_scan(const ChainArgs& a, ChainAcc& acc, int64_t from, int64_t end,
                                              int64_t ts0, int64_t* stk, int stride, uint32_t kf = 0) {
    const ChainSpec& sp = a.sp;
    if (!GEN || sp.scan_mode != SCAN_GENERIC) {
        int64_t k = sp.scan_konst;
        uint8_t op = sp.scan_op;
        if (sp.scan_mode == SCAN_TRUE) {
            op = OP_ALWAYS;
        } else if (sp.scan_mode == SCAN_E1) {  // e1 operand, hoisted out of the scan
            bool nl;
            acc.load(0, sp.e1_col, 0, sp.e1_col_kind, &k, &nl);
            if (nl) op = OP_NEVER;
            else k = cvt(k, sp.e1_col_kind, sp.scan_t);
        }
        switch (sp.scan_t) {
            case VK_I32: return scan_typed<VK_I32>(a, acc.V, from, end, ts0, k, op, kf);
            case VK_I64: return scan_typed<VK_I64>(a, acc.V, from, end, ts0, k, op, kf);
            case VK_F32: return scan_typed<VK_F32>(a, acc.V, from, end, ts0, k, op, kf);
            case VK_F64: return scan_typed<VK_F64>(a, acc.V, from, end, ts0, k, op, kf);
            case VK_BOOL: return scan_typed<VK_BOOL>(a, acc.V, from, end, ts0, k, op, kf);
            default: return scan_typed<VK_STR>(a, acc.V, from, end, ts0, k, op, kf);
        }
    }
    if (!GEN) return -2;  // unreachable: the host picks GEN for SCAN_GENERIC
    for (int64_t q = from; q < end; ++q) {
        if (a.bstart) {  // bucket view: time-ordered rows (see scan_typed)
            if (sp.has_within && ts_row(a, acc.V, q) - ts0 > sp.within_ms) return -1;
            if (!bkey_is(a, q, kf)) continue;
            if (ts_row(a, acc.V, q) < ts0) atomicOr(&a.flags[1], 1);
        }
        if (sp.has_within) {
            int64_t d = ts0 - ts_row(a, acc.V, q);
            if (d < 0) d = -d;
            if (d > sp.within_ms) return -1;
        }
        if (qs_row(a, acc.V, q) != a.s1) continue;
        acc.r1 = q;
        const bool ok = sp.f1.kind == FP_NONE ? pass(a.code, sp.prog1, a.consts, acc, stk, stride)
                                              : fast_pass(sp.f1, acc);
        acc.r1 = -1;
        if (ok) return q;
    }
    return -2;
}

// An Instr read as whole dwords. Reading its byte fields through a reference into the kernel-argument block
// let the compiler form a scalar-load base at the unaligned byte address of `k`; SMEM drops the low address bits,
// so `b` came back as the op/k/a/pad word (observed on gfx950, ROCm 7.2).
__device__ __forceinline__ Instr load_instr(const Instr* p) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
    const uint32_t w0 = w[0];
    Instr in;
    in.op = (uint8_t)(w0 & 0xFF);
    in.k = (uint8_t)((w0 >> 8) & 0xFF);
    in.a = (uint8_t)((w0 >> 16) & 0xFF);
    in.pad = 0;
    in.b = (int32_t)w[1];
    in.c = (int32_t)w[2];
    in.imm = (int32_t)w[3];
    return in;
}

template <bool GEN>
__device__ __forceinline__ void emit_match(const ChainArgs& a, ChainAcc& acc, int64_t slot, int64_t q, uint32_t key,
                                           int64_t first_seq, int64_t* stk, int stride) {
    const ChainSpec& sp = a.sp;
    a.out_ts[slot] = ts_row(a, acc.V, q);
    if (a.out_key) a.out_key[slot] = key;
    a.out_emit_seq[slot] = a.seq_base + (a.orig ? (int64_t)a.orig[q] : q);
    a.out_first_seq[slot] = first_seq;
    uint32_t nm = 0;
    acc.r1 = sp.n_states > 1 ? q : -1;
    for (int j = 0; j < sp.n_out; ++j) {
        int64_t v;
        bool nl;
        if (!GEN || sp.out_direct[j]) {  // a plain attribute (`e1.id`)
            const Instr in = load_instr(&sp.out_ins[j]);
            acc.load(in.a, in.b, in.c, in.k, &v, &nl);
        } else {
            run(a.code, sp.out_prog[j], a.consts, acc, stk, stride, &v, &nl);
        }
        a.out_vals[(int64_t)j * a.out_cap + slot] = v;
        if (nl) nm |= 1u << j;
    }
    if (a.write_nulls) a.out_nulls[slot] = nm;
}

__device__ __forceinline__ void emit_carry(const ChainArgs& a, const View& v, int64_t cs, int64_t p, uint32_t key,
                                           int64_t seq) {
    a.carry_key[cs] = key;
    a.carry_ts[cs] = ts_row(a, v, p);
    a.carry_seq[cs] = seq;
    uint32_t nm = 0;
    for (int c = 0; c < a.sp.n_cols; ++c) {
        a.carry_vals[(int64_t)c * a.carry_cap + cs] = col_at(a, c, a.sp.col_kind[c], p);
        if (null_row(a, c, p)) nm |= 1u << c;
    }
    a.carry_nulls[cs] = nm;
}

constexpr uint32_t CM_NONE = 0xFFFFFFFFu, CM_CARRY = 0xFFFFFFFEu;
static_assert(MQ_NONE == CM_NONE && MQ_CARRY == CM_CARRY, "emit-only mode reads mq as chain_match_k results");

// GEN = false is compiled for 8 waves per SIMD (its 102 SGPRs admitted 6); the interpreter variant keeps its registers
template <bool GEN>
__global__ __launch_bounds__(CM_THREADS, GEN ? 1 : 8) void chain_match_k(const ChainArgs* __restrict__ pa) {
    const ChainArgs& a = *pa;
    const ChainSpec& sp = a.sp;
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * CM_TILE;
    const int stride = CM_THREADS;
    View v;
    v.lo = base;
    v.hi = a.mq_in ? base : min(a.n, base + CM_ROWS);  // emit-only: nothing to stage
    v.ots = a.lds_stack ? STACK * CM_THREADS : 0;
    v.oc0 = v.ots + CM_ROWS;
    v.oc1 = v.oc0 + CM_ROWS;
    v.oqs = (v.ots + (1 + a.n_stage) * CM_ROWS) * 8;
    // u32 index of the per-event results (emit-only: right after the stack -- nothing is staged, and the launch
    // allocates only the stack and the results, chain_lds_bytes)
    const int ores = a.mq_in ? v.ots * 2 : (v.oqs + (a.qstream ? CM_ROWS : 0) + 3) / 4;
    int64_t* stk = cm_lds + tid;                                   // used only when a.lds_stack
    uint32_t* res = (uint32_t*)cm_lds + ores;
    __shared__ uint32_t wcnt[2][CM_EPT][CM_THREADS / 64];          // matches / carries per (round, wave)
    __shared__ unsigned long long bbase[2];
    const int lane = lane_id(), w = tid >> 6;
    const uint64_t lt = lanemask_lt();
    // ---- stage the tile + halo (coalesced) -------------------------------------------------------------
    const int nr = (int)(v.hi - v.lo);
    for (int i = tid; i < nr; i += CM_THREADS) cm_lds[v.ots + i] = a.ts[base + i];
    for (int c = 0; c < a.n_stage; ++c) {
        const int col = a.stage_col[c];
        const uint8_t kind = sp.col_kind[col];
        const int off = c == 0 ? v.oc0 : v.oc1;
        for (int i = tid; i < nr; i += CM_THREADS) cm_lds[off + i] = load_col(a.cols[col], kind, base + i);
    }
    if (a.qstream)
        for (int i = tid; i < nr; i += CM_THREADS) ((uint8_t*)cm_lds)[v.oqs + i] = a.qstream[base + i];
    __syncthreads();
    // ---- match: lane tid takes events base + r * CM_THREADS + tid ---------------------------------------
#pragma unroll 1
    for (int r = 0; r < CM_EPT; ++r) {
        const int64_t p = base + r * CM_THREADS + tid;
        uint32_t out = CM_NONE;
        if (p < a.n && a.mq_in) {
            out = a.mq_in[p];  // MQ_NONE == CM_NONE, MQ_CARRY == CM_CARRY
        } else if (p < a.n) {
            ChainAcc acc{&a, v, p, -1, -1};
            const uint32_t key = a.key ? a.key[p] : 0u;
            const int64_t tp = ts_row(a, v, p);
            if (p > 0 && tp < ts_row(a, v, p - 1) && (!a.key || a.key[p - 1] == key)) atomicOr(&a.flags[1], 1);
            bool c0 = false;
            if (qs_row(a, v, p) == a.s0)
                c0 = sp.f0.kind == FP_TRUE ? true
                     : (GEN && sp.f0.kind == FP_NONE) ? pass(a.code, sp.prog0, a.consts, acc, stk, stride)
                                                      : fast_pass(sp.f0, acc);
            if (c0) {
                if (sp.n_states == 1) {
                    out = (uint32_t)p;
                } else {
                    const int64_t end = a.key ? (int64_t)a.seg_end[min(key, (uint32_t)a.K - 1u)] : a.n;
                    const int64_t q = chain_scan<GEN>(a, acc, p + 1, end, tp, stk, stride);
                    out = q >= 0 ? (uint32_t)q : q == -2 ? CM_CARRY : CM_NONE;
                }
            }
        }
        res[r * CM_THREADS + tid] = out;
        const uint64_t bm = __ballot(out < CM_CARRY), bc = __ballot(out == CM_CARRY);
        if (lane == 0) {
            wcnt[0][r][w] = (uint32_t)__popcll(bm);
            wcnt[1][r][w] = (uint32_t)__popcll(bc);
        }
    }
    __syncthreads();
    // round-major exclusive scan over (round, wave): the matches of one round are consecutive slots in lane
    // order, so every store below writes one contiguous run (coalesced)
    if (tid < 2) {
        uint32_t run = 0;
        for (int r = 0; r < CM_EPT; ++r)
            for (int x = 0; x < CM_THREADS / 64; ++x) {
                const uint32_t c = wcnt[tid][r][x];
                wcnt[tid][r][x] = run;
                run += c;
            }
        bbase[tid] = run ? atomicAdd(tid == 0 ? a.out_count : a.carry_count, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    // ---- emit -------------------------------------------------------------------------------------------
#pragma unroll 1
    for (int r = 0; r < CM_EPT; ++r) {
        const uint32_t out = res[r * CM_THREADS + tid];
        const uint64_t bm = __ballot(out < CM_CARRY), bc = __ballot(out == CM_CARRY);
        if (out == CM_NONE) continue;
        const int64_t p = base + r * CM_THREADS + tid;
        const uint32_t key = a.key ? a.key[p] : 0u;
        const int64_t seq = a.seq_base + (a.orig ? (int64_t)a.orig[p] : p);
        if (out != CM_CARRY) {
            const int64_t slot = (int64_t)bbase[0] + wcnt[0][r][w] + __popcll(bm & lt);
            if (slot >= a.out_cap) {
                atomicOr(&a.flags[0], 1);
            } else {
                ChainAcc acc{&a, v, p, -1, -1};
                emit_match<GEN>(a, acc, slot, (int64_t)out, key, seq, stk, stride);
            }
        } else {
            const int64_t cs = (int64_t)bbase[1] + wcnt[1][r][w] + __popcll(bc & lt);
            if (cs >= a.carry_cap) atomicOr(&a.flags[0], 1);
            else emit_carry(a, v, cs, p, key, seq);
        }
    }
}

// ---------------------------------------------------------------------------------------------------------
// Deque path. For `every e1=S[c0] -> e2=S[e2.x OP e1.x]` with OP in {<, <=, >, >=} (one stream, one column),
// the partials pending at any time in one key, in arrival order, have monotonic x: an event with value x
// completes exactly a suffix of them (those with `x OP y`), and if it starts a partial itself its y = x is
// then the extreme value. Expiry (`within`) removes a prefix. So one pass over a key's events with a deque
// is the reference's result, with O(1) amortised work per event instead of a forward scan per partial.
// DQ_ALL: c1 does not involve e1 (`e2.x OP const`, or none): an event passing c1 completes every partial.
// Each lane owns DQ_CHUNK consecutive rows: it pushes partials from its rows only, then keeps popping over
// the following rows of the key (no pushes) until its deque drains, or carries what is left at the key's end.
// Deque entries live in an LDS ring (DQ_DEPTH per lane, [entry][lane] = conflict-free); a lane that would
// exceed it evicts its oldest entry to ovf_rows (resolved by chain_ovf_k with the forward scan).
// Every row gets exactly one mq write: its e2 row, MQ_NONE (no partial / expired / cannot match), MQ_CARRY or
// MQ_OVF (then overwritten by chain_ovf_k).
template <int K>
__global__ __launch_bounds__(DQ_THREADS) void chain_deque_k(const ChainArgs* __restrict__ pa) {
    using C = KT<K>;
    using T = typename C::T;
    const ChainArgs& a = *pa;
    const ChainSpec& sp = a.sp;
    __shared__ int64_t dq_y[DQ_DEPTH][DQ_THREADS];
    __shared__ int64_t dq_ts[DQ_DEPTH][DQ_THREADS];
    __shared__ uint32_t dq_row[DQ_DEPTH][DQ_THREADS];
    const int tid = threadIdx.x;
    const int64_t lane_rows = a.dq_lane > 0 ? a.dq_lane : DQ_CHUNK;
    const int64_t c0 = ((int64_t)blockIdx.x * DQ_THREADS + tid) * lane_rows;
    if (c0 >= a.n) return;
    const int64_t c1 = min(a.n, c0 + lane_rows);
    const int col = sp.scan_col;
    const uint8_t kind = sp.scan_col_kind;
    const uint8_t* xnull = a.nulls[col];
    const bool stack = a.deque_mode == DQ_STACK;
    const CmpMask m = cmp_mask(stack ? sp.scan_op : (sp.scan_mode == SCAN_TRUE ? OP_ALWAYS : sp.scan_op));
    const bool left = sp.scan_e2_left;
    const T kc = C::get(sp.scan_konst);
    const int32_t has_within = sp.has_within;
    const int64_t within = sp.within_ms;
    const FastPred& f0 = sp.f0;
    int head = 0, cnt = 0;
    uint32_t cur_key = a.key ? a.key[c0] : 0u;
    int64_t prev_ts = (c0 > 0 && (!a.key || a.key[c0 - 1] == cur_key)) ? a.ts[c0 - 1] : INT64_MIN;

    // one row q: expire the oldest entries, complete a suffix (or all), then (push) start a partial
    auto step = [&](int64_t q, int64_t tq, int64_t xraw, bool xn, bool push) {
        if (has_within) {
            while (cnt > 0) {
                int64_t d = dq_ts[head][tid] - tq;
                if (d < 0) d = -d;
                if (d <= within) break;
                a.mq[dq_row[head][tid]] = MQ_NONE;  // expired before completing
                head = (head + 1) & (DQ_DEPTH - 1);
                --cnt;
            }
        }
        const T x = C::get(cvt(xraw, kind, (uint8_t)K));
        if (stack) {
            if (!xn) {
                while (cnt > 0) {
                    const int top = (head + cnt - 1) & (DQ_DEPTH - 1);
                    const T y = C::get(dq_y[top][tid]);
                    if (!(left ? cmp_m(m, x, y) : cmp_m(m, y, x))) break;
                    a.mq[dq_row[top][tid]] = (uint32_t)q;
                    --cnt;
                }
            }
        } else if (cnt > 0 && (sp.scan_mode == SCAN_TRUE || (!xn && (left ? cmp_m(m, x, kc) : cmp_m(m, kc, x))))) {
            for (; cnt > 0; --cnt, head = (head + 1) & (DQ_DEPTH - 1)) a.mq[dq_row[head][tid]] = (uint32_t)q;
        }
        if (!push) return;
        // e1: the every-seed starts a partial when c0 passes (visible from the next row on)
        bool c0ok;
        if (a.f0_on_x) {
            c0ok = !xn && cmp(f0.op, f0.t, cvt(xraw, kind, f0.t), f0.konst);
        } else {
            ChainAcc acc{&a, View{}, q, -1, -1};
            c0ok = f0.kind == FP_TRUE ? true : fast_pass(f0, acc);
        }
        // an e1 whose operand is null / NaN can never complete (compare -> false): no partial
        if (!c0ok || (stack && (xn || !(x == x)))) {
            a.mq[q] = MQ_NONE;
            return;
        }
        if (cnt == DQ_DEPTH) {  // evict the oldest to the forward-scan fallback
            const uint32_t r = dq_row[head][tid];
            a.mq[r] = MQ_OVF;
            a.ovf_rows[atomicAdd(a.ovf_count, 1ull)] = r;
            head = (head + 1) & (DQ_DEPTH - 1);
            --cnt;
        }
        const int slot = (head + cnt) & (DQ_DEPTH - 1);
        dq_y[slot][tid] = (int64_t)xraw;  // raw payload, converted at compare time
        dq_ts[slot][tid] = tq;
        dq_row[slot][tid] = (uint32_t)q;
        ++cnt;
    };
    auto carry_all = [&]() {
        for (; cnt > 0; --cnt, head = (head + 1) & (DQ_DEPTH - 1)) a.mq[dq_row[head][tid]] = MQ_CARRY;
    };

    // own rows, DQ_GROUP at a time (contiguous per lane)
    for (int64_t g = c0; g < c1; g += DQ_GROUP) {
        int64_t ts[DQ_GROUP], xr[DQ_GROUP];
        uint32_t ky[DQ_GROUP];
        bool xn[DQ_GROUP];
#pragma unroll
        for (int j = 0; j < DQ_GROUP; ++j) {
            const int64_t q = min(g + j, c1 - 1);
            ts[j] = a.ts[q];
            xr[j] = load_col(a.cols[col], kind, q);
            ky[j] = a.key ? a.key[q] : 0u;
            xn[j] = xnull ? xnull[q] != 0 : false;
        }
#pragma unroll
        for (int j = 0; j < DQ_GROUP; ++j) {
            const int64_t q = g + j;
            if (q >= c1) break;
            if (ky[j] != cur_key) {  // key segment ends inside the chunk: its pending partials carry
                carry_all();
                cur_key = ky[j];
                prev_ts = INT64_MIN;
            }
            if (ts[j] < prev_ts) atomicOr(&a.flags[1], 1);
            prev_ts = ts[j];
            step(q, ts[j], xr[j], xn[j], true);
        }
    }
    // continuation: pop over the key's following rows until the deque drains, DQ_GROUP rows per round of loads.
    // With chunk summaries (one-key batches), a whole 64-row chunk none of whose rows can complete the deque's top
    // (stack: a completion pops from the top, so nothing below it goes first; all-mode: any passing row completes
    // everything) only ages the deque: the entries whose window ends inside it expire, exactly as row by row.
    // Without it the lanes whose highest partial waits ~a window of rows (C1: 1000) set the pace of the flush.
    const int64_t end = a.key ? (int64_t)a.seg_end[min(cur_key, (uint32_t)a.K - 1u)] : a.n;
    const bool summ = a.dq_any != nullptr;
    for (int64_t g = c1; g < end && cnt > 0;) {
        // a whole 64-row chunk, else a whole 8-row group (g stays a multiple of DQ_GROUP: lane_rows is one)
        const bool whole64 = (g & (DQ_CHUNK - 1)) == 0 && g + DQ_CHUNK <= end;
        if (summ && (whole64 || g + DQ_GROUP <= end)) {
            const int64_t span = whole64 ? DQ_CHUNK : DQ_GROUP;
            const int64_t ch = g / span;
            bool may = false;
            if (whole64 ? a.dq_any[ch] : a.dq_any8[ch]) {
                const T hi = C::get(whole64 ? a.dq_hi[ch] : a.dq_hi8[ch]);
                const T lo = C::get(whole64 ? a.dq_lo[ch] : a.dq_lo8[ch]);
                const T y = stack ? C::get(dq_y[(head + cnt - 1) & (DQ_DEPTH - 1)][tid]) : kc;
                may = left ? (cmp_m(m, hi, y) || cmp_m(m, lo, y)) : (cmp_m(m, y, hi) || cmp_m(m, y, lo));
            }
            if (!may) {
                if (has_within) {
                    const int64_t tl = a.ts[g + span - 1];
                    while (cnt > 0) {
                        int64_t d = dq_ts[head][tid] - tl;
                        if (d < 0) d = -d;
                        if (d <= within) break;
                        a.mq[dq_row[head][tid]] = MQ_NONE;
                        head = (head + 1) & (DQ_DEPTH - 1);
                        --cnt;
                    }
                }
                g += span;
                continue;
            }
        }
        int64_t ts[DQ_GROUP], xr[DQ_GROUP];
        bool xn[DQ_GROUP];
#pragma unroll
        for (int j = 0; j < DQ_GROUP; ++j) {
            const int64_t q = min(g + j, end - 1);
            ts[j] = a.ts[q];
            xr[j] = load_col(a.cols[col], kind, q);
            xn[j] = xnull ? xnull[q] != 0 : false;
        }
#pragma unroll
        for (int j = 0; j < DQ_GROUP; ++j) {
            if (g + j >= end || cnt == 0) break;
            step(g + j, ts[j], xr[j], xn[j], false);
        }
        g += DQ_GROUP;
    }
    carry_all();  // reached the end of the key's segment in this batch
}

// chunk summaries for chain_deque_k's continuation: one wave per DQ_CHUNK = 64 rows, the largest and smallest
// converted scan value among the rows whose comparison can hold (not null, not NaN)
static_assert(DQ_CHUNK == 64, "chain_dq_summ_k: one wave per chunk");
template <int K>
__global__ __launch_bounds__(256) void chain_dq_summ_k(const ChainArgs* __restrict__ pa) {
    using C = KT<K>;
    const ChainArgs& a = *pa;
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int col = a.sp.scan_col;
    const uint8_t kind = a.sp.scan_col_kind;
    int64_t r = 0;
    bool ok = false;
    if (q < a.n) {
        r = cvt(load_col(a.cols[col], kind, q), kind, (uint8_t)K);
        const typename C::T x = C::get(r);
        ok = !(a.nulls[col] && a.nulls[col][q]) && x == x;
    }
    int64_t hi = r, lo = r;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t h2 = __shfl_xor((long long)hi, o), l2 = __shfl_xor((long long)lo, o);
        const bool ok2 = __shfl_xor((int)ok, o) != 0;
        if (ok2) {
            if (!ok || C::get(h2) > C::get(hi)) hi = h2;
            if (!ok || C::get(l2) < C::get(lo)) lo = l2;
            ok = true;
        }
        if (o == DQ_GROUP / 2 && (lane_id() & (DQ_GROUP - 1)) == 0 && q < a.n) {  // the 8-row group's summary
            const int64_t gi = q / DQ_GROUP;
            a.dq_hi8[gi] = hi;
            a.dq_lo8[gi] = lo;
            a.dq_any8[gi] = ok;
        }
    }
    if (lane_id() == 0 && q < a.n) {
        const int64_t ch = q / DQ_CHUNK;
        a.dq_hi[ch] = hi;
        a.dq_lo[ch] = lo;
        a.dq_any[ch] = ok;
    }
}

// rows evicted from a lane's deque: the forward scan of the generic path
__global__ __launch_bounds__(256) void chain_ovf_k(const ChainArgs* __restrict__ pa) {
    const ChainArgs& a = *pa;
    __shared__ int64_t stack_mem[STACK * 256];
    int64_t* stk = stack_mem + threadIdx.x;
    const int64_t total = (int64_t)*a.ovf_count;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t p = a.ovf_rows[i];
        ChainAcc acc{&a, View{}, p, -1, -1};
        const uint32_t key = a.key ? a.key[p] : 0u;
        const int64_t end = a.key ? (int64_t)a.seg_end[min(key, (uint32_t)a.K - 1u)] : a.n;
        const int64_t q = chain_scan<true>(a, acc, p + 1, end, a.ts[p], stk, 256);
        a.mq[p] = q >= 0 ? (uint32_t)q : q == -2 ? MQ_CARRY : MQ_NONE;
    }
}

__global__ __launch_bounds__(256, 8) void chain_carry_k(const ChainArgs* __restrict__ pa) {
    const ChainArgs& a = *pa;
    __shared__ int64_t stack_mem[STACK * 256];
    int64_t* stk = stack_mem + threadIdx.x;
    const int stride = 256;
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool has = false, carry = false;
    int64_t qhit = -1;
    const View v;  // empty: everything from HBM
    ChainAcc acc{&a, v, -1, c, -1};
    uint32_t key = 0;
    if (c < a.cin_n) {
        key = a.cin_key[c];
        int64_t b = 0, e = a.n;
        if (a.bstart) {  // bucket view: the key's bucket, key-filtered
            const uint32_t bk = key & ((1u << a.bbits) - 1u);
            b = a.bstart[bk];
            e = a.bstart[bk + 1];
        } else if (a.key) {
            b = key < (uint32_t)a.K ? (int64_t)a.seg_start[key] : 0;
            e = key < (uint32_t)a.K ? (int64_t)a.seg_end[key] : 0;
        }
        // per-key time order across the batch boundary (within the batch the chain kernels check it)
        if (!a.bstart && b < e && ts_row(a, v, b) < a.cin_ts[c]) atomicOr(&a.flags[1], 1);
        const int64_t r = chain_scan<true>(a, acc, b, e, a.cin_ts[c], stk, stride, key);
        if (r >= 0) { has = true; qhit = r; }
        else if (r == -2 && !a.sub_dead) carry = true;  // (a sub-batch's bucket end: dead)
    }
    const int64_t slot = wave_reserve(has, a.out_count);
    if (has) {
        if (slot >= a.out_cap) atomicOr(&a.flags[0], 1);
        else emit_match<true>(a, acc, slot, qhit, key, a.cin_seq[c], stk, stride);
    }
    const int64_t cs = wave_reserve(carry, a.carry_count);
    if (carry) {
        if (cs >= a.carry_cap) {
            atomicOr(&a.flags[0], 1);
        } else {
            a.carry_key[cs] = key;
            a.carry_ts[cs] = a.cin_ts[c];
            a.carry_seq[cs] = a.cin_seq[c];
            for (int k = 0; k < a.sp.n_cols; ++k)
                a.carry_vals[(int64_t)k * a.carry_cap + cs] = a.cin_vals[(int64_t)k * a.cin_cap + c];
            a.carry_nulls[cs] = a.cin_nulls[c];
        }
    }
}


// Carried partials (typed scans): one WAVE per carried partial scans its key's rows 64 at a time, coalesced; the
// first lane that completes the partial or proves it dead decides (rows are in arrival order, so this is the
// lane-serial scan_typed result). One lane per partial scanning ~a window of the bucket serially was the latency
// tail of the step (chain_carry_k: 0.2 ms for ~10^4 partials).
template <int K>
__device__ int64_t wave_scan_typed(const ChainArgs& a, int64_t from, int64_t end, int64_t ts0, int64_t k, uint8_t op,
                                   uint32_t kf) {
    using C = KT<K>;
    const typename C::T y = C::get(k);
    const ChainSpec& sp = a.sp;
    const int col = sp.scan_col;
    const uint8_t kind = sp.scan_col_kind;
    const bool left = sp.scan_e2_left, always = op == OP_ALWAYS, filt = a.bstart != nullptr;
    const int32_t has_within = sp.has_within;
    const int64_t within = sp.within_ms;
    const CmpMask m = cmp_mask(op);
    const int lane = lane_id();
    constexpr int U = 4;  // rows per lane per round: U independent loads in flight (the scan is latency-bound)
    for (int64_t q0 = from; q0 < end; q0 += 64 * U) {
        uint64_t bh[U], bs[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = q0 + u * 64 + lane;
            bool stop = false, hit = false;
            if (q < end) {
                const int64_t d = vts(a, q) - ts0;
                if (filt && has_within && d > within) {
                    stop = true;  // time-ordered bucket: no later row of the key is alive
                } else if (!filt || bkey_is(a, q, kf)) {
                    if (filt && d < 0) atomicOr(&a.flags[1], 1);  // the key's time went back across batches
                    if (has_within && (d < 0 ? -d : d) > within) stop = true;  // isExpired at this event of the key
                    else if (qs_row(a, View{}, q) == a.s1) {
                        if (always) hit = true;
                        else if (!null_row(a, col, q)) {
                            const typename C::T x = C::get(cvt(load_col(a.cols[col], kind, q), kind, (uint8_t)K));
                            hit = left ? cmp_m(m, x, y) : cmp_m(m, y, x);
                        }
                    }
                }
            }
            bh[u] = __ballot(hit);
            bs[u] = __ballot(stop);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t any = bh[u] | bs[u];
            if (any) {
                const int l = __ffsll((unsigned long long)any) - 1;
                return ((bh[u] >> l) & 1u) ? q0 + u * 64 + l : -1;
            }
        }
    }
    return -2;
}

#ifndef SDG_CW_PER_WAVE
#define SDG_CW_PER_WAVE 4  // r6e: the C2 carry pass 0.10 -> 0.053 ms against 16 (same box)
#endif
constexpr int CW_PER_WAVE = SDG_CW_PER_WAVE;  // carried partials resolved one after another by one wave

// the typed e2 scan of partial (row p / carried c): the e1 operand hoisted as chain_scan does
__device__ __forceinline__ int64_t wave_scan_partial(const ChainArgs& a, ChainAcc& acc, int64_t b, int64_t e,
                                                     int64_t ts0, uint32_t key) {
    const ChainSpec& sp = a.sp;
    int64_t k = sp.scan_konst;
    uint8_t op = sp.scan_op;
    if (sp.scan_mode == SCAN_TRUE) {
        op = OP_ALWAYS;
    } else if (sp.scan_mode == SCAN_E1) {
        bool nl;
        acc.load(0, sp.e1_col, 0, sp.e1_col_kind, &k, &nl);
        if (nl) op = OP_NEVER;
        else k = cvt(k, sp.e1_col_kind, sp.scan_t);
    }
    switch (sp.scan_t) {
        case VK_I32: return wave_scan_typed<VK_I32>(a, b, e, ts0, k, op, key);
        case VK_I64: return wave_scan_typed<VK_I64>(a, b, e, ts0, k, op, key);
        case VK_F32: return wave_scan_typed<VK_F32>(a, b, e, ts0, k, op, key);
        case VK_F64: return wave_scan_typed<VK_F64>(a, b, e, ts0, k, op, key);
        case VK_BOOL: return wave_scan_typed<VK_BOOL>(a, b, e, ts0, k, op, key);
        default: return wave_scan_typed<VK_STR>(a, b, e, ts0, k, op, key);
    }
}

// rows evicted from a lane's deque (chain_deque_k), typed scans: one wave per row, CW_PER_WAVE rows per wave, the
// key's following rows scanned 256 at a time (chain_ovf_k's lane-serial scan of up to a window of rows was half
// of the C1 flush)
__global__ __launch_bounds__(256) void chain_ovf_wave_k(const ChainArgs* __restrict__ pa) {
    const ChainArgs& a = *pa;
    const int64_t total = (int64_t)*a.ovf_count;
    const int64_t stride = (int64_t)gridDim.x * 4 * CW_PER_WAVE;
    for (int64_t i = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * CW_PER_WAVE; i < total;
         i += (i % CW_PER_WAVE == CW_PER_WAVE - 1) ? stride - (CW_PER_WAVE - 1) : 1) {  // wave-uniform
        const int64_t p = a.ovf_rows[i];
        ChainAcc acc{&a, View{}, p, -1, -1};
        const uint32_t key = a.key ? a.key[p] : 0u;
        const int64_t end = a.key ? (int64_t)a.seg_end[min(key, (uint32_t)a.K - 1u)] : a.n;
        const int64_t q = wave_scan_partial(a, acc, p + 1, end, a.ts[p], key);
        if (lane_id() == 0) a.mq[p] = q >= 0 ? (uint32_t)q : q == -2 ? MQ_CARRY : MQ_NONE;
    }
}

// Block = 4 waves x CW_PER_WAVE partials; lane i of a wave keeps the result of its i-th partial, and the block
// reserves its match / carry output with one atomic per counter (one atomic per partial serialised in L2:
// ~10^8/s, 0.2 ms for 2 x 10^4 carries).
__global__ __launch_bounds__(256, 8) void chain_carry_wave_k(const ChainArgs* __restrict__ pa) {
    const ChainArgs& a = *pa;
    const ChainSpec& sp = a.sp;
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int64_t c_base = ((int64_t)blockIdx.x * 4 + w) * CW_PER_WAVE;
    int64_t mine = -1;  // lane i: the scan result of partial c_base + i
    for (int i = 0; i < CW_PER_WAVE; ++i) {
        const int64_t c = c_base + i;
        if (c >= a.cin_n) break;  // wave-uniform
        const uint32_t key = a.cin_key[c];
        int64_t b = 0, e = a.n;
        if (a.bstart) {
            const uint32_t bk = key & ((1u << a.bbits) - 1u);
            b = a.bstart[bk];
            e = a.bstart[bk + 1];
        } else if (a.key) {
            b = key < (uint32_t)a.K ? (int64_t)a.seg_start[key] : 0;
            e = key < (uint32_t)a.K ? (int64_t)a.seg_end[key] : 0;
        }
        if (!a.bstart && b < e && vts(a, b) < a.cin_ts[c] && lane == 0) atomicOr(&a.flags[1], 1);  // time went back
        ChainAcc acc{&a, View{}, -1, c, -1};
        int64_t k = sp.scan_konst;
        uint8_t op = sp.scan_op;
        if (sp.scan_mode == SCAN_TRUE) {
            op = OP_ALWAYS;
        } else if (sp.scan_mode == SCAN_E1) {
            bool nl;
            acc.load(0, sp.e1_col, 0, sp.e1_col_kind, &k, &nl);
            if (nl) op = OP_NEVER;
            else k = cvt(k, sp.e1_col_kind, sp.scan_t);
        }
        const int64_t ts0 = a.cin_ts[c];
        int64_t r;
        switch (sp.scan_t) {
            case VK_I32: r = wave_scan_typed<VK_I32>(a, b, e, ts0, k, op, key); break;
            case VK_I64: r = wave_scan_typed<VK_I64>(a, b, e, ts0, k, op, key); break;
            case VK_F32: r = wave_scan_typed<VK_F32>(a, b, e, ts0, k, op, key); break;
            case VK_F64: r = wave_scan_typed<VK_F64>(a, b, e, ts0, k, op, key); break;
            case VK_BOOL: r = wave_scan_typed<VK_BOOL>(a, b, e, ts0, k, op, key); break;
            default: r = wave_scan_typed<VK_STR>(a, b, e, ts0, k, op, key); break;
        }
        if (lane == i) mine = r;
    }
    const int64_t c = c_base + lane;
    const bool valid = lane < CW_PER_WAVE && c < a.cin_n;
    const bool has = valid && mine >= 0, carry = valid && mine == -2 && !a.sub_dead;
    int64_t slot, cs;
    block_reserve2<256>(has, carry, a.out_count, a.carry_count, &slot, &cs);
    if (has) {
        if (slot >= a.out_cap) {
            atomicOr(&a.flags[0], 1);
        } else {
            ChainAcc acc{&a, View{}, -1, c, -1};
            emit_match<false>(a, acc, slot, mine, a.cin_key[c], a.cin_seq[c], nullptr, 0);
        }
    }
    if (carry) {
        if (cs >= a.carry_cap) {
            atomicOr(&a.flags[0], 1);
        } else {
            a.carry_key[cs] = a.cin_key[c];
            a.carry_ts[cs] = a.cin_ts[c];
            a.carry_seq[cs] = a.cin_seq[c];
            for (int j = 0; j < sp.n_cols; ++j)
                a.carry_vals[(int64_t)j * a.carry_cap + cs] = a.cin_vals[(int64_t)j * a.cin_cap + c];
            a.carry_nulls[cs] = a.cin_nulls[c];
        }
    }
}

// ---------------------------------------------------------------------------------------------------------
// Fused bucket matcher (kernels.h). Block = (bucket b, segment s): rows [lo, lo + own) of the bucket are its
// candidates, rows [lo, lo + nr) (own + halo) are staged. Staging regroups the rows by local key (key >> bbits)
// with a stable counting sort in LDS (wave-private ballot-match ranking, as rx_scatter), so the rows of one key
// form one run in s_ts / s_x in arrival order -- the key-sorted view of chain_match_k, built per block in LDS
// instead of by a second radix pass over HBM.
// soft bounds checks (debugging aid): a failed check sets bit `id` of flags[2] and the access is skipped
#define FU_OK(cond, id) ((cond) ? true : (atomicOr(&a.flags[2], 1 << (id)), false))
// SDG_DEBUG progress trace: the last stage each wave reached, readable by the host after a fault
#define FU_TRACE(stage)                                                                                     \
    do {                                                                                                    \
        if (a.dbg && lane == 0) a.dbg[(int64_t)blockIdx.x * 4 + w] = (stage);                              \
    } while (0)

static_assert(FU_THREADS >= 256, "chain_fused_k: one thread per local key in the run tables");
static_assert(FU_DQ <= 32, "chain_fused_k: a lane's deque is a 32-bit mask over its positions");
static_assert(FU_DQ >= FU_PT && FU_ROWS % FU_DQ == 0, "chain_fused_k: deque chunks tile the staged rows");
constexpr uint16_t R_NONE = 0xFFFF, R_CARRY = 0xFFFE, R_OVF = 0xFFFD;
// LDS swizzle of the per-position arrays: the deque pass gives lane t the positions [FU_DQ t, FU_DQ (t + 1)), so
// unswizzled, one step of a wave hits every lane's element at an FU_DQ-position stride (few banks). XOR-ing the
// low log2(FU_DQ) bits with the next ones spreads those over the banks; runs of consecutive positions stay
// permuted within their aligned group of FU_DQ (still conflict-free for the per-round `k * FU_THREADS + t` accesses).
static_assert((FU_DQ & (FU_DQ - 1)) == 0, "sw() swizzles at the deque chunk size");
__device__ __forceinline__ int sw(int p) { return p ^ ((p / FU_DQ) & (FU_DQ - 1)); }
static_assert(FU_ROWS < 65536, "chain_fused_k: u16 rows / run offsets");
#ifndef SDG_WQ_U
#define SDG_WQ_U 2  // rows each lane of the work queue tests per iteration
#endif
#ifndef SDG_WQ_BF
#define SDG_WQ_BF 0  // the SOP build's work queue with a branch-free scan step (A/B)
#endif
#ifndef SDG_FIX_STAGE
#define SDG_FIX_STAGE 1  // the SOP build's staging loads without the view / kind dispatch (0: A/B)
#endif

// SAME: the scanned column's kind is the comparison kind (no conversion in the scan loop). W: minimum waves per SIMD
// the allocator must allow -- 8 = four 512-thread blocks per CU (LDS 4 x 40 KB fits); at 6 it used 104 SGPRs, which
// admits 6 waves per SIMD = 3 blocks (MI355X_MICROARCH residency rule). 8 costs SGPR / VGPR spills.
// ONEK: one-key batches (unpartitioned, C1): a.fu_own rows per segment, the staging's time-order check and the work
// queue's group summaries. Compile-time, so the many-key build keeps its registers (C2's matcher 2.04 -> 2.26 ms with
// them present but switched off at run time, r5t/r5u)
#ifndef SDG_FU_W8
#define SDG_FU_W8 8  // the SOP build's minimum waves per SIMD (A/B builds with more staged rows: 4)
#endif
#ifndef SDG_FU_ROWORDER
#define SDG_FU_ROWORDER 1  // chain_fused_k emits a block's records in e1-row order (0: regrouped order, A/B)
#endif
// OC: some output columns stay in arrival order (ChainArgs::ocols): time-major block order, and the emission reads
// them through orig (a separate instantiation: the selects cost the others 0.17 ms on C2, r5w)
// SOP (round 6): -1 the scan's operator is read at run time; else a compile-time ordering operator (CMP_GT / GE / LT
// / LE) for the common shape `e2.x OP e1.x` on the scan column (SCAN_E1, the e1 operand is the scanned value): x beats
// the partial's y iff x SOP y, with the host folding e2's side into SOP. Only the work-queue match pass is compiled
// then (the deque / fixed-scan A/B paths and the run-time operator dispatch drop out: fewer SGPRs, no uniform
// branches in the scan loop)
template <int K, bool SAME, int W, bool ONEK = false, bool OC = false, int SOP = -1>
__global__ __launch_bounds__(FU_THREADS, W) void chain_fused_k(const ChainArgs* __restrict__ pa) {
    using C = KT<K>;
    using T = typename C::T;
    constexpr bool FIX = SOP >= 0;
    static_assert(!FIX || SOP == CMP_GT || SOP == CMP_GE || SOP == CMP_LT || SOP == CMP_LE, "SOP: an ordering operator");
    static_assert(!FIX || (SAME && !ONEK && !OC), "SOP: the many-key build of the scan's own kind");
    constexpr int NW = FU_THREADS / 64;
    constexpr int WROWS = FU_ROWS / NW;  // staged rows ranked by one wave (contiguous)
    const ChainArgs& a = *pa;
    const ChainSpec& sp = a.sp;
    __shared__ uint32_t s_ts[FU_ROWS];   // ts - ts of the block's first staged row (bucket rows are time-ordered)
    __shared__ int64_t s_x[FU_ROWS];
    __shared__ uint16_t s_row[FU_ROWS];
    __shared__ uint8_t s_lk[FU_ROWS];
    __shared__ uint16_t s_res[FU_ROWS];  // per position: e2 position | R_NONE | R_CARRY | R_OVF
    // regrouping counters; then the deque chunks' summaries, or the work queue's candidate list (up to WROWS a wave)
    __shared__ __align__(16) uint16_t wc[NW][WROWS > 256 ? WROWS : 256];
    __shared__ __align__(8) uint16_t lstart[256];  // (reused by the work queue: 64 group extremes of 8 bytes)
    __shared__ uint16_t lend[256];
    __shared__ uint32_t wcnt[3][FU_PT][NW];
    __shared__ unsigned long long bbase[3];
    __shared__ int sb[2];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    // XCD-aware block order (kernels.h xcd_block): virtual id v gives each XCD a contiguous run of segments, so
    // neighbouring segments (which share halo rows) hit one L2
    const uint32_t v = xcd_block(blockIdx.x, gridDim.x, (uint32_t)a.xcds);
    if (t == 0) sb[0] = -1;
    __syncthreads();
    const uint32_t tS = (OC && a.tm) ? a.tm[0] : 0u;
    const uint32_t tmin = OC && tS ? a.tm[1] : 0u;
    if (OC && tS && v < tmin * (uint32_t)a.nb) {  // time-major, the levels every bucket has: closed form
        if (t == 0) {
            sb[0] = (int)(v % (uint32_t)a.nb);
            sb[1] = (int)(v / (uint32_t)a.nb);
        }
    } else if (OC && tS) {  // time-major (bucketize's plan): segment s of every bucket before segment s + 1 of any, so
                            // the blocks in flight cover one time band (the arrival-order columns stay in cache)
        __shared__ uint32_t s_sr[2], s_wc[FU_THREADS / 64];
        if (t == 0) {
            uint32_t lo_s = tmin, hi_s = tS;  // largest s in [tmin, S] with tm[2 + s] <= v
            while (lo_s < hi_s) {
                const uint32_t mid = (lo_s + hi_s + 1) >> 1;
                if (a.tm[2 + mid] <= v) lo_s = mid;
                else hi_s = mid - 1;
            }
            s_sr[0] = lo_s;
            s_sr[1] = v - a.tm[2 + lo_s];
        }
        __syncthreads();
        const uint32_t ss = s_sr[0], rr = s_sr[1];
        const bool has = ss < tS && t < a.nb && a.bseg[t + 1] - a.bseg[t] > ss;
        const uint64_t bal = __ballot(has);
        if (lane == 0) s_wc[w] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = (uint32_t)__popcll(bal & lanemask_lt());
        for (int x = 0; x < w; ++x) before += s_wc[x];
        if (has && before == rr) {
            sb[0] = t;
            sb[1] = (int)ss;
        }
    } else if (t < a.nb && a.bseg[t] <= v && v < a.bseg[t + 1]) {
        sb[0] = t;
        sb[1] = (int)(v - a.bseg[t]);
    }
    __syncthreads();
    const int b = sb[0];
    FU_TRACE(1);
    if (b < 0) { FU_TRACE(99); return; }  // block-uniform: past the plan
    const int64_t be = a.bstart[b + 1];
    const int fown = ONEK ? a.fu_own : FU_OWN;
    const int64_t lo = (int64_t)a.bstart[b] + (int64_t)sb[1] * fown;
    const int64_t oe = a.bown ? (int64_t)a.bown[b] : be;  // the bucket's own rows end (sub-batches: its halo after)
    const int own = (int)min((int64_t)fown, oe - lo);
    const int nr = (int)min((int64_t)FU_ROWS, be - lo);
    const bool to_end = lo + nr == be;  // the staged rows reach the bucket's (= batch's) end for every key
    const int col = sp.scan_col;
    const uint8_t kind = sp.scan_col_kind;
    const int nl = 1 << a.lbits;
    // ---- stage: coalesced loads (all rounds in flight), stable rank by local key -----------------------------
    for (int d = t; d < 256; d += FU_THREADS)
#pragma unroll
        for (int x = 0; x < NW; ++x) wc[x][d] = 0;
    if (!FU_OK(lo >= 0 && nr >= 1 && lo + nr <= a.n && b < a.nb, 1)) return;
    const int64_t tbase = vts(a, lo);
    const int64_t tlast = vts(a, lo + nr - 1);
    uint32_t rkey[FU_PT];
    int64_t rts[FU_PT], rx[FU_PT];
    const void* xcol = a.cols[col];
#pragma unroll
    for (int r = 0; r < FU_PT; ++r) {
        const int row = w * WROWS + r * 64 + lane;
        const int64_t g = lo + min(row, nr - 1);  // clamped: rows past nr are loaded but not staged
        if ((FIX && SDG_FIX_STAGE) || a.lkey) {  // slim view: u8 local key, u32 ts offset (the SOP build: always)
            rkey[r] = (uint32_t)a.lkey[g] << a.bbits;
            rts[r] = tbase + (int64_t)(uint32_t)(a.ts32[g] - a.ts32[lo]);
        } else {
            rkey[r] = ONEK ? 0u : a.key[g];
            rts[r] = a.ts[g];
        }
        if constexpr (FIX && SDG_FIX_STAGE)  // the scan column's own kind (SAME): its width, no kind dispatch
            rx[r] = sizeof(T) == 8 ? ((const int64_t*)xcol)[g] : (int64_t)((const int32_t*)xcol)[g];
        else
            rx[r] = kind == VK_F64 || kind == VK_I64 ? ((const int64_t*)xcol)[g] : load_col(xcol, kind, g);
    }
    if (ONEK) {  // one-key batch: arrival order must be time order (the chain path's precondition)
        bool bad = false;
#pragma unroll
        for (int r = 0; r < FU_PT; ++r) {
            const int row = w * WROWS + r * 64 + lane;
            int64_t prev = __shfl_up(rts[r], 1);
            if (lane == 0) prev = lo + row > 0 ? a.ts[lo + row - 1] : INT64_MIN;
            bad |= row < nr && rts[r] < prev;
        }
        if (__ballot(bad) && lane == 0) atomicOr(&a.flags[3], 1);
    }
    FU_TRACE(2);
    if (!(FIX && SDG_FIX_STAGE) && tlast - tbase > (int64_t)0xFFFFFFFF) {  // staged span does not fit the u32 offsets (slim view:
        if (t == 0) atomicOr(&a.flags[3], 1);     // it does) -> the host reruns the batch on the radix path
        return;                                   // block-uniform
    }
    if (a.fu_skip & 4) {
        if (rts[0] == -12345 && rx[FU_PT - 1] == 7 && rkey[FU_PT / 2] == 9) a.flags[2] = 1;  // keep the loads alive
        return;
    }
    __syncthreads();
    FU_TRACE(3);
    const uint64_t lt = lanemask_lt();
    uint32_t rank[FU_PT];
    uint8_t dig[FU_PT];
#pragma unroll
    for (int r = 0; r < FU_PT; ++r) {
        const int row = w * WROWS + r * 64 + lane;
        const bool valid = row < nr;
        const uint32_t d = valid ? (rkey[r] >> a.bbits) & (uint32_t)(nl - 1) : 0u;  // mask: no-op for keys < K
        uint64_t peers = __ballot(valid);
        for (int bit = 0; bit < a.lbits; ++bit) {
            const bool on = (d >> bit) & 1u;
            const uint64_t m = __ballot(on);
            peers &= on ? m : ~m;
        }
        const uint32_t before = valid ? wc[w][d] : 0u;
        rank[r] = before + (uint32_t)__popcll(peers & lt);
        dig[r] = (uint8_t)d;
        const int leader = peers ? __ffsll((unsigned long long)peers) - 1 : -1;
        if (valid && lane == leader) wc[w][d] = (uint16_t)(before + (uint32_t)__popcll(peers));
    }
    __syncthreads();
    uint32_t tot = 0;
    if (t < nl) {
#pragma unroll
        for (int x = 0; x < NW; ++x) {
            const uint32_t c = wc[x][t];
            wc[x][t] = (uint16_t)tot;
            tot += c;
        }
    }
    {  // inclusive scan of the run lengths (<= FU_ROWS: fits u16)
        const uint32_t inc = scan256_incl(t < 256 ? tot : 0u, &wcnt[0][0][0]);  // (wcnt is free until the counts)
        if (t < 256) {
            lend[t] = (uint16_t)inc;
            lstart[t] = (uint16_t)(inc - tot);
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < FU_PT; ++r) {
        const int row = w * WROWS + r * 64 + lane;
        if (row < nr) {
            const uint32_t pos = lstart[dig[r]] + wc[w][dig[r]] + rank[r];
            if (!FU_OK(pos < (uint32_t)nr, 2)) continue;
            s_ts[sw(pos)] = (uint32_t)(rts[r] - tbase);
            s_x[sw(pos)] = rx[r];
            s_row[sw(pos)] = (uint16_t)row;
            s_lk[sw(pos)] = dig[r];
            s_res[sw(pos)] = R_NONE;
        }
    }
    __syncthreads();
    FU_TRACE(4);
    if (a.fu_skip & 8) return;
    // ---- match: position pos = k * FU_THREADS + t (a run of consecutive positions per round) ---------------
    const bool stream_e1 = FIX || sp.scan_mode == SCAN_E1;
    const bool e1_is_x = FIX || (stream_e1 && sp.e1_col == col && sp.e1_col_kind == kind);
    const CmpMask m = cmp_mask(sp.scan_mode == SCAN_TRUE ? OP_ALWAYS : sp.scan_op);
    const bool left = sp.scan_e2_left;
    // x (a later row's value) completes the partial whose e1 operand is y
    auto beats = [&](T x, T y) -> bool {
        if constexpr (SOP == CMP_GT) return x > y;
        else if constexpr (SOP == CMP_GE) return x >= y;
        else if constexpr (SOP == CMP_LT) return x < y;
        else if constexpr (SOP == CMP_LE) return x <= y;
        else return left ? cmp_m(m, x, y) : cmp_m(m, y, x);
    };
    // bucket rows are time-ordered (bucketize checked it), so a later row's offset is never below the start's
    const uint64_t within_u = sp.has_within ? (uint64_t)sp.within_ms : ~0ull;
    const FastPred& f0 = sp.f0;
    const bool f0_on_x = a.f0_on_x;
    const bool f0_typed = f0_on_x && SAME && f0.t == K;  // c0 = `x OP const` in the scan's own type
    const CmpMask m0 = cmp_mask(f0.op);
    const T k0 = C::get(f0.konst);
    const T kc = C::get(sp.scan_konst);
    // a partial still pending when its key's staged rows end: carried at the flush's end, dead at a sub-batch's (its
    // halo reaches past the window), else its key continues past the staged rows (the HBM scan)
    const uint16_t ran_off = to_end ? (a.sub_dead ? R_NONE : R_CARRY) : R_OVF;
    // ... unless the staged span already reaches past its window: every later row of the bucket (so every later
    // event of its key) has ts >= tlast, where the partial is expired (isExpired) -- dead, no HBM scan needed
    const uint32_t tl_off = (uint32_t)(tlast - tbase);
    auto ran_res = [&](int pos) -> uint16_t {
        return (!to_end && (uint64_t)(tl_off - s_ts[sw(pos)]) > within_u) ? R_NONE : ran_off;
    };
    auto c0_at = [&](int pos, int64_t xr, T xv) -> bool {  // the e1 filter of the row at `pos`
        if (f0_typed) return cmp_m(m0, xv, k0);
        if (f0_on_x) return cmp(f0.op, f0.t, cvt(xr, kind, f0.t), f0.konst);
        ChainAcc acc{&a, View{}, lo + s_row[sw(pos)], -1, -1};
        return f0.kind == FP_TRUE ? true : fast_pass(f0, acc);
    };
    if (a.fu_skip & 16) {
        // phase timing: no matching
    } else if (!(a.fu_skip & 256)) {
        // ---- wave work queue (round 5): each candidate's result is independent of every other partial's (DESIGN.md
        // 4: a partial completes at the first later row of its key that passes c1 while it is alive), so it is a
        // forward scan over its key's run in LDS. Scan lengths are uneven (a high e1 price waits for expiry, ~a window
        // of its key's rows; most resolve within a few rows), so instead of a fixed candidate per lane (the wave
        // waiting for its slowest lane every round) or a deque per lane (rows revisited by several lanes), a lane
        // that resolves its candidate takes the wave's next one from a list: every lane stays busy and each
        // iteration advances 64 scans by WQ_U rows.
        constexpr int WQ_U = SDG_WQ_U;
        uint16_t* const cand = &wc[w][0];  // the wave's candidate positions in position order (wc is free now)
        int ncand = 0;
#pragma unroll
        for (int r = 0; r < FU_PT; ++r) {
            const int pos = w * WROWS + r * 64 + lane;
            bool c = false;
            if (pos < nr && s_row[sw(pos)] < own) {
                const int64_t xr = s_x[sw(pos)];
                c = c0_at(pos, xr, SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K)));
            }
            const uint64_t bm = __ballot(c);
            if (c) cand[ncand + __popcll(bm & lt)] = (uint16_t)pos;
            ncand += __popcll(bm);
        }
        // group summaries (stack mode, ordering compares): per 32 consecutive positions the extreme value that could
        // complete a partial (the max when "x beats y" grows with x, else the min; NaN rows never complete one).
        // A scan skips a whole group whose extreme cannot beat its partial's e1 value: no row in it completes the
        // partial, and an expiry inside it shows at the next row scanned (a key's rows are time-ordered). The groups
        // may mix keys (an upper bound is still an upper bound); they pay for one-key batches (C1), where a high
        // e1 price scans up to a whole window of rows
        constexpr int WQ_G = FU_ROWS <= 2048 ? 32 : FU_ROWS / 64;
        static_assert(FU_ROWS / WQ_G * 8 <= sizeof(lstart), "group summaries fit lstart");
        const bool wq_mono = ONEK && a.fu_mode == DQ_STACK && (m.gt != m.lt) && !m.ne && !(a.fu_skip & 128);
        const bool use_max = left == m.gt;
        T* const s_gx = reinterpret_cast<T*>(&lstart[0]);
        if (ONEK && wq_mono) {  // (block-uniform; lstart is free after the regrouping)
            T ext = use_max ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max();
#pragma unroll
            for (int i = 0; i < FU_ROWS / FU_THREADS; ++i) {
                const int pos = t * (FU_ROWS / FU_THREADS) + i;
                const T x = SAME ? C::get(s_x[sw(pos)]) : C::get(cvt(s_x[sw(pos)], kind, (uint8_t)K));
                if (pos < nr && x == x) ext = use_max ? (x > ext ? x : ext) : (x < ext ? x : ext);
            }
            constexpr int LPG = WQ_G / (FU_ROWS / FU_THREADS);  // lanes per group
#pragma unroll
            for (int o = 1; o < LPG; o <<= 1) {
                const T e2 = __shfl_xor(ext, o);
                ext = use_max ? (e2 > ext ? e2 : ext) : (e2 < ext ? e2 : ext);
            }
            if ((t & (LPG - 1)) == 0) s_gx[t / LPG] = ext;
        }
        if (ONEK) {
            __syncthreads();
        } else {  // the candidate list (written by other lanes of this wave) before the queue reads it
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
        int p = -1, q = 0, end = 0, head = 0;
        uint32_t t0 = 0;
        T y = kc;
        bool live = true;  // the e1 operand is not null (a null operand compares false on every row)
#if SDG_WQ_BF
        if constexpr (FIX) {
            // branch-free scan step (SOP build): every lane loads its WQ_U rows (clamped) and resolves them with
            // selects -- no divergent branches in the loop body; the window test on u32 offsets
            const uint32_t win32 = within_u > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)within_u;
            uint16_t rend = R_NONE;  // the candidate's result when its key's staged rows end with it pending
#pragma unroll 1
            for (;;) {
                const uint64_t need = __ballot(p < 0);
                if (need) {  // wave-uniform
                    const int idx = head + __popcll(need & lt);
                    head += __popcll(need);
                    if (p < 0 && idx < ncand) {
                        p = cand[idx];
                        const int sp0 = sw(p);
                        t0 = s_ts[sp0];
                        y = C::get(s_x[sp0]);
                        end = (int)lend[s_lk[sp0]];
                        if (!FU_OK(end <= nr && end > p, 4)) end = p + 1;
                        q = p + 1;
                        rend = (!to_end && tl_off - t0 > win32) ? R_NONE : ran_off;
                    }
                    if (__ballot(p >= 0) == 0) break;
                }
                int r = -1;  // the first of the WQ_U rows that decides the partial (from the last row back)
#pragma unroll
                for (int u = WQ_U - 1; u >= 0; --u) {
                    const int sq = sw(min(q + u, FU_ROWS - 1));
                    const uint32_t tq = s_ts[sq];
                    const T x = C::get(s_x[sq]);
                    const int d = q + u >= end ? (int)rend : tq - t0 > win32 ? (int)R_NONE : beats(x, y) ? q + u : -1;
                    r = d >= 0 ? d : r;
                }
                if (p >= 0 && r >= 0) {
                    s_res[sw(p)] = (uint16_t)r;
                    p = -1;
                } else {
                    q += WQ_U;
                }
            }
        } else
#endif
#pragma unroll 1
        for (;;) {
            const uint64_t need = __ballot(p < 0);
            if (need) {  // wave-uniform
                const int idx = head + __popcll(need & lt);
                head += __popcll(need);
                if (p < 0 && idx < ncand) {
                    p = cand[idx];
                    t0 = s_ts[sw(p)];
                    const int64_t xr = s_x[sw(p)];
                    end = (int)lend[s_lk[sw(p)]];
                    if (!FU_OK(end <= nr && end > p, 4)) end = p + 1;
                    q = p + 1;
                    live = true;
                    if (stream_e1) {
                        if (e1_is_x) {
                            y = SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K));
                        } else {
                            const int64_t g = lo + s_row[sw(p)];
                            live = !(a.nulls[sp.e1_col] && a.nulls[sp.e1_col][g]);
                            y = C::get(cvt(load_col(a.cols[sp.e1_col], sp.e1_col_kind, g), sp.e1_col_kind, (uint8_t)K));
                        }
                    }
                }
                if (__ballot(p >= 0) == 0) break;
            }
            if (ONEK && p >= 0 && wq_mono) {  // the rest of q's group, when its extreme cannot beat the partial
                const int ge = (q & ~(WQ_G - 1)) + WQ_G;
                if (ge <= end) {
                    const T g = s_gx[q / WQ_G];
                    if (!(left ? cmp_m(m, g, y) : cmp_m(m, y, g))) {
                        q = ge;
                        continue;
                    }
                }
            }
            if (p >= 0) {
                uint32_t tq[WQ_U];
                T xq[WQ_U];
#pragma unroll
                for (int u = 0; u < WQ_U; ++u) {
                    const int qq = min(q + u, FU_ROWS - 1);
                    tq[u] = s_ts[sw(qq)];
                    const int64_t xr = s_x[sw(qq)];
                    xq[u] = SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K));
                }
                int r = -1;  // -1 pending, else the s_res value
#pragma unroll
                for (int u = 0; u < WQ_U; ++u) {
                    if (r >= 0) break;
                    if (q + u >= end) {  // the key's staged rows ended with the partial pending
                        // ONEK: a group skip may have jumped straight to `end` over the row that expired the partial
                        // (its key's last staged row is the block's last, tl_off), so test the window even when the
                        // rows reach the batch end -- an expired partial must not be carried
                        r = ((ONEK || !to_end) && (uint64_t)(tl_off - t0) > within_u) ? R_NONE : ran_off;
                    } else if ((uint64_t)(tq[u] - t0) > within_u) {  // isExpired before the row is processed
                        r = R_NONE;
                    } else if ((FIX || live) && beats(xq[u], y)) {
                        r = q + u;
                    }
                }
                if (r >= 0) {
                    s_res[sw(p)] = (uint16_t)r;
                    p = -1;
                } else {
                    q += WQ_U;
                }
            }
        }
    } else if constexpr (FIX) {
        // (the host launches the SOP build for the work queue only)
    } else if (a.fu_mode != DQ_OFF) {
        // ---- monotone-deque pass (chain_deque_k), one lane per FU_DQ consecutive positions: the lane
        // pushes partials from its own positions only and keeps popping over the following positions of the key
        // until its deque drains. The deque is a bit mask over the lane's positions (bit i = position p0 + i
        // pending); arrival order = position order, so the front is the lowest bit and the top the highest.
        // The chunk's rows are prefetched into registers (static indices: the loop over them is unrolled); the
        // front's ts and the top's value are cached and re-read from LDS only when the front / top changes.
        const bool stack = a.fu_mode == DQ_STACK;
        const int p0 = t * FU_DQ;  // lanes with p0 >= nr (whole waves past FU_ROWS / FU_DQ) have no chunk
        uint32_t pend = 0, tf = 0;
        T ytop = T(0);
        // one row (ts tq, value x) against the pending partials: expire the prefix, then complete (a suffix / all).
        // The front's ts (tf) and the top's value (ytop) are cached; pops only ever remove from the top, so tf
        // changes only by expiry or by emptying.
        auto step = [&](int q, uint32_t tq, T x) {
            // StreamPreStateProcessor.expireEvents: the expired prefix (oldest first); s_res stays R_NONE
            while (pend && (uint64_t)(tq - tf) > within_u) {
                pend &= pend - 1;
                if (pend) tf = s_ts[sw(p0 + __builtin_ctz(pend))];
            }
            if (stack) {  // x completes the suffix of partials whose e1 value it beats
                while (pend && (left ? cmp_m(m, x, ytop) : cmp_m(m, ytop, x))) {
                    const int tp = 31 - __builtin_clz(pend);
                    s_res[sw(p0 + tp)] = (uint16_t)q;
                    pend &= ~(1u << tp);
                    if (pend) {
                        const int64_t yr = s_x[sw(p0 + 31 - __builtin_clz(pend))];
                        ytop = SAME ? C::get(yr) : C::get(cvt(yr, kind, (uint8_t)K));
                    }
                }
            } else if (pend && (left ? cmp_m(m, x, kc) : cmp_m(m, kc, x))) {  // complete-all
                for (; pend; pend &= pend - 1) s_res[sw(p0 + __builtin_ctz(pend))] = (uint16_t)q;
            }
        };
        const int pe = min(p0 + FU_DQ, nr);
        int cur_end = p0 < nr ? (int)lend[s_lk[sw(p0)]] : 0;
        // the chunk's own rows, read from LDS up front (all reads in flight together)
        uint32_t cts[FU_DQ];
        int64_t cx[FU_DQ];
        uint16_t crow[FU_DQ];
#pragma unroll
        for (int i = 0; i < FU_DQ; ++i) {
            const int q = min(p0 + i, FU_ROWS - 1);
            cts[i] = s_ts[sw(q)];
            cx[i] = s_x[sw(q)];
            crow[i] = s_row[sw(q)];
        }
        // chunk summaries (stack mode, ordering comparisons): per FU_DQ-position chunk the extreme value that could
        // complete a pending partial -- the max when "x beats y" grows with x, else the min; NaN rows never complete
        // one. A continuation skips a whole chunk of its key when the summary cannot beat its deque's top: pops only
        // ever take the top, so no row of the chunk changes the deque but expiry, which the chunk's last ts applies.
        // (wc is free after the regrouping: 512 chunks x 8 B)
        const bool mono = stack && (m.gt != m.lt) && !m.ne && !(a.fu_skip & 128);
        const bool use_max = left == m.gt;
        T* s_cs = reinterpret_cast<T*>(&wc[0][0]);
        static_assert(FU_ROWS / FU_DQ * sizeof(int64_t) <= sizeof(wc), "chunk summaries fit the regrouping counters");
        if (mono) {
            T ext = use_max ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max();
#pragma unroll
            for (int i = 0; i < FU_DQ; ++i) {
                const T x = SAME ? C::get(cx[i]) : C::get(cvt(cx[i], kind, (uint8_t)K));
                if (p0 + i < nr && x == x) ext = use_max ? (x > ext ? x : ext) : (x < ext ? x : ext);
            }
            if (p0 < FU_ROWS) s_cs[t] = ext;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < FU_DQ; ++i) {
            const int q = p0 + i;
            if (q >= pe) break;
            const uint32_t tq = cts[i];
            const int64_t xr = cx[i];
            const T x = SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K));
            step(q, tq, x);
            // e1: this lane's own (non-halo) rows start partials, visible from the next row on
            if (crow[i] < own && c0_at(q, xr, x) && (!stack || x == x)) {
                if (!pend) tf = tq;
                pend |= 1u << i;
                ytop = x;
            }
            if (q + 1 == cur_end) {  // the key's staged rows end here: its pending partials ran off
                for (; pend; pend &= pend - 1) s_res[sw(p0 + __builtin_ctz(pend))] = ran_res(p0 + __builtin_ctz(pend));
                if (q + 1 < pe) cur_end = (int)lend[s_lk[sw(q + 1)]];
            }
        }
        // continuation over the key's following positions (no pushes) until the deque drains
        // software-pipelined: row q + 1 is read from LDS while row q is processed (the step's branches depend on
        // the row, so without this every step waits out an LDS round trip)
        if (pe < cur_end && pend && mono) {
            int q = pe;  // chunk-aligned (pe = p0 + FU_DQ)
#pragma unroll 1
            while (q < cur_end && pend) {
                if (q + FU_DQ <= cur_end) {  // a whole chunk of this key
                    const T cs = s_cs[q / FU_DQ];
                    if (!(left ? cmp_m(m, cs, ytop) : cmp_m(m, ytop, cs))) {
                        const uint32_t tl = s_ts[sw(q + FU_DQ - 1)];  // the chunk's last (latest) row
                        while (pend && (uint64_t)(tl - tf) > within_u) {
                            pend &= pend - 1;
                            if (pend) tf = s_ts[sw(p0 + __builtin_ctz(pend))];
                        }
                        q += FU_DQ;
                        continue;
                    }
                }
                const int qe = min(cur_end, q + FU_DQ);
#pragma unroll 1
                for (; q < qe && pend; ++q) {
                    const int64_t xr = s_x[sw(q)];
                    step(q, s_ts[sw(q)], SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K)));
                }
            }
        } else if (pe < cur_end && pend) {
            uint32_t tn = s_ts[sw(pe)];
            int64_t xn = s_x[sw(pe)];
#pragma unroll 1
            for (int q = pe; q < cur_end && pend; ++q) {
                const uint32_t tq = tn;
                const int64_t xr = xn;
                if (q + 1 < cur_end) {
                    tn = s_ts[sw(q + 1)];
                    xn = s_x[sw(q + 1)];
                }
                step(q, tq, SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K)));
            }
        }
        for (; pend; pend &= pend - 1) s_res[sw(p0 + __builtin_ctz(pend))] = ran_res(p0 + __builtin_ctz(pend));
    } else if constexpr (!FIX) {
        // ---- forward scans: one lane per candidate, its key's run in LDS
#pragma unroll 1
        for (int k = 0; k < FU_PT; ++k) {
            const int pos = k * FU_THREADS + t;
            if (!(pos < nr && s_row[sw(pos)] < own)) continue;
            const int64_t p = lo + s_row[sw(pos)];
            const int64_t xr = s_x[sw(pos)];
            const T xv = SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K));
            if (!c0_at(pos, xr, xv)) continue;
            // the e1 operand of the e2 filter, hoisted (null -> the compare is false for every row)
            T y = kc;
            CmpMask mm = m;
            if (stream_e1) {
                if (e1_is_x) {
                    y = xv;
                } else {
                    if (a.nulls[sp.e1_col] && a.nulls[sp.e1_col][p]) mm = CmpMask{false, false, false, false};
                    y = C::get(cvt(load_col(a.cols[sp.e1_col], sp.e1_col_kind, p), sp.e1_col_kind, (uint8_t)K));
                }
            }
            const uint32_t t0 = s_ts[sw(pos)];
            int end = (int)lend[s_lk[sw(pos)]];
            if (!FU_OK(end <= nr && end > pos, 4)) end = pos + 1;
            if (a.fu_skip & 1) end = pos + 1;
            uint16_t out = ran_res(pos);
            for (int q = pos + 1; q < end; ++q) {
                if ((uint64_t)(s_ts[sw(q)] - t0) > within_u) { out = R_NONE; break; }  // isExpired: dead
                const T x = SAME ? C::get(s_x[sw(q)]) : C::get(cvt(s_x[sw(q)], kind, (uint8_t)K));
                if (left ? cmp_m(mm, x, y) : cmp_m(mm, y, x)) { out = (uint16_t)q; break; }
            }
            s_res[sw(pos)] = out;
        }
    }
    __syncthreads();
    // records leave in the order of their e1 ROW (time order within the block), not of the regrouped position: the
    // delivery-order export then gathers each block's records nearly sequentially (in regrouped order a cache line of
    // records spanned the whole segment's time: its gather fetched 3.5x the record bytes, r5ox). Position of row r:
    // s_inv[r], in the values' LDS, free after the matching
#if SDG_FU_ROWORDER
    uint16_t* const s_inv = reinterpret_cast<uint16_t*>(&s_x[0]);
#pragma unroll
    for (int k = 0; k < FU_PT; ++k) {
        const int pos = k * FU_THREADS + t;
        if (pos < nr) s_inv[s_row[sw(pos)]] = (uint16_t)pos;
    }
    __syncthreads();
    auto pos_of = [&](int k) -> int {
        const int row = k * FU_THREADS + t;
        return row < nr ? (int)s_inv[row] : row;
    };
#else
    auto pos_of = [&](int k) -> int { return k * FU_THREADS + t; };
#endif
    uint32_t res[FU_PT];
#pragma unroll
    for (int k = 0; k < FU_PT; ++k) {
        const int pos = pos_of(k);
        const uint16_t r16 = k * FU_THREADS + t < nr ? s_res[sw(pos)] : R_NONE;
        const uint32_t out = r16 == R_NONE ? MQ_NONE : r16 == R_CARRY ? MQ_CARRY : r16 == R_OVF ? MQ_OVF : (uint32_t)r16;
        res[k] = out;
        const uint64_t bm = __ballot(out < MQ_OVF), bc = __ballot(out == MQ_CARRY), bo = __ballot(out == MQ_OVF);
        if (lane == 0) {
            wcnt[0][k][w] = (uint32_t)__popcll(bm);
            wcnt[1][k][w] = (uint32_t)__popcll(bc);
            wcnt[2][k][w] = (uint32_t)__popcll(bo);
        }
    }
    FU_TRACE(5);
    __syncthreads();
    // per counter (matches / carries / overflow rows): exclusive prefix over (round, wave) -- one wave per counter,
    // a lane per count (a shuffle scan; one thread walking the FU_PT x NW counts was a chain of dependent LDS round
    // trips), then the block's reservation
    static_assert(FU_PT * NW <= 64, "chain_fused_k: one wave scans a counter's (round, wave) counts");
    if (w < 3) {
        const int ci = w;
        const bool on = lane < FU_PT * NW;
        const uint32_t c = on ? wcnt[ci][lane / NW][lane % NW] : 0u;
        uint32_t inc = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off);
            if (lane >= off) inc += y;
        }
        if (on) wcnt[ci][lane / NW][lane % NW] = inc - c;
        const uint32_t run = __shfl(inc, 63);
        if (lane == 0) {
            unsigned long long* ctr = ci == 0 ? a.out_count : ci == 1 ? a.carry_count : a.ovf_count;
            if (a.fu_skip & 32) bbase[ci] = ci == 0 ? (unsigned long long)v * fown : 0ull;  // phase timing only
            else bbase[ci] = run ? atomicAdd(ctr, (unsigned long long)run) : 0ull;
        }
    }
    __syncthreads();
    // ---- emit matches: slots and rows of every round first (LDS only), then every load of every round, then
    // the stores. Loads are issued before any store: gfx9's vmcnt retires loads and stores in issue order, so a
    // load issued after a store would wait for that store too. --------------------------------------------------
    if (a.fu_skip & 2) return;
    constexpr uint32_t NOSLOT = 0xFFFFFFFFu;
    uint32_t slot[FU_PT], prow[FU_PT], qrow[FU_PT];
    bool any_co = false;  // this lane has carries / overflow rows
#pragma unroll
    for (int k = 0; k < FU_PT; ++k) {
        const uint32_t out = res[k];
        const uint64_t bm = __ballot(out < MQ_OVF);
        const int pos = pos_of(k);
        slot[k] = NOSLOT;
        prow[k] = qrow[k] = 0;
        any_co |= out == MQ_CARRY || out == MQ_OVF;
        if (out < MQ_OVF) {
            const uint64_t sl = bbase[0] + wcnt[0][k][w] + (uint32_t)__popcll(bm & lt);
            if (sl >= (uint64_t)a.out_cap) {
                atomicOr(&a.flags[0], 1);
            } else {
                slot[k] = (uint32_t)sl;
                prow[k] = s_row[sw(pos)];
                qrow[k] = FU_OK(out < (uint32_t)nr, 5) ? s_row[sw(out)] : s_row[sw(pos)];
            }
        }
    }
    FU_TRACE(6);
    // the common select: <= 2 plain 8-byte attributes of e1 / e2 without nulls (block-uniform)
    const int n_out = sp.n_out;
    Instr in0 = {}, in1 = {};
    if (n_out >= 1) in0 = load_instr(&sp.out_ins[0]);
    if (n_out >= 2) in1 = load_instr(&sp.out_ins[1]);
    auto plain8 = [&](const Instr& in) {
        return (in.c == 0 || in.c == -1) && in.a < 2 && (in.k == VK_I64 || in.k == VK_F64) && !a.nulls[in.b];
    };
    const bool fast = n_out <= 2 && (n_out < 1 || plain8(in0)) && (n_out < 2 || plain8(in1));
    const int jfrom = fast ? n_out : 0;  // output columns left to the general loop below
    {
        const int64_t* c0p = n_out >= 1 ? (const int64_t*)a.cols[in0.b] : nullptr;
        const int64_t* c1p = n_out >= 2 ? (const int64_t*)a.cols[in1.b] : nullptr;
        // emission-only columns in arrival order: read at the rows' original positions (op / oq)
        const int64_t* o0 = OC && n_out >= 1 && ((a.ocol_mask >> in0.b) & 1u) ? (const int64_t*)a.ocols[in0.b] : nullptr;
        const int64_t* o1 = OC && n_out >= 2 && ((a.ocol_mask >> in1.b) & 1u) ? (const int64_t*)a.ocols[in1.b] : nullptr;
        int64_t* const ov0 = a.out_vals;
        int64_t* const ov1 = a.out_vals + a.out_cap;
        // FU_EH rounds at a time: their loads, then their stores. All FU_PT rounds at once needs 24 more VGPRs than
        // the 8-waves-per-SIMD build has (64): it spilled the values to scratch and waited on every load (r3zb)
        constexpr int FU_EH = W >= 8 ? 2 : FU_PT;
#pragma unroll
        for (int h = 0; h < FU_PT; h += FU_EH) {
            uint32_t op[FU_EH], oq[FU_EH];
            int64_t v0[FU_EH], v1[FU_EH];
#pragma unroll
            for (int i = 0; i < FU_EH; ++i) {
                const int k = h + i;
                if (slot[k] != NOSLOT) {
                    op[i] = ONEK ? (uint32_t)orig_of(a, lo + prow[k]) : a.orig[lo + prow[k]];
                    oq[i] = ONEK ? (uint32_t)orig_of(a, lo + qrow[k]) : a.orig[lo + qrow[k]];
                    if (fast && n_out >= 1) v0[i] = OC && o0 ? o0[in0.a == 0 ? op[i] : oq[i]] : c0p[lo + (in0.a == 0 ? prow[k] : qrow[k])];
                    if (fast && n_out >= 2) v1[i] = OC && o1 ? o1[in1.a == 0 ? op[i] : oq[i]] : c1p[lo + (in1.a == 0 ? prow[k] : qrow[k])];
                }
            }
#pragma unroll
            for (int i = 0; i < FU_EH; ++i) {
                const int k = h + i;
                if (slot[k] != NOSLOT) {
                    a.out_ts[slot[k]] = tbase + (int64_t)s_ts[sw(res[k])];
                    a.out_emit_seq[slot[k]] = a.seq_base + (int64_t)oq[i];
                    a.out_first_seq[slot[k]] = a.seq_base + (int64_t)op[i];
                    if (fast && n_out >= 1) ov0[slot[k]] = v0[i];
                    if (fast && n_out >= 2) ov1[slot[k]] = v1[i];
                }
            }
        }
    }
    uint32_t nm[FU_PT];
#pragma unroll
    for (int k = 0; k < FU_PT; ++k) nm[k] = 0;
    for (int j = jfrom; j < n_out; ++j) {
        const Instr in = load_instr(&sp.out_ins[j]);  // a plain attribute (the fused path has no select bytecode)
        const bool ok = (in.c == 0 || in.c == -1) && in.a < 2;
        const uint8_t* np = a.nulls[in.b];
        int64_t* const ov = a.out_vals + (int64_t)j * a.out_cap;
#pragma unroll
        for (int k = 0; k < FU_PT; ++k)
            if (slot[k] != NOSLOT)
                ov[slot[k]] = !ok ? 0 : OC ? col_at(a, in.b, in.k, lo + (in.a == 0 ? prow[k] : qrow[k]))
                                           : load_col(a.cols[in.b], in.k, lo + (in.a == 0 ? prow[k] : qrow[k]));
        if (!ok || np) {
#pragma unroll
            for (int k = 0; k < FU_PT; ++k)
                if (slot[k] != NOSLOT && (!ok || np[lo + (in.a == 0 ? prow[k] : qrow[k])])) nm[k] |= 1u << j;
        }
    }
    if (a.write_nulls) {
#pragma unroll
        for (int k = 0; k < FU_PT; ++k)
            if (slot[k] != NOSLOT) a.out_nulls[slot[k]] = nm[k];
    }
    // ---- carries / overflow rows (few: the batch end, long windows) ---------------------------------------------
    FU_TRACE(7);
    if (__ballot(any_co) == 0) { FU_TRACE(100); return; }  // wave-uniform
#pragma unroll 1
    for (int k = 0; k < FU_PT; ++k) {
        const uint32_t out = res[k];
        const uint64_t bc = __ballot(out == MQ_CARRY), bo = __ballot(out == MQ_OVF);
        if (out != MQ_CARRY && out != MQ_OVF) continue;
        const int pos = pos_of(k);
        const int64_t p = lo + s_row[sw(pos)];
        if (out == MQ_CARRY) {
            const int64_t cs = (int64_t)bbase[1] + wcnt[1][k][w] + __popcll(bc & lt);
            if (cs >= a.carry_cap) atomicOr(&a.flags[0], 1);
            else if (FU_OK(p < a.n, 7))
                emit_carry(a, View{}, cs, p, ((uint32_t)s_lk[sw(pos)] << a.bbits) | (uint32_t)b, a.seq_base + (ONEK ? orig_of(a, p) : (int64_t)a.orig[p]));
        } else {
            const int64_t os = (int64_t)bbase[2] + wcnt[2][k][w] + __popcll(bo & lt);
            if (FU_OK(os < a.n, 8)) a.ovf_rows[os] = (uint32_t)p;  // os < the batch's rows (capacity n)
        }
    }
    FU_TRACE(100);
}

// fused path: partials whose scan left the staged rows -- the forward scan over the rest of the key's bucket
// in HBM (key-filtered), then emitted directly (match / carry)
__global__ __launch_bounds__(256) void chain_fovf_k(const ChainArgs* __restrict__ pa) {
    const ChainArgs& a = *pa;
    const int64_t total = (int64_t)*a.ovf_count;
    for (int64_t i0 = (int64_t)blockIdx.x * 256; i0 < total; i0 += (int64_t)gridDim.x * 256) {
        const int64_t i = i0 + threadIdx.x;
        bool has = false, carry = false;
        int64_t p = -1, qhit = -1;
        uint32_t key = 0;
        ChainAcc acc{&a, View{}, -1, -1, -1};
        if (i < total) {
            p = a.ovf_rows[i];
            acc.r0 = p;
            int bl = 0, bh = a.nb;  // the bucket of row p: the last one starting at or before it
            while (bh - bl > 1) {
                const int mid = (bl + bh) >> 1;
                if ((int64_t)a.bstart[mid] <= p) bl = mid;
                else bh = mid;
            }
            key = a.lkey ? (((uint32_t)a.lkey[p] << a.bbits) | (uint32_t)bl) : (a.key ? a.key[p] : 0u);
            const int64_t end = a.bstart[bl + 1];
            const int64_t q = chain_scan<false>(a, acc, p + 1, end, vts(a, p), nullptr, 0, key);
            if (q >= 0) { has = true; qhit = q; }
            else if (q == -2 && !a.sub_dead) carry = true;  // (a sub-batch's bucket end: dead, its halo)
        }
        const int64_t slot = wave_reserve(has, a.out_count);
        const int64_t seq = p >= 0 ? a.seq_base + orig_of(a, p) : 0;
        if (has) {
            if (slot >= a.out_cap) atomicOr(&a.flags[0], 1);
            else emit_match<false>(a, acc, slot, qhit, key, seq, nullptr, 0);
        }
        const int64_t cs = wave_reserve(carry, a.carry_count);
        if (carry) {
            if (cs >= a.carry_cap) atomicOr(&a.flags[0], 1);
            else emit_carry(a, View{}, cs, p, key, seq);
        }
    }
}

}  // namespace

size_t chain_lds_bytes(const ChainArgs& a) {
    if (a.mq_in) return (a.lds_stack ? (size_t)STACK * CM_THREADS * 8 : 0) + (size_t)CM_EPT * CM_THREADS * 4;
    size_t b = (a.lds_stack ? (size_t)STACK * CM_THREADS * 8 : 0) + (size_t)(1 + a.n_stage) * CM_ROWS * 8;
    b += a.qstream ? CM_ROWS : 0;
    b = (b + 3) & ~size_t(3);
    return b + (size_t)CM_EPT * CM_THREADS * 4;
}

// ---------------------------------------------------------------------------------------------------------
// Sorted-view matcher (the radix path's counterpart of chain_fused_k, for key counts past the bucket path): the view
// is fully key-sorted (keygroup), so a block stages FU_ROWS consecutive sorted rows -- FU_OWN own rows plus a halo --
// coalesced into LDS and every key's run is already contiguous: no regrouping, run boundaries are key changes. The
// same chunked monotone deque (chain_deque_k), then the matches emitted straight from the block (no mq
// round trip through HBM, no separate emission kernel).
// Carried partials of the previous batch are FOLDED into the view (a.fold): the first radix pass read them as leading
// rows (orig = SV_CARRIED | carry index), so the stable sort puts them at the start of their key's run. They are not
// events: no deque step, no e1 filter; each resolves with a forward scan over the run (their order among themselves
// is the arbitrary carry-out order, which a forward scan does not depend on). No separate carry kernel.
// A partial whose run is cut by the staged rows (the key continues past the halo) goes to chain_sovf_k, which scans
// the rest of the run in HBM; one whose run ends in the batch is carried.
constexpr uint32_t SV_CARRIED = 0x80000000u;   // orig flag / s_key flag of a folded carried partial
constexpr uint32_t SV_KEY = 0x7FFFFFFFu;
__device__ __forceinline__ int64_t sv_seq(const ChainArgs& a, uint32_t o) {
    return (a.fold && (o & SV_CARRIED)) ? a.cin_seq[o & SV_KEY] : a.seq_base + (int64_t)o;
}

// group summaries of the sorted-view deque (stack mode, ordering comparisons): per SV_GROUP positions the extreme
// value that could complete a pending partial -- the max when "x beats y" grows with x, else the min; carried rows
// (not events) and NaN rows never complete one. A continuation skips a whole group of its key when the summary cannot
// beat its deque's top (pops only ever take the top, so the group changes the deque by expiry alone, which the
// group's last -- latest -- row applies). C5's keys keep partials for ~half a batch: continuations run long there.
constexpr int SV_GROUP = 2 * FU_DQ;
static_assert(SV_GROUP == 2 * FU_DQ, "a group summary combines two lanes' chunks");

// SOP (round 6): as chain_fused_k's -- a compile-time ordering operator for `e2.x OP e1.x` on the scan column (e2's
// side folded in on the host); only the work-queue pass is compiled then
template <int K, bool SAME, int SOP = -1>
__global__ __launch_bounds__(FU_THREADS, 8) void chain_sorted_k(const ChainArgs* __restrict__ pa) {
    using C = KT<K>;
    using T = typename C::T;
    constexpr bool FIX = SOP >= 0;
    static_assert(!FIX || SOP == CMP_GT || SOP == CMP_GE || SOP == CMP_LT || SOP == CMP_LE, "SOP: an ordering operator");
    static_assert(!FIX || SAME, "SOP: the scan's own kind");
    constexpr int NW = FU_THREADS / 64;
    constexpr int WROWS = FU_ROWS / NW;
    const ChainArgs& a = *pa;
    const ChainSpec& sp = a.sp;
    __shared__ uint32_t s_ts[FU_ROWS];   // ts - the block's smallest staged ts
    __shared__ int64_t s_x[FU_ROWS];
    __shared__ uint32_t s_key[FU_ROWS];  // key | SV_CARRIED for a folded carried partial
    __shared__ uint16_t s_res[FU_ROWS];  // per position: e2 position | R_NONE | R_CARRY | R_OVF
    __shared__ uint32_t wcnt[3][FU_PT][NW];
    __shared__ unsigned long long bbase[3];
    __shared__ int64_t wmin[NW], wmax[NW];
    __shared__ int64_t s_gs[FU_ROWS / SV_GROUP];  // per SV_GROUP positions: the value that could complete a partial
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    // XCD-aware block order: neighbouring blocks (shared halo rows) on one XCD
    const uint32_t v = xcd_block(blockIdx.x, gridDim.x, (uint32_t)a.xcds);
    const int64_t lo = (int64_t)v * FU_OWN;
    if (lo >= a.n) return;  // block-uniform: the rounding of the grid
    const int own = (int)min((int64_t)FU_OWN, a.n - lo);
    const int nr = (int)min((int64_t)FU_ROWS, a.n - lo);
    const int col = sp.scan_col;
    const uint8_t kind = sp.scan_col_kind;
    const void* xcol = a.cols[col];
    // ---- stage: coalesced loads -------------------------------------------------------------------------------
    uint32_t rkey[FU_PT];
    int64_t rts[FU_PT], rx[FU_PT];
    int64_t tmn = INT64_MAX, tmx = INT64_MIN;
#pragma unroll
    for (int r = 0; r < FU_PT; ++r) {
        const int row = w * WROWS + r * 64 + lane;
        const int64_t g = lo + min(row, nr - 1);
        const uint32_t o = a.orig[g];
        rkey[r] = (a.key[g] & SV_KEY) | ((a.fold && (o & SV_CARRIED)) ? SV_CARRIED : 0u);
        rts[r] = vts(a, g);
        rx[r] = kind == VK_F64 || kind == VK_I64 ? ((const int64_t*)xcol)[g] : load_col(xcol, kind, g);
        tmn = min(tmn, rts[r]);
        tmx = max(tmx, rts[r]);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        tmn = min(tmn, (int64_t)__shfl_xor(tmn, d));
        tmx = max(tmx, (int64_t)__shfl_xor(tmx, d));
    }
    if (lane == 0) {
        wmin[w] = tmn;
        wmax[w] = tmx;
    }
    __syncthreads();
    int64_t tbase = wmin[0], tlast = wmax[0];
#pragma unroll
    for (int x = 1; x < NW; ++x) {
        tbase = min(tbase, wmin[x]);
        tlast = max(tlast, wmax[x]);
    }
    if (tlast - tbase > (int64_t)0xFFFFFFFF) {  // staged span does not fit the u32 offsets: the host reruns the
        if (t == 0) atomicOr(&a.flags[3], 1);     // batch on the lane deque path
        return;                                   // block-uniform
    }
#pragma unroll
    for (int r = 0; r < FU_PT; ++r) {
        const int row = w * WROWS + r * 64 + lane;
        if (row < nr) {
            s_ts[sw(row)] = (uint32_t)(rts[r] - tbase);
            s_x[sw(row)] = rx[r];
            s_key[sw(row)] = rkey[r];
            s_res[sw(row)] = R_NONE;
        }
    }
    // the key of the first row past the staged ones: a run cut at the staged end continues in HBM (R_OVF) only if
    // that row is of the same key; else the key's rows of this batch end there (R_CARRY)
    const uint32_t next_key = lo + nr < a.n ? (a.key[lo + nr] & SV_KEY) : 0xFFFFFFFFu;
    __syncthreads();
    if (a.fu_skip & 8) return;  // SDG_FU_SKIP phase timing (results invalid): loads + LDS staging only
    // per-key time order (the chain path's precondition): own positions against their predecessor
#pragma unroll
    for (int r = 0; r < FU_PT; ++r) {
        const int pos = r * FU_THREADS + t;
        if (pos >= own) continue;
        const uint32_t kp = s_key[sw(pos)];
        if (kp & SV_CARRIED) continue;  // (a carried partial has no successor constraint among carried ones)
        int64_t pk, pt;
        if (pos > 0) {
            pk = s_key[sw(pos - 1)] & SV_KEY;
            pt = (int64_t)s_ts[sw(pos - 1)];
        } else if (lo > 0) {
            pk = a.key[lo - 1] & SV_KEY;
            pt = vts(a, lo - 1) - tbase;
        } else {
            continue;
        }
        if (pk == (kp & SV_KEY) && pt > (int64_t)s_ts[sw(pos)]) atomicOr(&a.flags[1], 1);
    }
    const CmpMask m = cmp_mask(sp.scan_mode == SCAN_TRUE ? OP_ALWAYS : sp.scan_op);
    const bool left = sp.scan_e2_left;
    const uint64_t within_u = sp.has_within ? (uint64_t)sp.within_ms : ~0ull;
    const FastPred& f0 = sp.f0;
    const bool f0_on_x = a.f0_on_x;
    const bool f0_typed = f0_on_x && SAME && f0.t == K;
    const CmpMask m0 = cmp_mask(f0.op);
    const T k0 = C::get(f0.konst);
    const T kc = C::get(sp.scan_konst);
    const bool stream_e1 = sp.scan_mode == SCAN_E1;
    const bool e1_is_x = stream_e1 && sp.e1_col == col && sp.e1_col_kind == kind;
    auto xval = [&](int64_t xr) -> T { return SAME ? C::get(xr) : C::get(cvt(xr, kind, (uint8_t)K)); };
    auto c0_at = [&](int pos, int64_t xr, T xv) -> bool {
        if (f0_typed) return cmp_m(m0, xv, k0);
        if (f0_on_x) return cmp(f0.op, f0.t, cvt(xr, kind, f0.t), f0.konst);
        ChainAcc acc{&a, View{}, lo + pos, -1, -1};
        return f0.kind == FP_TRUE ? true : fast_pass(f0, acc);
    };
    // where a pending partial of key k goes when its run leaves the staged rows at position q (q = the first
    // position not of the run): the key's end in this batch (carry) or the HBM continuation (overflow scan)
    auto off_res = [&](int q, uint32_t k) -> uint16_t {
        return (q < nr || next_key != (k & SV_KEY)) ? R_CARRY : R_OVF;
    };
    const bool no_match = (a.fu_skip & 16) != 0;  // phase timing: everything but the matching
    const bool wq = FIX || (a.fu_skip & 1024) != 0;  // the wave work queue (as chain_fused_k) instead of deque + scans
    auto beats = [&](T x, T y, const CmpMask& mm) -> bool {  // x (a later row's value) completes the partial of y
        if constexpr (SOP == CMP_GT) return x > y;
        else if constexpr (SOP == CMP_GE) return x >= y;
        else if constexpr (SOP == CMP_LT) return x < y;
        else if constexpr (SOP == CMP_LE) return x <= y;
        else return left ? cmp_m(mm, x, y) : cmp_m(mm, y, x);
    };
    if (wq && !no_match) {
        // ---- wave work queue: every candidate (an own e1 row passing c0, or a carried partial) is an independent
        // forward scan over its key's run; a lane that resolves one takes the wave's next. The wave's candidates go
        // through a 128-entry ring in s_gs (free without the deque's summaries), one round of 64 positions at a time
        constexpr int WQ_U = SDG_WQ_U;
        static_assert(sizeof(s_gs) >= NW * 128 * sizeof(uint16_t), "a 128-entry candidate ring per wave fits s_gs");
        uint16_t* const ring = reinterpret_cast<uint16_t*>(s_gs) + w * 128;
        uint32_t cm = 0;  // bit r: this lane's position of round r is a candidate
#pragma unroll
        for (int r = 0; r < FU_PT; ++r) {
            const int pos = w * WROWS + r * 64 + lane;
            if (pos < own) {
                const bool carried = (s_key[sw(pos)] & SV_CARRIED) != 0;
                const int64_t xr = s_x[sw(pos)];
                if (carried || c0_at(pos, xr, xval(xr))) cm |= 1u << r;
            }
        }
        int filled = 0, head = 0, rn = 0;
        int p = -1, q = 0;
        uint32_t t0 = 0, kp = 0;
        T y = kc;
        CmpMask mm = m;
#pragma unroll 1
        for (;;) {
            const uint64_t need = __ballot(p < 0);
            if (need) {  // wave-uniform
                // refill: a round's candidates (<= 64) go in while that cannot overwrite an entry not yet taken
                while (rn < FU_PT && filled - head <= 64) {
                    const bool c = (cm >> rn) & 1u;
                    const uint64_t bm = __ballot(c);
                    if (c) ring[(filled + __popcll(bm & lanemask_lt())) & 127] = (uint16_t)(w * WROWS + rn * 64 + lane);
                    filled += __popcll(bm);
                    ++rn;
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                const int idx = head + __popcll(need & lanemask_lt());
                head += __popcll(need);
                if (p < 0 && idx < filled) {
                    p = ring[idx & 127];
                    t0 = s_ts[sw(p)];
                    kp = s_key[sw(p)] & SV_KEY;
                    q = p + 1;
                    const int64_t xr = s_x[sw(p)];
                    mm = m;
                    if (stream_e1) {
                        if (e1_is_x) {
                            y = xval(xr);
                        } else {
                            const int64_t g = lo + p;
                            if (a.nulls[sp.e1_col] && a.nulls[sp.e1_col][g]) mm = CmpMask{false, false, false, false};
                            y = C::get(cvt(load_col(a.cols[sp.e1_col], sp.e1_col_kind, g), sp.e1_col_kind, (uint8_t)K));
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();  // (every take of this round before the next refill writes)
                if (__ballot(p >= 0) == 0) break;
            }
            if (p >= 0) {
                int r = -1;  // -1 pending, else the s_res value
#pragma unroll
                for (int u = 0; u < WQ_U; ++u) {
                    if (r >= 0) break;
                    const int qq = q + u;
                    if (qq >= nr) { r = off_res(nr, kp); break; }  // the staged rows end with the key's run
                    const uint32_t kq = s_key[sw(qq)];
                    if ((kq & SV_KEY) != kp) { r = R_CARRY; break; }  // the key's rows of this batch end here
                    if (kq & SV_CARRIED) continue;                    // another carried partial: not an event
                    if ((uint64_t)(s_ts[sw(qq)] - t0) > within_u) { r = R_NONE; break; }  // isExpired: dead
                    const T x = xval(s_x[sw(qq)]);
                    if (beats(x, y, mm)) r = qq;
                }
                if (r >= 0) {
                    s_res[sw(p)] = (uint16_t)r;
                    p = -1;
                } else {
                    q += WQ_U;
                }
            }
        }
    } else if constexpr (!FIX) {
      if (a.fu_mode != DQ_OFF && !no_match) {
        // ---- monotone-deque pass: lane t owns positions [FU_DQ t, FU_DQ (t + 1)) ------------------------------
        const bool stack = a.fu_mode == DQ_STACK;
        const int p0 = t * FU_DQ;
        // the chunk's rows up front (all LDS reads in flight together); the deque holds only the lane's own
        // positions, so its front's ts and top's value are register selects
        uint32_t cts[FU_DQ], ckey[FU_DQ];
        int64_t cx[FU_DQ];
        T cxv[FU_DQ];
#pragma unroll
        for (int i = 0; i < FU_DQ; ++i) {
            const int q = min(p0 + i, FU_ROWS - 1);
            cts[i] = s_ts[sw(q)];
            cx[i] = s_x[sw(q)];
            ckey[i] = s_key[sw(q)];
            cxv[i] = xval(cx[i]);
        }
        auto ts_of = [&](int i) -> uint32_t {
            uint32_t r = cts[0];
#pragma unroll
            for (int j = 1; j < FU_DQ; ++j) r = i == j ? cts[j] : r;
            return r;
        };
        auto x_of = [&](int i) -> T {
            T r = cxv[0];
#pragma unroll
            for (int j = 1; j < FU_DQ; ++j) r = i == j ? cxv[j] : r;
            return r;
        };
        uint32_t pend = 0, tf = 0;
        T ytop = T(0);
        // branch-free step (SDG_FU_SKIP bit 512: the loops): the pending positions' ts and values are registers, so a
        // row's effect is two masks over the FU_DQ positions -- `live` (not expired: the expired ones are a prefix,
        // positions being in time order) and `beat` (completed: the pending values are monotone -- every push first
        // popped what it beats --, so the ones a row beats are exactly the suffix the pop loop takes; complete-all
        // mode: all or none). Measured neutral on C5 (10.63 vs 10.59 ms, r4j); on the fused matcher the register
        // copies cost more than the LDS round trips they save (2.91 vs 2.42 ms, r4k), so chain_fused_k keeps LDS.
        const bool bf = !(a.fu_skip & 512) && (!stack || (m.gt != m.lt && !m.ne));
        auto step = [&](int q, uint32_t tq, T x) {
            if (bf) {
                uint32_t beat = 0, live = 0;
#pragma unroll
                for (int i = 0; i < FU_DQ; ++i) {
                    live |= (uint32_t)((uint64_t)(tq - cts[i]) <= within_u) << i;
                    if (stack) beat |= (uint32_t)(left ? cmp_m(m, x, cxv[i]) : cmp_m(m, cxv[i], x)) << i;
                }
                if (!stack) beat = (left ? cmp_m(m, x, kc) : cmp_m(m, kc, x)) ? ~0u : 0u;
                pend &= live;
                const uint32_t done = pend & beat;
                pend &= ~done;
#pragma unroll
                for (int i = 0; i < FU_DQ; ++i)
                    if ((done >> i) & 1u) s_res[sw(p0 + i)] = (uint16_t)q;
                return;
            }
            while (pend && (uint64_t)(tq - tf) > within_u) {  // expireEvents: the expired prefix
                pend &= pend - 1;
                if (pend) tf = ts_of(__builtin_ctz(pend));
            }
            if (stack) {
                while (pend && (left ? cmp_m(m, x, ytop) : cmp_m(m, ytop, x))) {
                    const int tp = 31 - __builtin_clz(pend);
                    s_res[sw(p0 + tp)] = (uint16_t)q;
                    pend &= ~(1u << tp);
                    if (pend) ytop = x_of(31 - __builtin_clz(pend));
                }
            } else if (pend && (left ? cmp_m(m, x, kc) : cmp_m(m, kc, x))) {
                for (; pend; pend &= pend - 1) s_res[sw(p0 + __builtin_ctz(pend))] = (uint16_t)q;
            }
        };
        const bool mono = bf && stack && (m.gt != m.lt) && !m.ne && !(a.fu_skip & 128);
        const bool use_max = left == m.gt;
        T* s_gsum = reinterpret_cast<T*>(s_gs);
        if (mono) {  // (every lane: the pair combine is a cross-lane shuffle)
            T ext = use_max ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max();
#pragma unroll
            for (int i = 0; i < FU_DQ; ++i) {
                const T x = cxv[i];
                if (p0 + i < nr && !(ckey[i] & SV_CARRIED) && x == x) ext = use_max ? (x > ext ? x : ext) : (x < ext ? x : ext);
            }
            const T o = __shfl_xor(ext, 1);
            ext = use_max ? (o > ext ? o : ext) : (o < ext ? o : ext);
            if (!(t & 1)) s_gsum[t >> 1] = ext;
        }
        __syncthreads();
        const int pe = min(p0 + FU_DQ, own);  // (FU_OWN is a multiple of FU_DQ: a chunk is all own rows or none)
        uint32_t cur = p0 < own ? (ckey[0] & SV_KEY) : 0u;
#pragma unroll
        for (int i = 0; i < FU_DQ; ++i) {
            const int q = p0 + i;
            if (q >= pe) break;
            const uint32_t kq = ckey[i];
            if ((kq & SV_KEY) != cur) {  // the previous key's run ended inside the chunk: its partials are carried
                for (; pend; pend &= pend - 1) s_res[sw(p0 + __builtin_ctz(pend))] = R_CARRY;
                cur = kq & SV_KEY;
            }
            if (kq & SV_CARRIED) continue;  // a carried partial: resolved by its forward scan below
            const uint32_t tq = cts[i];
            const int64_t xr = cx[i];
            const T x = cxv[i];
            step(q, tq, x);
            if (c0_at(q, xr, x) && (!stack || x == x)) {  // e1: visible from the next row on
                if (!pend) tf = tq;
                pend |= 1u << i;
                ytop = x;
            }
        }
        // continuation over the key's following positions until the deque drains (whole groups that cannot complete
        // the deque's top are skipped, their last row's ts applied)
        int q = pe;
        while (pend && q < nr) {
            if (mono && (q & (SV_GROUP - 1)) == 0 && q + SV_GROUP <= nr &&
                (s_key[sw(q + SV_GROUP - 1)] & SV_KEY) == cur && (s_key[sw(q)] & SV_KEY) == cur) {
                const T cs = s_gsum[q / SV_GROUP];
                const T yt = x_of(31 - __builtin_clz(pend));
                if (!(left ? cmp_m(m, cs, yt) : cmp_m(m, yt, cs))) {
                    const uint32_t tl = s_ts[sw(q + SV_GROUP - 1)];
                    uint32_t live = 0;
#pragma unroll
                    for (int i = 0; i < FU_DQ; ++i) live |= (uint32_t)((uint64_t)(tl - cts[i]) <= within_u) << i;
                    pend &= live;
                    q += SV_GROUP;
                    continue;
                }
            }
            if ((s_key[sw(q)] & SV_KEY) != cur) break;
            step(q, s_ts[sw(q)], xval(s_x[sw(q)]));
            ++q;
        }
        if (pend) {
            const uint16_t rr = off_res(q, cur);
            for (; pend; pend &= pend - 1) s_res[sw(p0 + __builtin_ctz(pend))] = rr;
        }
      }
    }
    // ---- forward scans: carried partials (and every candidate without a deque mode) -------------------------
#pragma unroll 1
    for (int k = 0; k < FU_PT && !no_match && !wq; ++k) {
        const int pos = k * FU_THREADS + t;
        if (pos >= own) continue;
        const uint32_t kp = s_key[sw(pos)];
        const bool carried = (kp & SV_CARRIED) != 0;
        if (!carried && a.fu_mode != DQ_OFF) continue;
        const int64_t xr = s_x[sw(pos)];
        const T xv = xval(xr);
        if (!carried && !c0_at(pos, xr, xv)) continue;
        T y = kc;
        CmpMask mm = m;
        if (stream_e1) {
            if (e1_is_x) {
                y = xv;
            } else {
                const int64_t p = lo + pos;
                if (a.nulls[sp.e1_col] && a.nulls[sp.e1_col][p]) mm = CmpMask{false, false, false, false};
                y = C::get(cvt(load_col(a.cols[sp.e1_col], sp.e1_col_kind, p), sp.e1_col_kind, (uint8_t)K));
            }
        }
        const uint32_t t0 = s_ts[sw(pos)];
        uint16_t out = R_NONE;
        int q = pos + 1;
        for (; q < nr; ++q) {
            const uint32_t kq = s_key[sw(q)];
            if ((kq & SV_KEY) != (kp & SV_KEY)) break;
            if (kq & SV_CARRIED) continue;  // another carried partial: not an event
            if ((uint64_t)(s_ts[sw(q)] - t0) > within_u) { out = R_NONE; q = -1; break; }  // isExpired: dead
            const T x = xval(s_x[sw(q)]);
            if (left ? cmp_m(mm, x, y) : cmp_m(mm, y, x)) { out = (uint16_t)q; q = -1; break; }
        }
        if (q >= 0) out = off_res(q, kp);
        s_res[sw(pos)] = out;
    }
    __syncthreads();
    // ---- counts, one reservation per block and counter ----------------------------------------------------
    uint32_t res[FU_PT];
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int k = 0; k < FU_PT; ++k) {
        const int pos = k * FU_THREADS + t;
        const uint16_t r16 = pos < own ? s_res[sw(pos)] : R_NONE;
        const uint32_t out = r16 == R_NONE ? MQ_NONE : r16 == R_CARRY ? MQ_CARRY : r16 == R_OVF ? MQ_OVF : (uint32_t)r16;
        res[k] = out;
        const uint64_t bm = __ballot(out < MQ_OVF), bc = __ballot(out == MQ_CARRY), bo = __ballot(out == MQ_OVF);
        if (lane == 0) {
            wcnt[0][k][w] = (uint32_t)__popcll(bm);
            wcnt[1][k][w] = (uint32_t)__popcll(bc);
            wcnt[2][k][w] = (uint32_t)__popcll(bo);
        }
    }
    __syncthreads();
    if (t < 3) {
        uint32_t run = 0;
        for (int k = 0; k < FU_PT; ++k)
            for (int x = 0; x < NW; ++x) {
                const uint32_t c = wcnt[t][k][x];
                wcnt[t][k][x] = run;
                run += c;
            }
        unsigned long long* ctr = t == 0 ? a.out_count : t == 1 ? a.carry_count : a.ovf_count;
        bbase[t] = run ? atomicAdd(ctr, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    // ---- emit matches (loads of a group of rounds, then its stores: see chain_fused_k) ---------------------
    if (a.fu_skip & 2) return;  // phase timing: no emission
    constexpr uint32_t NOSLOT = 0xFFFFFFFFu;
    uint32_t slot[FU_PT];
    bool any_co = false;
#pragma unroll
    for (int k = 0; k < FU_PT; ++k) {
        const uint32_t out = res[k];
        const uint64_t bm = __ballot(out < MQ_OVF);
        slot[k] = NOSLOT;
        any_co |= out == MQ_CARRY || out == MQ_OVF;
        if (out < MQ_OVF) {
            const uint64_t sl = bbase[0] + wcnt[0][k][w] + (uint32_t)__popcll(bm & lt);
            if (sl >= (uint64_t)a.out_cap) atomicOr(&a.flags[0], 1);
            else slot[k] = (uint32_t)sl;
        }
    }
    const int n_out = sp.n_out;
    Instr in0 = {}, in1 = {};
    if (n_out >= 1) in0 = load_instr(&sp.out_ins[0]);
    if (n_out >= 2) in1 = load_instr(&sp.out_ins[1]);
    auto plain8 = [&](const Instr& in) {
        return (in.c == 0 || in.c == -1) && in.a < 2 && (in.k == VK_I64 || in.k == VK_F64) && !a.nulls[in.b];
    };
    const bool fast = n_out <= 2 && (n_out < 1 || plain8(in0)) && (n_out < 2 || plain8(in1));
    const int jfrom = fast ? n_out : 0;
    {
        const int64_t* c0p = n_out >= 1 ? (const int64_t*)a.cols[in0.b] : nullptr;
        const int64_t* c1p = n_out >= 2 ? (const int64_t*)a.cols[in1.b] : nullptr;
        int64_t* const ov0 = a.out_vals;
        int64_t* const ov1 = a.out_vals + a.out_cap;
        constexpr int EH = 2;
#pragma unroll
        for (int h = 0; h < FU_PT; h += EH) {
            uint32_t op[EH], oq[EH];
            int64_t v0[EH], v1[EH];
#pragma unroll
            for (int i = 0; i < EH; ++i) {
                const int k = h + i;
                if (slot[k] != NOSLOT) {
                    const int pos = k * FU_THREADS + t;
                    op[i] = a.orig[lo + pos];
                    oq[i] = a.orig[lo + res[k]];
                    if (fast && n_out >= 1) v0[i] = c0p[lo + (in0.a == 0 ? pos : (int)res[k])];
                    if (fast && n_out >= 2) v1[i] = c1p[lo + (in1.a == 0 ? pos : (int)res[k])];
                }
            }
#pragma unroll
            for (int i = 0; i < EH; ++i) {
                const int k = h + i;
                if (slot[k] != NOSLOT) {
                    a.out_ts[slot[k]] = tbase + (int64_t)s_ts[sw(res[k])];
                    a.out_emit_seq[slot[k]] = a.seq_base + (int64_t)oq[i];
                    a.out_first_seq[slot[k]] = sv_seq(a, op[i]);
                    if (fast && n_out >= 1) ov0[slot[k]] = v0[i];
                    if (fast && n_out >= 2) ov1[slot[k]] = v1[i];
                }
            }
        }
    }
    uint32_t nm[FU_PT];
#pragma unroll
    for (int k = 0; k < FU_PT; ++k) nm[k] = 0;
    for (int j = jfrom; j < n_out; ++j) {
        const Instr in = load_instr(&sp.out_ins[j]);
        const bool ok = (in.c == 0 || in.c == -1) && in.a < 2;
        const void* cp = a.cols[in.b];
        const uint8_t* np = a.nulls[in.b];
        int64_t* const ov = a.out_vals + (int64_t)j * a.out_cap;
#pragma unroll
        for (int k = 0; k < FU_PT; ++k) {
            if (slot[k] == NOSLOT) continue;
            const int64_t r = lo + (in.a == 0 ? k * FU_THREADS + t : (int)res[k]);
            ov[slot[k]] = ok ? load_col(cp, in.k, r) : 0;
            if (!ok || (np && np[r])) nm[k] |= 1u << j;
        }
    }
    if (a.write_nulls) {
#pragma unroll
        for (int k = 0; k < FU_PT; ++k)
            if (slot[k] != NOSLOT) a.out_nulls[slot[k]] = nm[k];
    }
    // ---- carries / overflow rows --------------------------------------------------------------------------
    if (__ballot(any_co) == 0) return;  // wave-uniform
#pragma unroll 1
    for (int k = 0; k < FU_PT; ++k) {
        const uint32_t out = res[k];
        const uint64_t bc = __ballot(out == MQ_CARRY), bo = __ballot(out == MQ_OVF);
        if (out != MQ_CARRY && out != MQ_OVF) continue;
        const int64_t p = lo + k * FU_THREADS + t;
        if (out == MQ_CARRY) {
            const int64_t cs = (int64_t)bbase[1] + wcnt[1][k][w] + __popcll(bc & lt);
            if (cs >= a.carry_cap) atomicOr(&a.flags[0], 1);
            else emit_carry(a, View{}, cs, p, a.key[p] & SV_KEY, sv_seq(a, a.orig[p]));
        } else {
            const int64_t os = (int64_t)bbase[2] + wcnt[2][k][w] + __popcll(bo & lt);
            if (os < a.n) a.ovf_rows[os] = (uint32_t)p;
        }
    }
}

// sorted view: partials whose key's run continues past the staged rows of their block. One wave per partial
// (CW_PER_WAVE per wave) scans the run's remaining rows 64 at a time; the block then emits the matches and carries.
template <int K>
__device__ int64_t sv_wave_scan(const ChainArgs& a, int64_t p, uint32_t kp, int64_t ts0, int64_t k, uint8_t op) {
    using C = KT<K>;
    const typename C::T y = C::get(k);
    const ChainSpec& sp = a.sp;
    const int col = sp.scan_col;
    const uint8_t kind = sp.scan_col_kind;
    const bool left = sp.scan_e2_left, always = op == OP_ALWAYS;
    const uint64_t within_u = sp.has_within ? (uint64_t)sp.within_ms : ~0ull;
    const CmpMask m = cmp_mask(op);
    const int lane = lane_id();
    for (int64_t q0 = p + 1; q0 < a.n; q0 += 64) {
        const int64_t q = q0 + lane;
        bool stop = false, hit = false, end = false;
        if (q >= a.n || (a.key[q] & SV_KEY) != kp) {
            end = true;  // the key's rows of this batch end: carried
        } else if (!(a.fold && (a.orig[q] & SV_CARRIED))) {
            if ((uint64_t)(vts(a, q) - ts0) > within_u) stop = true;  // isExpired at this event of the key
            else if (always) hit = true;
            else hit = left ? cmp_m(m, C::get(cvt(load_col(a.cols[col], kind, q), kind, (uint8_t)K)), y)
                            : cmp_m(m, y, C::get(cvt(load_col(a.cols[col], kind, q), kind, (uint8_t)K)));
        }
        const uint64_t bh = __ballot(hit), bs = __ballot(stop), be = __ballot(end);
        const uint64_t any = bh | bs | be;
        if (any) {
            const int l = __ffsll((unsigned long long)any) - 1;
            return ((bh >> l) & 1u) ? q0 + l : ((bs >> l) & 1u) ? -1 : -2;
        }
    }
    return -2;
}

__global__ __launch_bounds__(256, 8) void chain_sovf_k(const ChainArgs* __restrict__ pa) {
    const ChainArgs& a = *pa;
    const ChainSpec& sp = a.sp;
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int64_t total = (int64_t)*a.ovf_count;
    // grid-stride over groups of 4 x CW_PER_WAVE partials (block-uniform bounds: block_reserve2 needs every thread)
    for (int64_t g0 = (int64_t)blockIdx.x * 4 * CW_PER_WAVE; g0 < total; g0 += (int64_t)gridDim.x * 4 * CW_PER_WAVE) {
        const int64_t c_base = g0 + (int64_t)w * CW_PER_WAVE;
        int64_t mine = -1;
        for (int i = 0; i < CW_PER_WAVE; ++i) {
            const int64_t c = c_base + i;
            if (c >= total) break;  // wave-uniform
            const int64_t p = a.ovf_rows[c];
            const uint32_t kp = a.key[p] & SV_KEY;
            int64_t k = sp.scan_konst;
            uint8_t op = sp.scan_op;
            if (sp.scan_mode == SCAN_TRUE) {
                op = OP_ALWAYS;
            } else if (sp.scan_mode == SCAN_E1) {
                if (a.nulls[sp.e1_col] && a.nulls[sp.e1_col][p]) op = OP_NEVER;
                else k = cvt(load_col(a.cols[sp.e1_col], sp.e1_col_kind, p), sp.e1_col_kind, sp.scan_t);
            }
            int64_t r;
            switch (sp.scan_t) {
                case VK_I32: r = sv_wave_scan<VK_I32>(a, p, kp, vts(a, p), k, op); break;
                case VK_I64: r = sv_wave_scan<VK_I64>(a, p, kp, vts(a, p), k, op); break;
                case VK_F32: r = sv_wave_scan<VK_F32>(a, p, kp, vts(a, p), k, op); break;
                case VK_F64: r = sv_wave_scan<VK_F64>(a, p, kp, vts(a, p), k, op); break;
                case VK_BOOL: r = sv_wave_scan<VK_BOOL>(a, p, kp, vts(a, p), k, op); break;
                default: r = sv_wave_scan<VK_STR>(a, p, kp, vts(a, p), k, op); break;
            }
            if (lane == i) mine = r;
        }
        const int64_t c = c_base + lane;
        const bool valid = lane < CW_PER_WAVE && c < total;
        const bool has = valid && mine >= 0, carry = valid && mine == -2;
        int64_t slot, cs;
        block_reserve2<256>(has, carry, a.out_count, a.carry_count, &slot, &cs);
        if (valid) {
            const int64_t p = a.ovf_rows[c];
            if (has) {
                if (slot >= a.out_cap) {
                    atomicOr(&a.flags[0], 1);
                } else {
                    ChainAcc acc{&a, View{}, p, -1, -1};
                    emit_match<false>(a, acc, slot, mine, a.key[p] & SV_KEY, sv_seq(a, a.orig[p]), nullptr, 0);
                }
            }
            if (carry) {
                if (cs >= a.carry_cap) atomicOr(&a.flags[0], 1);
                else emit_carry(a, View{}, cs, p, a.key[p] & SV_KEY, sv_seq(a, a.orig[p]));
            }
        }
        __syncthreads();  // block_reserve2's shared words are reused by the next group
    }
}

void chain_match(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream) {
    if (a.n <= 0) return;
    const dim3 grid((unsigned)((a.n + CM_TILE - 1) / CM_TILE));
    if (a.generic)
        hipLaunchKernelGGL(chain_match_k<true>, grid, dim3(CM_THREADS), chain_lds_bytes(a), stream, d_a);
    else
        hipLaunchKernelGGL(chain_match_k<false>, grid, dim3(CM_THREADS), chain_lds_bytes(a), stream, d_a);
}

void chain_deque(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream) {
    if (a.n <= 0) return;
    const int64_t lane_rows = a.dq_lane > 0 ? a.dq_lane : DQ_CHUNK;
    if (a.dq_any) {
        const dim3 sg((unsigned)((a.n + 255) / 256));
        switch (a.sp.scan_t) {
            case VK_I32: hipLaunchKernelGGL(chain_dq_summ_k<VK_I32>, sg, dim3(256), 0, stream, d_a); break;
            case VK_I64: hipLaunchKernelGGL(chain_dq_summ_k<VK_I64>, sg, dim3(256), 0, stream, d_a); break;
            case VK_F32: hipLaunchKernelGGL(chain_dq_summ_k<VK_F32>, sg, dim3(256), 0, stream, d_a); break;
            case VK_F64: hipLaunchKernelGGL(chain_dq_summ_k<VK_F64>, sg, dim3(256), 0, stream, d_a); break;
            default: break;  // engine.cpp sets dq_any for numeric scans only
        }
    }
    const dim3 grid((unsigned)((a.n + DQ_THREADS * lane_rows - 1) / (DQ_THREADS * lane_rows)));
    switch (a.sp.scan_t) {
        case VK_I32: hipLaunchKernelGGL(chain_deque_k<VK_I32>, grid, dim3(DQ_THREADS), 0, stream, d_a); break;
        case VK_I64: hipLaunchKernelGGL(chain_deque_k<VK_I64>, grid, dim3(DQ_THREADS), 0, stream, d_a); break;
        case VK_F32: hipLaunchKernelGGL(chain_deque_k<VK_F32>, grid, dim3(DQ_THREADS), 0, stream, d_a); break;
        case VK_F64: hipLaunchKernelGGL(chain_deque_k<VK_F64>, grid, dim3(DQ_THREADS), 0, stream, d_a); break;
        case VK_BOOL: hipLaunchKernelGGL(chain_deque_k<VK_BOOL>, grid, dim3(DQ_THREADS), 0, stream, d_a); break;
        default: hipLaunchKernelGGL(chain_deque_k<VK_STR>, grid, dim3(DQ_THREADS), 0, stream, d_a); break;
    }
    if (!a.generic && a.sp.scan_mode != SCAN_GENERIC && !a.bstart && !getenv("SDG_OVF_LANE"))
        hipLaunchKernelGGL(chain_ovf_wave_k,
                           dim3((unsigned)std::min<int64_t>(4096, (a.n + 4 * CW_PER_WAVE - 1) / (4 * CW_PER_WAVE))),
                           dim3(256), 0, stream, d_a);  // grid-stride over ovf_count (<= n)
    else
        hipLaunchKernelGGL(chain_ovf_k, dim3(512), dim3(256), 0, stream, d_a);
}

void chain_carry(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream) {
    if (a.cin_n <= 0) return;
    // a wave per carried partial pays when its key's rows are many (one key, C1; 10^4 keys, C2: ~10^4 rows each);
    // with short segments (C5: ~21 rows per key) one lane per partial is 3.7x faster (profiles/r3i_c5_carry_ab.log)
    static const int force = getenv("SDG_CARRY_LANE") ? 1 : getenv("SDG_CARRY_WAVE") ? 2 : 0;
    const bool short_segments = a.key && a.K > 0 && a.n <= (int64_t)a.K * 256;
    const bool lane = force ? force == 1 : short_segments;
    if (!a.generic && a.sp.scan_mode != SCAN_GENERIC && !lane)
        hipLaunchKernelGGL(chain_carry_wave_k, dim3((unsigned)((a.cin_n + 4 * CW_PER_WAVE - 1) / (4 * CW_PER_WAVE))),
                           dim3(256), 0, stream, d_a);
    else
        hipLaunchKernelGGL(chain_carry_k, dim3((unsigned)((a.cin_n + 255) / 256)), dim3(256), 0, stream, d_a);
}

#ifndef SDG_FU_W8_DEFAULT
#define SDG_FU_W8_DEFAULT 1  // r3v: fused 2.52 ms at 8 vs 2.68 ms at 6 waves per SIMD (C2, same box)
#endif
int64_t chain_fused_grid(int64_t n, int nb, int own) {
    return xcd_round((n + own - 1) / own + nb);
}

bool chain_fused_ocols_ok(const ChainArgs& a) {  // the OC instantiation: the scan's own kind, 8 waves per SIMD
    static const char* wv = getenv("SDG_FU_WPS");
    const bool w8 = wv ? atoi(wv) == 8 : SDG_FU_W8_DEFAULT;
    return a.sp.scan_col_kind == a.sp.scan_t && w8 && !a.fu_check_ts;
}

void chain_fused(const ChainArgs& a, const ChainArgs* d_a, int64_t grid, hipStream_t stream) {
    if (a.n <= 0) return;
    if (a.ocol_mask && !chain_fused_ocols_ok(a)) throw std::runtime_error("chain_fused: arrival-order columns need the OC build");
    const dim3 g((unsigned)grid), b(FU_THREADS);
    const bool same = a.sp.scan_col_kind == a.sp.scan_t;
    static const char* wv = getenv("SDG_FU_WPS");  // A/B: 8 (four blocks per CU) or 6
    const bool w8 = wv ? atoi(wv) == 8 : SDG_FU_W8_DEFAULT;
#define FU_LAUNCH(KK)                                                                                    \
    do {                                                                                                 \
        if (a.ocol_mask) hipLaunchKernelGGL((chain_fused_k<KK, true, 8, false, true>), g, b, 0, stream, d_a); \
        else if (a.fu_check_ts && same) hipLaunchKernelGGL((chain_fused_k<KK, true, 8, true>), g, b, 0, stream, d_a); \
        else if (a.fu_check_ts) hipLaunchKernelGGL((chain_fused_k<KK, false, 8, true>), g, b, 0, stream, d_a); \
        else if (same && w8) hipLaunchKernelGGL((chain_fused_k<KK, true, 8>), g, b, 0, stream, d_a);     \
        else if (same) hipLaunchKernelGGL((chain_fused_k<KK, true, 6>), g, b, 0, stream, d_a);          \
        else if (w8) hipLaunchKernelGGL((chain_fused_k<KK, false, 8>), g, b, 0, stream, d_a);           \
        else hipLaunchKernelGGL((chain_fused_k<KK, false, 6>), g, b, 0, stream, d_a);                   \
    } while (0)
    // the compile-time operator build (SOP): `e2.x OP e1.x` on the scan column, an ordering OP, the work queue
    const bool e1_is_x = a.sp.scan_mode == SCAN_E1 && a.sp.e1_col == a.sp.scan_col && a.sp.e1_col_kind == a.sp.scan_col_kind;
    const uint8_t op = a.sp.scan_op;
    const bool ord = op == CMP_GT || op == CMP_GE || op == CMP_LT || op == CMP_LE;
    static const bool no_sop = getenv("SDG_FU_NO_SOP") != nullptr;  // A/B: the run-time operator build
    if (!no_sop && !a.ocol_mask && !a.fu_check_ts && same && w8 && e1_is_x && ord && !(a.fu_skip & 256) && a.lkey &&
        (a.sp.scan_t == VK_F64 || a.sp.scan_t == VK_I64 || a.sp.scan_t == VK_I32 || a.sp.scan_t == VK_F32)) {
        // x beats y: e2 on the left (e2.x OP e1.x) is x OP y, else y OP x = x OP' y (the flipped ordering)
        const uint8_t sop = a.sp.scan_e2_left ? op : op == CMP_GT ? CMP_LT : op == CMP_GE ? CMP_LE : op == CMP_LT ? CMP_GT : CMP_GE;
#define FU_SOP(KK)                                                                                                    \
    do {                                                                                                              \
        if (sop == CMP_GT) hipLaunchKernelGGL((chain_fused_k<KK, true, SDG_FU_W8, false, false, CMP_GT>), g, b, 0, stream, d_a); \
        else if (sop == CMP_GE) hipLaunchKernelGGL((chain_fused_k<KK, true, SDG_FU_W8, false, false, CMP_GE>), g, b, 0, stream, d_a); \
        else if (sop == CMP_LT) hipLaunchKernelGGL((chain_fused_k<KK, true, SDG_FU_W8, false, false, CMP_LT>), g, b, 0, stream, d_a); \
        else hipLaunchKernelGGL((chain_fused_k<KK, true, SDG_FU_W8, false, false, CMP_LE>), g, b, 0, stream, d_a);             \
    } while (0)
        switch (a.sp.scan_t) {
            case VK_I32: FU_SOP(VK_I32); break;
            case VK_I64: FU_SOP(VK_I64); break;
            case VK_F32: FU_SOP(VK_F32); break;
            default: FU_SOP(VK_F64); break;
        }
#undef FU_SOP
        return;
    }
    switch (a.sp.scan_t) {
        case VK_I32: FU_LAUNCH(VK_I32); break;
        case VK_I64: FU_LAUNCH(VK_I64); break;
        case VK_F32: FU_LAUNCH(VK_F32); break;
        case VK_F64: FU_LAUNCH(VK_F64); break;
        case VK_BOOL: FU_LAUNCH(VK_BOOL); break;
        default: FU_LAUNCH(VK_STR); break;
    }
#undef FU_LAUNCH
}

void chain_sorted(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream) {
    if (a.n <= 0) return;
    const int64_t grid = xcd_round((a.n + FU_OWN - 1) / FU_OWN);  // rounded for the XCD remap
    const dim3 g((unsigned)grid), b(FU_THREADS);
    const bool same = a.sp.scan_col_kind == a.sp.scan_t;
    {  // the compile-time operator build (SOP), work-queue mode only
        const bool e1_is_x = a.sp.scan_mode == SCAN_E1 && a.sp.e1_col == a.sp.scan_col && a.sp.e1_col_kind == a.sp.scan_col_kind;
        const uint8_t op = a.sp.scan_op;
        const bool ord = op == CMP_GT || op == CMP_GE || op == CMP_LT || op == CMP_LE;
        static const bool no_sop = getenv("SDG_SV_NO_SOP") != nullptr;  // A/B: the run-time operator build
        if (!no_sop && (a.fu_skip & 1024) && same && e1_is_x && ord &&
            (a.sp.scan_t == VK_F64 || a.sp.scan_t == VK_I64 || a.sp.scan_t == VK_I32 || a.sp.scan_t == VK_F32)) {
            const uint8_t sop = a.sp.scan_e2_left ? op : op == CMP_GT ? CMP_LT : op == CMP_GE ? CMP_LE : op == CMP_LT ? CMP_GT : CMP_GE;
#define SV_SOP(KK)                                                                                        \
    do {                                                                                                  \
        if (sop == CMP_GT) hipLaunchKernelGGL((chain_sorted_k<KK, true, CMP_GT>), g, b, 0, stream, d_a);      \
        else if (sop == CMP_GE) hipLaunchKernelGGL((chain_sorted_k<KK, true, CMP_GE>), g, b, 0, stream, d_a); \
        else if (sop == CMP_LT) hipLaunchKernelGGL((chain_sorted_k<KK, true, CMP_LT>), g, b, 0, stream, d_a); \
        else hipLaunchKernelGGL((chain_sorted_k<KK, true, CMP_LE>), g, b, 0, stream, d_a);                    \
    } while (0)
            switch (a.sp.scan_t) {
                case VK_I32: SV_SOP(VK_I32); break;
                case VK_I64: SV_SOP(VK_I64); break;
                case VK_F32: SV_SOP(VK_F32); break;
                default: SV_SOP(VK_F64); break;
            }
#undef SV_SOP
            return;
        }
    }
#define SV_LAUNCH(KK)                                                                    \
    do {                                                                                 \
        if (same) hipLaunchKernelGGL((chain_sorted_k<KK, true>), g, b, 0, stream, d_a);  \
        else hipLaunchKernelGGL((chain_sorted_k<KK, false>), g, b, 0, stream, d_a);     \
    } while (0)
    switch (a.sp.scan_t) {
        case VK_I32: SV_LAUNCH(VK_I32); break;
        case VK_I64: SV_LAUNCH(VK_I64); break;
        case VK_F32: SV_LAUNCH(VK_F32); break;
        case VK_F64: SV_LAUNCH(VK_F64); break;
        case VK_BOOL: SV_LAUNCH(VK_BOOL); break;
        default: SV_LAUNCH(VK_STR); break;
    }
#undef SV_LAUNCH
}

void chain_sovf(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream) {
    if (a.n <= 0) return;
    hipLaunchKernelGGL(chain_sovf_k, dim3(2048), dim3(256), 0, stream, d_a);  // grid-stride over ovf_count
}

void chain_fovf(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream) {
    if (a.n <= 0) return;
    hipLaunchKernelGGL(chain_fovf_k, dim3(512), dim3(256), 0, stream, d_a);
}

}  // namespace sdg
