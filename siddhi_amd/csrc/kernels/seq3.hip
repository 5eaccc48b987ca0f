// gfx950 register kernel for the SEQUENCE shape `every e1=S[f1], e2=S[f2]<m:n>, e3=S[f3]` on one stream (C3).
//
// Why a key's state fits in registers (kernels.h Seq3Spec; reference paths under modules/siddhi-core/src/main/java/
// io/siddhi/core/query/input/stream/state/): before each event SequenceMultiProcessStreamReceiver resets every state
// (pending lists cleared, StreamPreStateProcessor.java:288-305) and moves newAndEvery to pending (:308-323); SEQUENCE
// addState keeps at most one state event per newAndEvery list (:214-227, CountPreStateProcessor.java:97-125). So per
// key there is one partial waiting at e2 (Q) and one at e3 (P) at most. Per event, in the receiver's reverse state
// order (PatternMultiProcessStreamReceiver.java:33-39):
//   e3: P matches -> emitted; its e3 slot stays set, so e2 drops the same object (CountPreStateProcessor.java:58-62)
//   e2: Q takes the event (addEvent before the filter, :64-66); passing, CountPostStateProcessor.java:49-58 forwards it
//       to e3 and keeps it at e2 (n != max) -- both only when n >= min -- else it is gone with the next reset
//   e1: the every-seed (one per key, StreamPostStateProcessor.java:64-83 re-arms it) starts a new partial, which e2
//       accepts only if Q did not stay there (its newAndEvery list is still empty)
// tests/seq3_model.py is this model in Python; tests/test_seq3_model.py checks it against the oracle.
//
// One lane per partition key walks the key's events of the key-sorted view (8 rows loaded per step); the rest of
// the state machine is register arithmetic. Matches (at most one per event) are ranked with a wave ballot, staged
// in LDS and written out as coalesced runs with one global reservation per S3_STAGE - 64 records (a reservation per
// wave-step would serialise ~10^6 atomics on one L2 address).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../engine/eval.h"
#include "kernels.h"
#include "wave.h"

namespace sdg {

namespace {

// Rows are loaded S3_G per step (all loads issued before the step's state machine runs), the registers rotating by
// four through one copy of the 4-row body. Measured on C3 (10^8 events, 10^6 keys; profiles/r3q_*, r3r): the kernel
// is issue-bound, not memory-bound -- FETCH_SIZE 2-3x the algorithmic bytes, ~600 instructions per row (26k VALU +
// 33k SALU per wave for ~100 rows: uniform operand dispatch, divergent state updates). 4-row steps with the kind
// dispatch inlined at every compare made a 48-63 KB kernel (6.6 ms); the F64 variant (8-byte columns, double
// compares) and an out-of-line generic compare brought it to ~25 KB (6.0 ms at 16 rows per step, less at 8).

template <int NC>
struct S3Ev {
    int64_t v[NC];
    // element-wise (a struct copy of 24+ bytes becomes a memcpy that pins the arrays to scratch)
    __device__ __forceinline__ void set(const S3Ev& o) {
#pragma unroll
        for (int i = 0; i < NC; ++i) v[i] = o.v[i];
    }
    __device__ __forceinline__ void set_if(bool c, const S3Ev& o) {  // a select, not a branch
#pragma unroll
        for (int i = 0; i < NC; ++i) v[i] = c ? o.v[i] : v[i];
    }
};

// e.v[c] for a (wave-uniform) column index, as masked ORs: a select chain over 3+ entries is turned into an
// indexed load by the optimizer, which moves every such register array to scratch
template <int NC>
__device__ __forceinline__ int64_t s3_pick(const S3Ev<NC>& e, int c) {
    int64_t r = 0;
#pragma unroll
    for (int i = 0; i < NC; ++i) r |= e.v[i] & -(int64_t)(c == i);
    return r;
}

// operand of a filter / select item in one partial's context (nm: the partial's null bits, yn: the event's);
// false = null. `src` is wave-uniform, so this is a scalar branch; the empty asm in each arm keeps the optimizer
// from merging the arms into one load through a selected pointer (which moves the four events to scratch)
template <int NC>
__device__ __forceinline__ bool s3_get(const S3Operand& o, const S3Ev<NC>& e1, const S3Ev<NC>& ef, const S3Ev<NC>& el,
                                       const S3Ev<NC>& y, uint32_t nm, uint32_t yn, int64_t* v) {
    const int c = o.col;
    int64_t x = 0;
    uint32_t nb = 1u;
    switch (o.src) {
        case S3_E1: x = s3_pick(e1, c); asm volatile("" : "+v"(x)); nb = nm >> c; break;
        case S3_E2F: x = s3_pick(ef, c); asm volatile("" : "+v"(x)); nb = nm >> (8 + c); break;
        case S3_E2L: x = s3_pick(el, c); asm volatile("" : "+v"(x)); nb = nm >> (16 + c); break;
        case S3_Y: x = s3_pick(y, c); asm volatile("" : "+v"(x)); nb = yn >> c; break;
        default: break;
    }
    *v = x;
    return !(nb & 1u);
}

// the generic comparison (any kinds, Java binary numeric promotion): one out-of-line copy -- inlined at every call
// site, its kind / operator switches made the kernel ~60 KB, and instruction fetch, not memory, bound it
__device__ __noinline__ bool s3_cmp_generic(uint32_t opt, uint32_t kinds, int64_t x, int64_t z) {
    const uint8_t op = (uint8_t)opt, t = (uint8_t)(opt >> 8), ka = (uint8_t)kinds, kb = (uint8_t)(kinds >> 8);
    x = cvt(x, ka, t);
    if (!(kinds >> 16)) z = cvt(z, kb, t);  // FP_CONST: already of kind t
    return cmp(op, t, x, z);
}

// fast_pass (eval.h) over resolved operands: null -> false, Java binary numeric promotion to f.t. F64: every
// predicate compares doubles (operands and constants already double: no conversion)
template <bool F64, int NC>
__device__ __forceinline__ bool s3_pass(const S3Pred& f, const S3Ev<NC>& e1, const S3Ev<NC>& ef, const S3Ev<NC>& el,
                                        const S3Ev<NC>& y, uint32_t nm, uint32_t yn) {
    if (f.kind == FP_TRUE) return true;
    int64_t x, z;
    if (!s3_get(f.a, e1, ef, el, y, nm, yn, &x)) return false;
    if (f.kind == FP_CONST) z = f.konst;
    else if (!s3_get(f.b, e1, ef, el, y, nm, yn, &z)) return false;
    if (F64) return cmpT<double>(f.op, bits_f64(x), bits_f64(z));
    return s3_cmp_generic((uint32_t)f.op | ((uint32_t)f.t << 8), (uint32_t)f.a.kind | ((uint32_t)f.b.kind << 8) |
                                                                     (f.kind == FP_CONST ? 1u << 16 : 0u), x, z);
}

// Per-query specialisation: a predicate's operands as compile-time codes (src * 8 + col; -1: FP_TRUE for the first
// operand / the constant for the second; -2: resolved at run time by s3_get). With fixed codes an operand is one
// register (no masked-OR pick over the columns, no per-operand source switch) -- the uniform operand dispatch was
// most of the ~600 instructions per row. F64 only.
template <int CODE, int NC>
__device__ __forceinline__ int64_t s3_fx(const S3Ev<NC>& e1, const S3Ev<NC>& ef, const S3Ev<NC>& el, const S3Ev<NC>& y) {
    constexpr int src = CODE / 8, c = CODE % 8;
    static_assert(c < NC, "operand column");
    if constexpr (src == S3_E1) return e1.v[c];
    else if constexpr (src == S3_E2F) return ef.v[c];
    else if constexpr (src == S3_E2L) return el.v[c];
    else return y.v[c];
}
template <int CODE>
__device__ __forceinline__ bool s3_fx_null(uint32_t nm, uint32_t yn) {
    constexpr int src = CODE / 8, c = CODE % 8;
    if constexpr (src == S3_E1) return (nm >> c) & 1u;
    else if constexpr (src == S3_E2F) return (nm >> (8 + c)) & 1u;
    else if constexpr (src == S3_E2L) return (nm >> (16 + c)) & 1u;
    else return (yn >> c) & 1u;
}
template <bool F64, int FA, int FB, int NC>
__device__ __forceinline__ bool s3_pass_x(const S3Pred& f, const S3Ev<NC>& e1, const S3Ev<NC>& ef, const S3Ev<NC>& el,
                                          const S3Ev<NC>& y, uint32_t nm, uint32_t yn) {
    if constexpr (FA == -2) {
        return s3_pass<F64>(f, e1, ef, el, y, nm, yn);
    } else if constexpr (FA == -1) {
        return true;
    } else {
        static_assert(F64, "fixed operands: the double-compare variant");
        if (s3_fx_null<FA>(nm, yn)) return false;
        const int64_t x = s3_fx<FA>(e1, ef, el, y);
        int64_t z;
        if constexpr (FB == -1) {
            z = f.konst;
        } else {
            if (s3_fx_null<FB>(nm, yn)) return false;
            z = s3_fx<FB>(e1, ef, el, y);
        }
        return cmpT<double>(f.op, bits_f64(x), bits_f64(z));
    }
}

template <int NC, int S3_G, bool F64, bool SEL, int FA0 = -2, int FA1 = -2, int FB1 = -2, int FA2 = -2, int FB2 = -2,
          int W = 1>
__global__ __launch_bounds__(64, W) void seq3_k(const Seq3Args* __restrict__ pa) {
    const Seq3Args& a = *pa;
    const Seq3Spec& sp = a.sp;
    extern __shared__ __align__(16) uint8_t s3_lds[];
    int64_t* l_ts = (int64_t*)s3_lds;
    int64_t* l_seq = l_ts + S3_STAGE;
    int64_t* l_vals = l_seq + S3_STAGE;  // [n_out][S3_STAGE]
    uint32_t* l_key = (uint32_t*)(l_vals + (int64_t)sp.n_out * S3_STAGE);
    uint32_t* l_nul = l_key + S3_STAGE;
    const int lane = threadIdx.x;
    const int64_t k = (int64_t)blockIdx.x * 64 + lane;
    int64_t b = 0, e = 0;
    if (k < a.K) {
        if (a.seg_start) {
            b = a.seg_start[k];
            e = a.seg_end[k];
        } else {
            e = a.n;
        }
    }
    const bool has = b < e;
    if (!__any(has)) return;  // one wave per block: a uniform exit
    const int64_t kc = a.kcap;
    uint32_t hdr = 0, pn = 0, qn = 0;
    S3Ev<NC> P1{}, PF{}, PL{}, Q1{}, QF{}, QL{};
    int64_t pts = 0, qts = 0;  // e1 timestamps (within)
    const bool wth = sp.has_within != 0;
    const int64_t within = sp.within_ms;
    if (has) {
        hdr = a.st_hdr[k];
        if (hdr & 2u) {
            qn = a.st_qn[k];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                Q1.v[c] = a.st_vals[(int64_t)(3 * NC + c) * kc + k];
                QF.v[c] = a.st_vals[(int64_t)(4 * NC + c) * kc + k];
                QL.v[c] = a.st_vals[(int64_t)(5 * NC + c) * kc + k];
            }
        }
        if (wth) {
            if (hdr & 1u) pts = a.st_ts[k];
            if (hdr & 2u) qts = a.st_ts[kc + k];
        }
        if (hdr & 4u) {  // P is Q: stored once
            P1.set(Q1); PF.set(QF); PL.set(QL);
            pn = qn;
        } else if (hdr & 1u) {
            pn = a.st_pn[k];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                P1.v[c] = a.st_vals[(int64_t)(0 * NC + c) * kc + k];
                PF.v[c] = a.st_vals[(int64_t)(1 * NC + c) * kc + k];
                PL.v[c] = a.st_vals[(int64_t)(2 * NC + c) * kc + k];
            }
        }
    }
    const uint32_t mn = (uint32_t)sp.min_count, mx = (uint32_t)sp.max_count;
    const uint64_t lt = lanemask_lt();
    int staged = 0;
    auto flush = [&]() __attribute__((always_inline)) {
        __syncthreads();  // the staged records of every lane (one-wave block)
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(a.out_count, (unsigned long long)staged);
        base = __shfl(base, 0);
        for (int i = lane; i < staged; i += 64) {
            const int64_t o = (int64_t)base + i;
            if (o >= a.out_cap) {
                atomicOr(&a.flags[0], 1);
                continue;
            }
            a.out_ts[o] = l_ts[i];
            a.out_emit_seq[o] = l_seq[i];
            a.out_sub[o] = 0;
            a.out_key[o] = l_key[i];
            a.out_nulls[o] = l_nul[i];
            for (int j = 0; j < sp.n_out; ++j) a.out_vals[(int64_t)j * a.out_cap + o] = l_vals[j * S3_STAGE + i];
        }
        __syncthreads();
        staged = 0;
    };
    // one event through e3, e2, e1 (the state machine; y = the event, r its sorted row)
    // The state updates are selects, not branches: with divergent lanes every branch of a per-row if/else ran anyway,
    // and the exec-mask bookkeeping around them cost more than the selects
    auto row_step = [&](const S3Ev<NC>& y, uint32_t ynn, int64_t yt, int64_t r) __attribute__((always_inline)) {
        const bool act = r < e;
        bool hasP = act && (hdr & 1u), hasQ = act && (hdr & 2u);
        const bool same = (hdr & 4u) != 0;
        if (wth) {  // stabilizeStates: expireEvents drops a partial whose e1 is more than T away (isExpired)
            int64_t d = pts - yt;
            hasP = hasP && (d < 0 ? -d : d) <= within;
            d = qts - yt;
            hasQ = hasQ && (d < 0 ? -d : d) <= within;
        }
        // e3 (first in the receiver's order)
        const bool em = hasP && s3_pass_x<F64, FA2, FB2>(sp.f[2], P1, PF, PL, y, pn, ynn);
        const uint64_t m = __ballot(em);
        if (m) {
            if (em) {
                const int at = staged + __popcll(m & lt);
                const int64_t o = a.orig ? (int64_t)a.orig[r] : a.pos_off + r;
                l_ts[at] = a.ts ? yt : a.ts_view[o];
                l_seq[at] = a.seq_base + o;
                l_key[at] = (uint32_t)k;
                uint32_t nm = 0;
                for (int j = 0; j < sp.n_out; ++j) {
                    int64_t v;
                    const bool ok = s3_get(sp.out[j], P1, PF, PL, y, pn, ynn, &v);
                    l_vals[j * S3_STAGE + at] = ok ? v : 0;
                    if (!ok) nm |= 1u << j;
                }
                l_nul[at] = nm;
            }
            staged += __popcll(m);
        }
        // e2: Q takes the event unless e3 just consumed the same object; e2[0] is this event when Q has none yet
        const uint32_t cnt = hdr >> 8;
        const uint32_t n1 = cnt < 0xFFFFFFu ? cnt + 1 : cnt;
        const bool qfirst = cnt == 0;
        QF.set_if(qfirst, y);
        const uint32_t qn2 = qfirst ? ((qn & ~0xFF00u) | (ynn << 8)) : qn;
        const bool adv = hasQ && !(em && same) && n1 >= mn && s3_pass_x<F64, FA1, FB1>(sp.f[1], Q1, QF, y, y, qn2, ynn);
        const bool keep = adv && n1 != mx;  // kept at e2 too: one object
        const uint32_t pn2 = (qn2 & 0xFFFFu) | (ynn << 16);
        P1.set_if(adv, Q1);
        PF.set_if(adv, QF);
        PL.set_if(adv, y);
        pn = adv ? pn2 : pn;
        pts = adv ? qts : pts;
        QL.set_if(keep, y);
        // e1: the every-seed starts a partial when e2's list is still empty
        const bool fresh = act && !keep && s3_pass_x<F64, FA0, -1>(sp.f[0], y, y, y, y, 0u, ynn);
        Q1.set_if(fresh, y);
        qts = fresh ? yt : qts;
        qn = fresh ? ynn : keep ? pn2 : qn;
        const uint32_t ncnt = fresh ? 0u : keep ? n1 : cnt;
        const uint32_t nh = (adv ? 1u : 0u) | (keep || fresh ? 2u : 0u) | (keep ? 4u : 0u);
        hdr = act ? (nh | (ncnt << 8)) : hdr;
        if (staged > S3_STAGE - 64) flush();
    };
    // the branchy form of the same step (A/B: SDG_S3_BRANCH=1)
    auto row_step_br = [&](const S3Ev<NC>& y, uint32_t ynn, int64_t yt, int64_t r) __attribute__((always_inline)) {
        const bool act = r < e;
        if (wth && act) {  // stabilizeStates: expireEvents drops a partial whose e1 is more than T away (isExpired)
            int64_t d = pts - yt;
            if ((hdr & 1u) && (d < 0 ? -d : d) > within) hdr &= ~5u;
            d = qts - yt;
            if ((hdr & 2u) && (d < 0 ? -d : d) > within) hdr &= ~6u;
        }
        // e3 (first in the receiver's order)
        const bool em = act && (hdr & 1u) && s3_pass<F64>(sp.f[2], P1, PF, PL, y, pn, ynn);
        const uint64_t m = __ballot(em);
        if (m) {
            if (em) {
                const int at = staged + __popcll(m & lt);
                const int64_t o = a.orig ? (int64_t)a.orig[r] : a.pos_off + r;
                l_ts[at] = a.ts ? yt : a.ts_view[o];
                l_seq[at] = a.seq_base + o;
                l_key[at] = (uint32_t)k;
                uint32_t nm = 0;
                for (int j = 0; j < sp.n_out; ++j) {
                    int64_t v;
                    const bool ok = s3_get(sp.out[j], P1, PF, PL, y, pn, ynn, &v);
                    l_vals[j * S3_STAGE + at] = ok ? v : 0;
                    if (!ok) nm |= 1u << j;
                }
                l_nul[at] = nm;
            }
            staged += __popcll(m);
        }
        if (act) {
            // e2: Q takes the event unless e3 just consumed the same object
            uint32_t cnt = hdr >> 8, nh = 0;
            if ((hdr & 2u) && !(em && (hdr & 4u))) {
                const uint32_t n1 = cnt < 0xFFFFFFu ? cnt + 1 : cnt;
                if (cnt == 0) {  // e2[0] is this event
                    QF.set(y);
                    qn = (qn & ~0xFF00u) | (ynn << 8);
                }
                if (s3_pass<F64>(sp.f[1], Q1, QF, y, y, qn, ynn) && n1 >= mn) {
                    pts = qts;
                    P1.set(Q1);
                    PF.set(QF);
                    PL.set(y);
                    pn = (qn & 0xFFFFu) | (ynn << 16);
                    nh = 1u;
                    if (n1 != mx) {  // kept at e2 too: one object
                        QL.set(y);
                        qn = pn;
                        cnt = n1;
                        nh |= 2u | 4u;
                    }
                }
            }
            // e1: the every-seed starts a partial when e2's list is still empty
            if (!(nh & 2u) && s3_pass<F64>(sp.f[0], y, y, y, y, 0u, ynn)) {
                Q1.set(y);
                qts = yt;
                qn = ynn;
                cnt = 0;
                nh |= 2u;
            }
            hdr = nh | (cnt << 8);
        }
        if (staged > S3_STAGE - 64) flush();
    };
    for (int64_t i = 0; __any(b + i < e); i += S3_G) {
        S3Ev<NC> yv[S3_G];
        uint32_t yn[S3_G];
        int64_t yts[S3_G];
#pragma unroll
        for (int g = 0; g < S3_G; ++g) {  // the step's loads first: they overlap
            const int64_t r = b + i + g;
            yn[g] = 0;
            yts[g] = 0;
#pragma unroll
            for (int c = 0; c < NC; ++c) yv[g].v[c] = 0;
            if (r < e) {
                if (a.ts) yts[g] = a.ts[r];
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    yv[g].v[c] = F64 ? ((const int64_t*)a.cols[c])[r] : load_col(a.cols[c], sp.col_kind[c], r);
                    if (a.nulls[c] && a.nulls[c][r]) yn[g] |= 1u << c;
                }
            }
        }
        // four rows per round through one copy of the state machine, then the registers rotate by four (static
        // indices throughout: a dynamically indexed register array would live in scratch)
#pragma unroll 1
        for (int q4 = 0; q4 < S3_G; q4 += 4) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if (SEL) row_step(yv[g], yn[g], yts[g], b + i + q4 + g);
                else row_step_br(yv[g], yn[g], yts[g], b + i + q4 + g);
            }
            if (q4 + 4 < S3_G) {
#pragma unroll
                for (int g = 0; g + 4 < S3_G; ++g) {
                    yv[g].set(yv[g + 4]);
                    yn[g] = yn[g + 4];
                    yts[g] = yts[g + 4];
                }
            }
        }
    }
    if (staged) flush();
    if (has) {
        a.st_hdr[k] = hdr;
        if (wth) {
            if (hdr & 1u) a.st_ts[k] = pts;
            if (hdr & 2u) a.st_ts[kc + k] = qts;
        }
        if (hdr & 2u) {
            a.st_qn[k] = qn;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                a.st_vals[(int64_t)(3 * NC + c) * kc + k] = Q1.v[c];
                a.st_vals[(int64_t)(4 * NC + c) * kc + k] = QF.v[c];
                a.st_vals[(int64_t)(5 * NC + c) * kc + k] = QL.v[c];
            }
        }
        if ((hdr & 1u) && !(hdr & 4u)) {
            a.st_pn[k] = pn;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                a.st_vals[(int64_t)(0 * NC + c) * kc + k] = P1.v[c];
                a.st_vals[(int64_t)(1 * NC + c) * kc + k] = PF.v[c];
                a.st_vals[(int64_t)(2 * NC + c) * kc + k] = PL.v[c];
            }
        }
    }
}

}  // namespace

void seq3_run(const Seq3Args& a, const Seq3Args* d_a, hipStream_t stream) {
    if (a.K <= 0 || a.n <= 0) return;
    const unsigned grid = (unsigned)((a.K + 63) / 64);
    const size_t lds = (size_t)S3_STAGE * (16 + 8 * (size_t)a.sp.n_out + 8);
    // rows loaded per step: 8 (C3 12.9 ms per 10^8 events vs 13.6 with 16: fewer VGPRs, more waves; r3q)
    static const char* gs = getenv("SDG_S3_G");  // A/B
    const bool g16 = gs && atoi(gs) == 16;
    // F64: 8-byte columns and double comparisons only (C3): no kind dispatch in the row loop
    bool f64 = !getenv("SDG_S3_GENERIC");
    static const bool sel = !getenv("SDG_S3_BRANCH");  // A/B: the branchy state update (F64 variant only)
    for (int c = 0; c < a.sp.nc; ++c) f64 &= a.sp.col_kind[c] == VK_I64 || a.sp.col_kind[c] == VK_F64;
    for (int p = 0; p < 3; ++p) {
        const S3Pred& f = a.sp.f[p];
        if (f.kind == FP_TRUE) continue;
        f64 &= f.t == VK_F64 && f.a.kind == VK_F64 && (f.kind == FP_CONST || f.b.kind == VK_F64);
    }
    // the predicates' operand codes (s3_pass_x): a kernel compiled for them when the query is the C3 form
    // (e1 = S[x > c], e2 = S[x > e1.x], e3 = S[x < e2[last].x] over a double column x, two columns)
    auto code = [](const S3Operand& o) { return o.src < 0 ? -9 : (int)o.src * 8 + (int)o.col; };
    const S3Pred &f0 = a.sp.f[0], &f1 = a.sp.f[1], &f2 = a.sp.f[2];
    static const bool no_fix = getenv("SDG_S3_NOFIX") != nullptr;  // A/B: the run-time operand dispatch
    int fx = -1;  // column of x in a C3-form query
    if (f64 && sel && !no_fix && a.sp.nc == 2 && !g16 && f0.kind == FP_CONST && f1.kind == FP_SLOT && f2.kind == FP_SLOT) {
        const int x = f0.a.col;
        if (code(f0.a) == S3_Y * 8 + x && code(f1.a) == S3_Y * 8 + x && code(f1.b) == S3_E1 * 8 + x &&
            code(f2.a) == S3_Y * 8 + x && code(f2.b) == S3_E2L * 8 + x && x < 2)
            fx = x;
    }
    // waves per SIMD the fixed kernels are compiled for: 3 (<= 168 VGPRs, no spills) measured 11.03 vs 11.49 ms per
    // C3 step at 2 (~190 VGPRs; r4j, same box); SDG_S3_W=2 for A/B
    static const char* ws = getenv("SDG_S3_W");
    const bool w3 = !(ws && atoi(ws) == 2);
#define S3_FIX(X)                                                                                                  \
    do {                                                                                                           \
        if (w3) hipLaunchKernelGGL((seq3_k<2, 8, true, true, S3_Y * 8 + X, S3_Y * 8 + X, S3_E1 * 8 + X, S3_Y * 8 + X,  \
                                           S3_E2L * 8 + X, 3>), dim3(grid), dim3(64), lds, stream, d_a);            \
        else hipLaunchKernelGGL((seq3_k<2, 8, true, true, S3_Y * 8 + X, S3_Y * 8 + X, S3_E1 * 8 + X, S3_Y * 8 + X,     \
                                        S3_E2L * 8 + X, 1>), dim3(grid), dim3(64), lds, stream, d_a);               \
    } while (0)
    if (fx == 0) {
        S3_FIX(0);
        return;
    }
    if (fx == 1) {
        S3_FIX(1);
        return;
    }
#undef S3_FIX
#define S3_LAUNCH(NC_, G_)                                                                              \
    do {                                                                                                \
        if (f64 && sel) hipLaunchKernelGGL((seq3_k<NC_, G_, true, true>), dim3(grid), dim3(64), lds, stream, d_a);  \
        else if (f64) hipLaunchKernelGGL((seq3_k<NC_, G_, true, false>), dim3(grid), dim3(64), lds, stream, d_a);   \
        else hipLaunchKernelGGL((seq3_k<NC_, G_, false, true>), dim3(grid), dim3(64), lds, stream, d_a);           \
    } while (0)
    switch (a.sp.nc) {
        case 1:
            if (g16) S3_LAUNCH(1, 16);
            else S3_LAUNCH(1, 8);
            break;
        case 2:
            if (g16) S3_LAUNCH(2, 16);
            else S3_LAUNCH(2, 8);
            break;
        case 3: S3_LAUNCH(3, 8); break;
        default: S3_LAUNCH(4, 8); break;
    }
#undef S3_LAUNCH
}

}  // namespace sdg
