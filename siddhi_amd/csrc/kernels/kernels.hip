// gfx950 kernels of the pattern/sequence path: key grouping and the chain matcher.
//
// Wave64 throughout: ballots are 64-bit, lane masks use __lanemask_lt(), compaction is ballot + mbcnt with one
// atomic per wave. Everything is integer/byte work bound by HBM, so no MFMA.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../engine/eval.h"
#include "kernels.h"

namespace sdg {

namespace {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
    int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// wave-level compaction: returns this lane's slot (valid only where `take`), one atomic per wave
__device__ __forceinline__ int64_t wave_reserve(bool take, unsigned long long* counter) {
    uint64_t m = __ballot(take);
    if (m == 0) return -1;
    int leader = __ffsll((unsigned long long)m) - 1;
    unsigned long long base = 0;
    if (lane_id() == leader) base = atomicAdd(counter, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    return (int64_t)base + __popcll(m & lanemask_lt());
}

// ---------------------------------------------------------------------------------------------------------
// key grouping: LSD radix passes

__device__ __forceinline__ uint32_t digit_of(uint32_t k, int shift, uint32_t mask) { return (k >> shift) & mask; }

// per-tile digit histogram: counts[tile * nb + d]
__global__ __launch_bounds__(RX_THREADS) void rx_hist(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                      uint32_t mask, int nb, uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[1 << RX_MAXBITS];
    for (int d = threadIdx.x; d < nb; d += RX_THREADS) h[d] = 0;
    __syncthreads();
    int64_t base = (int64_t)blockIdx.x * RX_TILE;
#pragma unroll 4
    for (int r = 0; r < RX_TILE / RX_THREADS; ++r) {
        int64_t i = base + r * RX_THREADS + threadIdx.x;
        if (i < n) atomicAdd(&h[digit_of(keys[i], shift, mask)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nb; d += RX_THREADS) counts[(int64_t)blockIdx.x * nb + d] = h[d];
}

// group sums over KG_GROUP tiles: thread (g, d)
__global__ __launch_bounds__(256) void rx_p1(const uint32_t* __restrict__ counts, int ntiles, int nb,
                                             uint32_t* __restrict__ gsum) {
    int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int ng = (ntiles + KG_GROUP - 1) / KG_GROUP;
    if (idx >= (int64_t)ng * nb) return;
    int g = (int)(idx / nb), d = (int)(idx % nb);
    int b0 = g * KG_GROUP, b1 = min(ntiles, b0 + KG_GROUP);
    uint32_t s = 0;
    for (int b = b0; b < b1; ++b) s += counts[(int64_t)b * nb + d];
    gsum[idx] = s;
}

// one block: per digit, exclusive scan over groups (in place) + digit totals; then exclusive scan over digits
__global__ __launch_bounds__(256) void rx_p2(uint32_t* __restrict__ gsum, int ng, int nb, uint32_t* __restrict__ tot) {
    __shared__ uint32_t part[256];
    int d = threadIdx.x;
    uint32_t run = 0;
    if (d < nb) {
        for (int g = 0; g < ng; ++g) {
            uint32_t c = gsum[(int64_t)g * nb + d];
            gsum[(int64_t)g * nb + d] = run;
            run += c;
        }
    }
    part[d] = d < nb ? run : 0;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        uint32_t x = d >= off ? part[d - off] : 0;
        __syncthreads();
        part[d] += x;
        __syncthreads();
    }
    if (d < nb) tot[d] = part[d] - run;  // exclusive digit base
}

// per (group, digit): rewrite the group's tile counts as absolute start offsets
__global__ __launch_bounds__(256) void rx_p3(uint32_t* __restrict__ counts, const uint32_t* __restrict__ gsum,
                                             const uint32_t* __restrict__ tot, int ntiles, int nb) {
    int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int ng = (ntiles + KG_GROUP - 1) / KG_GROUP;
    if (idx >= (int64_t)ng * nb) return;
    int g = (int)(idx / nb), d = (int)(idx % nb);
    uint32_t run = tot[d] + gsum[idx];
    int b0 = g * KG_GROUP, b1 = min(ntiles, b0 + KG_GROUP);
    for (int b = b0; b < b1; ++b) {
        uint32_t c = counts[(int64_t)b * nb + d];
        counts[(int64_t)b * nb + d] = run;
        run += c;
    }
}

struct RxPass {
    const uint32_t* keys_in;
    uint32_t* keys_out;
    const uint32_t* orig_in;  // nullptr: identity (first pass)
    uint32_t* orig_out;
    int ncols;
    const void* src[MAX_COLS + 2];
    void* dst[MAX_COLS + 2];
    uint8_t width[MAX_COLS + 2];
    const uint32_t* offsets;  // counts rewritten by rx_p3: [tile * nb + d]
    int64_t n;
    int shift;
    uint32_t mask;
    int nb;
    int bits;
};

// stable tile scatter
__global__ __launch_bounds__(RX_THREADS) void rx_scatter(RxPass a) {
    constexpr int R = RX_TILE / RX_THREADS;  // rounds (16): element r*256 + t of the tile
    __shared__ uint32_t cnt[1 << RX_MAXBITS];
    __shared__ uint32_t wavecnt[RX_THREADS / 64][1 << RX_MAXBITS];
    __shared__ uint32_t tstart[1 << RX_MAXBITS];
    __shared__ uint32_t gbase[1 << RX_MAXBITS];
    __shared__ uint32_t dest[RX_TILE];
    __shared__ uint64_t stage[RX_TILE];
    const int t = threadIdx.x, w = t >> 6;
    const int64_t base = (int64_t)blockIdx.x * RX_TILE;
    const int64_t tile_n = min((int64_t)RX_TILE, a.n - base);
    for (int d = t; d < a.nb; d += RX_THREADS) {
        cnt[d] = 0;
        gbase[d] = a.offsets[(int64_t)blockIdx.x * a.nb + d];
        for (int v = 0; v < RX_THREADS / 64; ++v) wavecnt[v][d] = 0;
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt();
    uint32_t rank[R];
    uint16_t dig[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int64_t i = base + r * RX_THREADS + t;
        bool valid = i < a.n;
        uint32_t d = valid ? digit_of(a.keys_in[i], a.shift, a.mask) : 0u;
        uint64_t peers = __ballot(valid);
        for (int bit = 0; bit < a.bits; ++bit) {
            bool on = (d >> bit) & 1u;
            uint64_t b = __ballot(on);
            peers &= on ? b : ~b;
        }
        int leader = peers ? __ffsll((unsigned long long)peers) - 1 : 0;
        if (valid && lane_id() == leader) wavecnt[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        uint32_t pre = 0;
        if (valid) {
            pre = cnt[d];
            for (int v = 0; v < w; ++v) pre += wavecnt[v][d];
        }
        rank[r] = pre + (uint32_t)__popcll(peers & lt);
        dig[r] = (uint16_t)d;
        __syncthreads();
        for (int dd = t; dd < a.nb; dd += RX_THREADS) {
            uint32_t s = 0;
            for (int v = 0; v < RX_THREADS / 64; ++v) {
                s += wavecnt[v][dd];
                wavecnt[v][dd] = 0;
            }
            cnt[dd] += s;
        }
        __syncthreads();
    }
    // tile-local start of each digit run (exclusive scan of cnt over nb <= 256 digits)
    if (t < 256) tstart[t] = t < a.nb ? cnt[t] : 0;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        uint32_t x = (t < 256 && t >= off) ? tstart[t - off] : 0;
        __syncthreads();
        if (t < 256) tstart[t] += x;
        __syncthreads();
    }
    if (t < 256) tstart[t] -= (t < a.nb ? cnt[t] : 0);
    __syncthreads();
    uint32_t sp[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int64_t i = base + r * RX_THREADS + t;
        sp[r] = tstart[dig[r]] + rank[r];
        if (i < a.n) dest[sp[r]] = gbase[dig[r]] + rank[r];
    }
    __syncthreads();
    // keys, original rows, then every payload column: stage in digit order, write runs out coalesced
    for (int c = -2; c < a.ncols; ++c) {
        int wd = c < 0 ? 4 : a.width[c];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            int64_t i = base + r * RX_THREADS + t;
            if (i < a.n) {
                uint64_t v;
                if (c == -2) v = a.keys_in[i];
                else if (c == -1) v = a.orig_in ? a.orig_in[i] : (uint32_t)i;
                else if (wd == 8) v = ((const uint64_t*)a.src[c])[i];
                else if (wd == 4) v = ((const uint32_t*)a.src[c])[i];
                else v = ((const uint8_t*)a.src[c])[i];
                stage[sp[r]] = v;
            }
        }
        __syncthreads();
        for (int j = t; j < tile_n; j += RX_THREADS) {
            uint32_t o = dest[j];
            uint64_t v = stage[j];
            if (c == -2) a.keys_out[o] = (uint32_t)v;
            else if (c == -1) a.orig_out[o] = (uint32_t)v;
            else if (wd == 8) ((uint64_t*)a.dst[c])[o] = v;
            else if (wd == 4) ((uint32_t*)a.dst[c])[o] = (uint32_t)v;
            else ((uint8_t*)a.dst[c])[o] = (uint8_t)v;
        }
        __syncthreads();
    }
}

// key segments of the sorted keys
__global__ __launch_bounds__(256) void rx_segments(const uint32_t* __restrict__ keys, int64_t n,
                                                   uint32_t* __restrict__ seg_start, uint32_t* __restrict__ seg_end) {
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint32_t k = keys[p];
    if (p == 0 || keys[p - 1] != k) seg_start[k] = (uint32_t)p;
    if (p == n - 1 || keys[p + 1] != k) seg_end[k] = (uint32_t)(p + 1);
}

// ---------------------------------------------------------------------------------------------------------
// chain matcher

struct ChainAcc {
    const ChainArgs* A;
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
        *v = load_col(A->cols[col], kind, row);
        *null = A->nulls[col] ? A->nulls[col][row] != 0 : false;
    }
    __device__ bool slot_empty(int slot, int chain) {
        if (!(chain == 0 || chain == -1)) return true;
        if (slot == 0) return !(c0 >= 0 || r0 >= 0);
        if (slot == 1) return r1 < 0;
        return true;
    }
};

__device__ __forceinline__ int qstream_of(const ChainArgs& a, int64_t row) {
    return a.qstream ? (int)a.qstream[row] : 0;
}

// scan the key's events after `from` (exclusive) for the e2 of a partial whose e1 is at ts0.
// returns: >= 0 the matching row; -1 expired (dead); -2 reached the end of the segment (carry)
__device__ __forceinline__ int64_t chain_scan(const ChainArgs& a, ChainAcc& acc, int64_t from, int64_t end, int64_t ts0,
                                              int64_t* stk, int stride) {
    const Plan* P = a.plan;
    const int32_t has_within = P->has_within;
    const int64_t within = P->within_ms;
    const Prog c1 = P->st[1].filter;
    const FastPred f1 = P->fast[1];
    for (int64_t q = from; q < end; ++q) {
        int64_t tq = a.ts[q];
        // StreamPreStateProcessor.isExpired: |start.ts - now| > within, checked before the event is processed
        if (has_within) {
            int64_t d = ts0 - tq;
            if (d < 0) d = -d;
            if (d > within) return -1;
        }
        if (qstream_of(a, q) == a.s1) {
            acc.r1 = q;
            bool ok = f1.kind == FP_TRUE ? true
                      : f1.kind == FP_NONE ? pass(a.code, c1, a.consts, acc, stk, stride)
                                           : fast_pass(f1, acc);
            if (ok) return q;
            acc.r1 = -1;
        }
    }
    return -2;
}

// select expressions: a plain attribute (`e1.id`) is loaded directly, anything else runs the bytecode
__device__ __forceinline__ void eval_out(const ChainArgs& a, const Prog pr, ChainAcc& acc, int64_t* stk, int stride,
                                         int64_t* v, bool* nl) {
    if (pr.len == 1 && a.code[pr.start].op == OP_LOAD) {
        const Instr in = a.code[pr.start];
        acc.load(in.a, in.b, in.c, in.k, v, nl);
    } else {
        run(a.code, pr, a.consts, acc, stk, stride, v, nl);
    }
}

__device__ __forceinline__ void emit_match(const ChainArgs& a, ChainAcc& acc, int64_t slot, int64_t q, uint32_t key,
                                           int64_t first_seq, int64_t* stk, int stride) {
    const Plan* P = a.plan;
    a.out_ts[slot] = a.ts[q];
    a.out_key[slot] = key;
    a.out_emit_seq[slot] = a.seq_base + (a.orig ? (int64_t)a.orig[q] : q);
    a.out_first_seq[slot] = first_seq;
    uint32_t nm = 0;
    acc.r1 = P->n_states > 1 ? q : -1;
    for (int j = 0; j < P->n_out; ++j) {
        int64_t v;
        bool nl;
        eval_out(a, P->out_prog[j], acc, stk, stride, &v, &nl);
        a.out_vals[(int64_t)j * a.out_cap + slot] = v;
        if (nl) nm |= 1u << j;
    }
    a.out_nulls[slot] = nm;
}

// block-wide exclusive scan of two per-thread counts; one atomic per block and counter reserves the block's
// output range (per-wave reservations on one global counter serialise in L2 at ~10^8/s)
__device__ __forceinline__ void block_reserve2(uint32_t c0, uint32_t c1, unsigned long long* ctr0,
                                               unsigned long long* ctr1, int64_t* off0, int64_t* off1) {
    __shared__ uint32_t wtot[2][CM_THREADS / 64];
    __shared__ unsigned long long bbase[2];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t x0 = c0, x1 = c1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y0 = __shfl_up(x0, d), y1 = __shfl_up(x1, d);
        if (lane >= d) { x0 += y0; x1 += y1; }
    }
    if (lane == 63) { wtot[0][w] = x0; wtot[1][w] = x1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t0 = 0, t1 = 0;
        for (int v = 0; v < CM_THREADS / 64; ++v) {
            uint32_t u0 = wtot[0][v], u1 = wtot[1][v];
            wtot[0][v] = t0; wtot[1][v] = t1;
            t0 += u0; t1 += u1;
        }
        bbase[0] = t0 ? atomicAdd(ctr0, (unsigned long long)t0) : 0ull;
        bbase[1] = t1 ? atomicAdd(ctr1, (unsigned long long)t1) : 0ull;
    }
    __syncthreads();
    *off0 = (int64_t)bbase[0] + wtot[0][w] + (x0 - c0);
    *off1 = (int64_t)bbase[1] + wtot[1][w] + (x1 - c1);
}

constexpr uint32_t CM_NONE = 0xFFFFFFFFu, CM_CARRY = 0xFFFFFFFEu;

// one block per tile of CM_THREADS * CM_EPT sorted events; lane t takes events base + r * CM_THREADS + t
__global__ __launch_bounds__(CM_THREADS) void chain_match_k(ChainArgs a) {
    __shared__ int64_t stack_mem[STACK * CM_THREADS];
    int64_t* stk = stack_mem + threadIdx.x;
    const int stride = CM_THREADS;
    const Plan* P = a.plan;
    const int64_t base = (int64_t)blockIdx.x * (CM_THREADS * CM_EPT);
    const FastPred f0 = P->fast[0];
    uint32_t res[CM_EPT];
    uint32_t nmatch = 0, ncarry = 0;
#pragma unroll
    for (int r = 0; r < CM_EPT; ++r) {
        const int64_t p = base + r * CM_THREADS + threadIdx.x;
        res[r] = CM_NONE;
        if (p >= a.n) continue;
        ChainAcc acc{&a, p, -1, -1};
        const uint32_t key = a.key ? a.key[p] : 0u;
        if (p > 0 && a.ts[p] < a.ts[p - 1] && (!a.key || a.key[p - 1] == key)) atomicOr(&a.flags[1], 1);
        bool c0 = false;
        if (qstream_of(a, p) == a.s0)
            c0 = f0.kind == FP_TRUE ? true
                 : f0.kind == FP_NONE ? pass(a.code, P->st[0].filter, a.consts, acc, stk, stride) : fast_pass(f0, acc);
        if (!c0) continue;
        if (P->n_states == 1) {
            res[r] = (uint32_t)p;
        } else {
            const int64_t end = a.key ? (int64_t)a.seg_end[key] : a.n;
            const int64_t q = chain_scan(a, acc, p + 1, end, a.ts[p], stk, stride);
            res[r] = q >= 0 ? (uint32_t)q : q == -2 ? CM_CARRY : CM_NONE;
        }
        nmatch += res[r] < CM_CARRY;
        ncarry += res[r] == CM_CARRY;
    }
    int64_t slot, cs;
    block_reserve2(nmatch, ncarry, a.out_count, a.carry_count, &slot, &cs);
#pragma unroll
    for (int r = 0; r < CM_EPT; ++r) {
        if (res[r] == CM_NONE) continue;
        const int64_t p = base + r * CM_THREADS + threadIdx.x;
        const uint32_t key = a.key ? a.key[p] : 0u;
        const int64_t seq = a.seq_base + (a.orig ? (int64_t)a.orig[p] : p);
        if (res[r] != CM_CARRY) {
            if (slot >= a.out_cap) {
                atomicOr(&a.flags[0], 1);
            } else {
                ChainAcc acc{&a, p, -1, -1};
                emit_match(a, acc, slot, (int64_t)res[r], key, seq, stk, stride);
            }
            ++slot;
        } else {
            if (cs >= a.carry_cap) {
                atomicOr(&a.flags[0], 1);
            } else {
                a.carry_key[cs] = key;
                a.carry_ts[cs] = a.ts[p];
                a.carry_seq[cs] = seq;
                uint32_t nm = 0;
                for (int c = 0; c < P->n_cols; ++c) {
                    a.carry_vals[(int64_t)c * a.carry_cap + cs] = load_col(a.cols[c], P->col_kind[c], p);
                    if (a.nulls[c] && a.nulls[c][p]) nm |= 1u << c;
                }
                a.carry_nulls[cs] = nm;
            }
            ++cs;
        }
    }
}

__global__ __launch_bounds__(256) void chain_carry_k(ChainArgs a) {
    __shared__ int64_t stack_mem[STACK * 256];
    int64_t* stk = stack_mem + threadIdx.x;
    const int stride = 256;
    const Plan* P = a.plan;
    int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool active = c < a.cin_n;
    bool has = false, carry = false;
    int64_t qhit = -1;
    ChainAcc acc{&a, -1, c, -1};
    uint32_t key = 0;
    if (active) {
        key = a.cin_key[c];
        int64_t b = 0, e = a.n;
        if (a.key) {
            b = key < (uint32_t)a.K ? (int64_t)a.seg_start[key] : 0;
            e = key < (uint32_t)a.K ? (int64_t)a.seg_end[key] : 0;
        }
        int64_t r = chain_scan(a, acc, b, e, a.cin_ts[c], stk, stride);
        if (r >= 0) { has = true; qhit = r; }
        else if (r == -2) carry = true;
    }
    int64_t slot = wave_reserve(has, a.out_count);
    if (has) {
        if (slot >= a.out_cap) atomicOr(&a.flags[0], 1);
        else emit_match(a, acc, slot, qhit, key, a.cin_seq[c], stk, stride);
    }
    int64_t cs = wave_reserve(carry, a.carry_count);
    if (carry) {
        if (cs >= a.carry_cap) {
            atomicOr(&a.flags[0], 1);
        } else {
            a.carry_key[cs] = key;
            a.carry_ts[cs] = a.cin_ts[c];
            a.carry_seq[cs] = a.cin_seq[c];
            for (int k = 0; k < P->n_cols; ++k)
                a.carry_vals[(int64_t)k * a.carry_cap + cs] = a.cin_vals[(int64_t)k * a.cin_cap + c];
            a.carry_nulls[cs] = a.cin_nulls[c];
        }
    }
}

// one lane per key: the key's arena is private to the lane, so the state machine runs without atomics; only
// the output slot reservation is shared
__global__ __launch_bounds__(256) void nfa_k(NfaArgs a) {
    __shared__ int64_t stack_mem[STACK * 256];
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= a.K) return;
    int64_t b = 0, e = a.n;
    if (a.seg_start) {
        b = a.seg_start[k];
        e = a.seg_end[k];
    }
    if (b >= e) return;  // initPartition happens at a key's first event
    const Plan* P = a.plan;
    nfa::Ctx c;
    c.P = P;
    c.code = a.code;
    c.consts = a.consts;
    c.L = a.L;
    c.base = a.arena + k * a.L.bytes;
    c.stk = stack_mem + threadIdx.x;
    c.stride = 256;
    c.emit_ts = a.out_ts;
    c.emit_vals = a.out_vals;
    c.emit_nulls = a.out_nulls;
    c.emit_seq = a.out_emit_seq;
    c.emit_sub = a.out_sub;
    c.emit_key = a.out_key;
    c.emit_count = a.out_count;
    c.emit_cap = a.out_cap;
    c.flags = &a.flags[0];
    c.key = (uint32_t)k;
    nfa::KeyEvents ev{a.ts, a.qstream, a.orig, a.cols, a.nulls, b, e, a.seq_base};
    nfa::run_key(c, ev);
    if (c.ovf()) atomicOr(&a.flags[2], 1);
}

}  // namespace

static int64_t rx_ntiles(int64_t n) { return n <= 0 ? 1 : (n + RX_TILE - 1) / RX_TILE; }

size_t keygroup_workspace(int64_t n, int32_t K, int32_t ncols, const uint8_t* widths) {
    int64_t nt = rx_ntiles(n);
    int64_t ng = (nt + KG_GROUP - 1) / KG_GROUP;
    size_t b = (size_t)nt * 256 * 4 + (size_t)ng * 256 * 4 + 257 * 4 + 4 * (size_t)n * 4;
    for (int c = 0; c < ncols; ++c) b += 2 * (size_t)n * widths[c] + 256;
    return b + 4096;
}

void keygroup_bind(KeyGroupArgs& a, void* base) {
    uint8_t* p = (uint8_t*)base;
    auto take = [&](size_t bytes) {
        uint8_t* r = p;
        p += (bytes + 255) & ~size_t(255);
        return (void*)r;
    };
    int64_t nt = rx_ntiles(a.n);
    int64_t ng = (nt + KG_GROUP - 1) / KG_GROUP;
    a.counts = (uint32_t*)take((size_t)nt * 256 * 4);
    a.gsum = (uint32_t*)take((size_t)ng * 256 * 4);
    a.tot = (uint32_t*)take(257 * 4);
    for (int i = 0; i < 2; ++i) {
        a.tmp_keys[i] = (uint32_t*)take((size_t)a.n * 4);
        a.tmp_orig[i] = (uint32_t*)take((size_t)a.n * 4);
    }
    for (int i = 0; i < 2; ++i)
        for (int c = 0; c < a.ncols; ++c) a.tmp_cols[i][c] = take((size_t)a.n * a.width[c]);
}

void keygroup(const KeyGroupArgs& a, hipStream_t stream, hipEvent_t* marks) {
    int kbits = 0;
    while ((1ll << kbits) < (int64_t)a.K) ++kbits;
    if (kbits == 0) kbits = 1;
    int npass = (kbits + RX_MAXBITS - 1) / RX_MAXBITS;
    int bits = (kbits + npass - 1) / npass;
    int64_t nt = rx_ntiles(a.n);
    int ng = (int)((nt + KG_GROUP - 1) / KG_GROUP);
    if (marks) (void)hipEventRecord(marks[0], stream);
    for (int p = 0; p < npass; ++p) {
        int shift = p * bits;
        int b = min(bits, kbits - shift);
        int nb = 1 << b;
        uint32_t mask = (uint32_t)nb - 1;
        const uint32_t* kin = p == 0 ? a.keys : a.tmp_keys[(p - 1) & 1];
        bool last = p == npass - 1;
        hipLaunchKernelGGL(rx_hist, dim3((unsigned)nt), dim3(RX_THREADS), 0, stream, kin, a.n, shift, mask, nb, a.counts);
        int64_t gk = (int64_t)ng * nb;
        hipLaunchKernelGGL(rx_p1, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, (int)nt, nb, a.gsum);
        hipLaunchKernelGGL(rx_p2, dim3(1), dim3(256), 0, stream, a.gsum, ng, nb, a.tot);
        hipLaunchKernelGGL(rx_p3, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, a.gsum, a.tot,
                           (int)nt, nb);
        if (marks && p == 0) (void)hipEventRecord(marks[1], stream);
        RxPass rp;
        std::memset(&rp, 0, sizeof rp);
        rp.keys_in = kin;
        rp.keys_out = last ? a.keys_sorted : a.tmp_keys[p & 1];
        rp.orig_in = p == 0 ? nullptr : a.tmp_orig[(p - 1) & 1];
        rp.orig_out = last ? a.orig_sorted : a.tmp_orig[p & 1];
        rp.ncols = a.ncols;
        for (int c = 0; c < a.ncols; ++c) {
            rp.src[c] = p == 0 ? a.src[c] : a.tmp_cols[(p - 1) & 1][c];
            rp.dst[c] = last ? a.dst[c] : a.tmp_cols[p & 1][c];
            rp.width[c] = a.width[c];
        }
        rp.offsets = a.counts;
        rp.n = a.n;
        rp.shift = shift;
        rp.mask = mask;
        rp.nb = nb;
        rp.bits = b;
        hipLaunchKernelGGL(rx_scatter, dim3((unsigned)nt), dim3(RX_THREADS), 0, stream, rp);
    }
    if (marks) (void)hipEventRecord(marks[2], stream);
    (void)hipMemsetAsync(a.seg_start, 0, (size_t)a.K * 4, stream);
    (void)hipMemsetAsync(a.seg_end, 0, (size_t)a.K * 4, stream);
    hipLaunchKernelGGL(rx_segments, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, stream, a.keys_sorted, a.n,
                       a.seg_start, a.seg_end);
    if (marks) (void)hipEventRecord(marks[3], stream);
}

void chain_match(const ChainArgs& a, hipStream_t stream) {
    if (a.n <= 0) return;
    const int64_t tile = CM_THREADS * CM_EPT;
    hipLaunchKernelGGL(chain_match_k, dim3((unsigned)((a.n + tile - 1) / tile)), dim3(CM_THREADS), 0, stream, a);
}

void chain_carry(const ChainArgs& a, hipStream_t stream) {
    if (a.cin_n <= 0) return;
    hipLaunchKernelGGL(chain_carry_k, dim3((unsigned)((a.cin_n + 255) / 256)), dim3(256), 0, stream, a);
}

void nfa_run(const NfaArgs& a, hipStream_t stream) {
    if (a.K <= 0 || a.n <= 0) return;
    hipLaunchKernelGGL(nfa_k, dim3((unsigned)((a.K + 255) / 256)), dim3(256), 0, stream, a);
}

}  // namespace sdg
