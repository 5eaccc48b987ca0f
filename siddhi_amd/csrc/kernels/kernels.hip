// gfx950 kernels of the pattern/sequence path: key grouping and the generic keyed NFA (the chain matcher is
// in chain.hip).
//
// Wave64 throughout: ballots are 64-bit, lane masks use __lanemask_lt(), compaction is ballot + mbcnt with one
// atomic per wave. Everything is integer/byte work bound by HBM, so no MFMA.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "../engine/eval.h"
#include "kernels.h"
#include "wave.h"

namespace sdg {

namespace {

// ---------------------------------------------------------------------------------------------------------
// key grouping: LSD radix passes

__device__ __forceinline__ uint32_t digit_of(uint32_t k, int shift, uint32_t mask) { return (k >> shift) & mask; }

// per-tile digit histogram: counts[tile * nb + d]
// kcheck (first pass only): keys >= K (device-resident batches whose ids did not come from this engine) set
// *kflag; every later kernel masks its key-derived indices, so such a batch fails the flush without a fault
// prefix rows (keygroup's pre_n, first pass): virtual rows [0, hole) are not rows (they align the batch rows: the
// batch starts at the 64-row boundary hole + pre_n), rows [hole, hole + pre_n) take their keys from pre_keys, the rest
// from keys[i - hole - pre_n]; n counts the hole
template <int RX_TILE, int RX_THREADS>
__global__ __launch_bounds__(RX_THREADS) void rx_hist(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                      uint32_t mask, int nb, uint32_t* __restrict__ counts,
                                                      uint32_t kcheck, int* __restrict__ kflag,
                                                      const uint32_t* __restrict__ pre_keys, int64_t pre_n, int64_t hole) {
    __shared__ uint32_t h[1 << RX_MAXBITS];
    for (int d = threadIdx.x; d < nb; d += RX_THREADS) h[d] = 0;
    __syncthreads();
    int64_t base = (int64_t)blockIdx.x * RX_TILE;
    const int64_t pre_end = hole + pre_n;
    if (base + RX_TILE <= n && base >= pre_end && (((uintptr_t)(keys + base - pre_end)) & 15) == 0) {
        // full, 16-B aligned tile: 4 keys per load, every load of the thread in flight before the atomics
        constexpr int V = RX_TILE / RX_THREADS / 4;
        const uint4* kv = reinterpret_cast<const uint4*>(keys + base - pre_end);
        uint4 x[V];
#pragma unroll
        for (int r = 0; r < V; ++r) x[r] = kv[r * RX_THREADS + threadIdx.x];
#pragma unroll
        for (int r = 0; r < V; ++r) {
            if (kcheck && (x[r].x >= kcheck || x[r].y >= kcheck || x[r].z >= kcheck || x[r].w >= kcheck)) *kflag = 1;
            atomicAdd(&h[digit_of(x[r].x, shift, mask)], 1u);
            atomicAdd(&h[digit_of(x[r].y, shift, mask)], 1u);
            atomicAdd(&h[digit_of(x[r].z, shift, mask)], 1u);
            atomicAdd(&h[digit_of(x[r].w, shift, mask)], 1u);
        }
    } else {
#pragma unroll 4
        for (int r = 0; r < RX_TILE / RX_THREADS; ++r) {
            int64_t i = base + r * RX_THREADS + threadIdx.x;
            if (i < n && i >= hole) {
                const uint32_t k = i < pre_end ? pre_keys[i - hole] : keys[i - pre_end];
                if (kcheck && k >= kcheck) *kflag = 1;
                atomicAdd(&h[digit_of(k, shift, mask)], 1u);
            }
        }
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
#pragma unroll 8
    for (int b = b0; b < b1; ++b) s += counts[(int64_t)b * nb + d];  // independent loads: keep 8 in flight
    gsum[idx] = s;
}

// one block: per digit, exclusive scan over groups (in place) + digit totals; then exclusive scan over digits
__global__ __launch_bounds__(256) void rx_p2(uint32_t* __restrict__ gsum, int ng, int nb, uint32_t* __restrict__ tot) {
    __shared__ uint32_t part[256];
    int d = threadIdx.x;
    uint32_t run = 0;
    if (d < nb) {
        // 8 groups per round: the loads of a round are issued together (the scan itself is a register chain)
        int g = 0;
        for (; g + 8 <= ng; g += 8) {
            uint32_t c[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) c[j] = gsum[(int64_t)(g + j) * nb + d];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                gsum[(int64_t)(g + j) * nb + d] = run;
                run += c[j];
            }
        }
        for (; g < ng; ++g) {
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
    int b = b0;
    for (; b + 8 <= b1; b += 8) {  // as rx_p2: a round's loads issued together
        uint32_t c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = counts[(int64_t)(b + j) * nb + d];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            counts[(int64_t)(b + j) * nb + d] = run;
            run += c[j];
        }
    }
    for (; b < b1; ++b) {
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
    int mono_col;             // >= 0: payload column holding ts; flag a decrease in arrival order (bucketize)
    int* mono_flag;
    int ts32_col;             // >= 0: that payload column (int64 ts) is written as u32 offsets from *ts_base
    const int64_t* ts_base;
    uint8_t* lkey_out;        // non-null: u8 keys >> lkey_shift here instead of keys_out
    int lkey_shift;
    int ntiles;               // tiles; the grid is rounded up to a multiple of xcds (XCD remap)
    int xcds;                 // XCD count of the tile remap (1: tiles in block order)
    int64_t pre_n;            // first pass only: virtual rows [0, hole) are not rows (n counts them; the batch rows
    int64_t hole;             // start 64-row aligned at hole + pre_n), prefix rows [hole, hole + pre_n) come from
    const uint32_t* pre_keys; // pre_keys / pre_src (8-byte slots), the others from keys_in / src at i - hole - pre_n;
                              // a prefix row's orig is 0x80000000 | its index
    const void* pre_src[MAX_COLS + 2];
    int64_t orig_base;        // added to a row's orig when orig_in is nullptr (a sub-batch's first batch row)
    int32_t mono_prev;        // the mono check compares row 0 with src[-1] too (a sub-batch after the first)
    int32_t tile_off;         // the launch's first tile (ntiles counts from it)
};

// stable tile scatter. Tile element e = w * 1024 + r * 64 + lane belongs to wave w (16 rounds r), so a wave
// ranks its own elements in order with wave-private digit counters (ballot match over the digit bits; the
// LDS ops of one wave are in order, so no block barrier while counting). Then per digit: prefix over waves
// and the tile's digit starts; each column is staged in LDS in digit order and written out as coalesced runs
// (keys and original rows together as one 8-byte word).
// Tiles: 8192 rows x 512 threads (2 blocks per CU) or 16384 x 1024 (one block per CU, 154 KB of LDS): both 4
// waves/SIMD and 16 rows per lane; the larger tile doubles the average bucket run each tile writes (a 256-bucket
// pass writes runs of 64 rows instead of 32: fewer partial cache lines for the u8 / u32 columns).
// BITS: the digit width when fixed at compile time (8: every full 256-bucket pass; the ballot-match loop unrolls),
// 0: a.bits at run time
template <int RX_TILE, int RX_THREADS, bool PRE, int BITS = 0>
__global__ __launch_bounds__(RX_THREADS, 4) void rx_scatter(RxPass a) {
    constexpr int R = RX_TILE / RX_THREADS;  // 16 elements per lane
    constexpr int NW = RX_THREADS / 64;
    __shared__ uint16_t wc[NW][1 << RX_MAXBITS];  // per-wave digit counts (<= 1024), then per-wave digit bases
    __shared__ uint32_t tstart[1 << RX_MAXBITS];
    __shared__ uint32_t gbase[1 << RX_MAXBITS];
    __shared__ uint8_t sdig[RX_TILE];  // digit of each staged element: its destination is gbase + rank in the run
    __shared__ uint64_t stage[RX_TILE];
    __shared__ uint32_t gbase_ws[4];  // scan256_incl's wave totals
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    // XCD-aware tile order (kernels.h xcd_block): virtual tile v gives each XCD a contiguous run of tiles. A digit's
    // runs of consecutive tiles are adjacent in the output, so the cache line where one tile's run ends and the next
    // one's begins is completed in one XCD's L2 instead of being written back partially by two
    const uint32_t vt = xcd_block(blockIdx.x, gridDim.x, (uint32_t)a.xcds);
    if ((int)vt >= a.ntiles) return;  // block-uniform: the rounding of the grid
    const int64_t tile = (int64_t)vt + a.tile_off;  // (a launch may cover the pass's tiles from tile_off on)
    const int64_t base = tile * RX_TILE;
    const int64_t tile_n = min((int64_t)RX_TILE, a.n - base);
    const int64_t hole = PRE ? a.hole : 0;
    const int64_t pre_end = PRE ? a.hole + a.pre_n : 0;
    const int64_t tile_v = tile_n - (base < hole ? hole - base : 0);  // the tile's rows (its staged elements)
    const int64_t wbase = base + w * (R * 64);
    for (int d = t; d < a.nb; d += RX_THREADS) {
        gbase[d] = a.offsets[tile * a.nb + d];
#pragma unroll
        for (int v = 0; v < NW; ++v) wc[v][d] = 0;
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt();
    uint32_t rank[R];
    uint8_t dig[R];
    uint32_t kreg[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = wbase + r * 64 + lane;
        kreg[r] = i < a.n && i >= hole ? (PRE && i < pre_end ? a.pre_keys[i - hole] : a.keys_in[i - pre_end]) : 0u;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = wbase + r * 64 + lane;
        const bool valid = i < a.n && i >= hole;
        const uint32_t d = valid ? digit_of(kreg[r], a.shift, a.mask) : 0u;
        uint64_t peers = __ballot(valid);
        if constexpr (BITS > 0) {
#pragma unroll
            for (int bit = 0; bit < BITS; ++bit) {
                const bool on = (d >> bit) & 1u;
                const uint64_t b = __ballot(on);
                peers &= on ? b : ~b;
            }
        } else {
            for (int bit = 0; bit < a.bits; ++bit) {
                const bool on = (d >> bit) & 1u;
                const uint64_t b = __ballot(on);
                peers &= on ? b : ~b;
            }
        }
        const uint32_t before = valid ? wc[w][d] : 0u;
        rank[r] = before + (uint32_t)__popcll(peers & lt);
        dig[r] = (uint8_t)d;
        const int leader = peers ? __ffsll((unsigned long long)peers) - 1 : -1;
        if (valid && lane == leader) wc[w][d] = (uint16_t)(before + (uint32_t)__popcll(peers));
    }
    __syncthreads();
    // per digit: exclusive prefix over waves (in place) and the digit's tile total
    uint32_t tot = 0;
    if (t < 256) {
        if (t < a.nb) {
#pragma unroll
            for (int v = 0; v < NW; ++v) {
                const uint32_t c = wc[v][t];
                wc[v][t] = (uint16_t)tot;
                tot += c;
            }
        }
    }
    // exclusive scan of the digit totals (nb <= 256) -> tile-local start of each digit run
    {
        const uint32_t inc = scan256_incl(t < 256 ? tot : 0u, &gbase_ws[0]);
        if (t < 256) tstart[t] = inc - tot;
    }
    __syncthreads();
    static_assert(RX_TILE <= 65536, "staged positions packed as u16 pairs");
    uint32_t sp2[R / 2];  // staged position of element r: u16 half (r & 1) of sp2[r / 2] (registers)
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = wbase + r * 64 + lane;
        const uint32_t wr = wc[w][dig[r]] + rank[r];  // rank among the tile's elements of this digit
        const uint32_t p = tstart[dig[r]] + wr;
        sp2[r / 2] = (r & 1) ? (sp2[r / 2] | (p << 16)) : p;
        if (i < a.n && i >= hole) sdig[p] = dig[r];
    }
    auto sp_of = [&](int r) -> uint32_t { return (sp2[r / 2] >> ((r & 1) * 16)) & 0xFFFFu; };
    // keys | original rows as one word, then every payload column. Software-pipelined: column c + 1 is loaded
    // into registers before column c's stores are issued, so waiting for those loads (vmcnt counts loads and
    // stores in issue order on gfx9) never waits for the stores.
    auto load_word = [&](int c, uint64_t* v) {
        const int wd = a.width[c];
        const void* src = a.src[c];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t i = wbase + r * 64 + lane;
            uint64_t x = 0;
            if (PRE && i < pre_end) {
                if (i >= hole) x = ((const uint64_t*)a.pre_src[c])[i - hole];  // an 8-byte slot: the store keeps the
            } else if (i < a.n) {                                               // column's low bytes
                const int64_t j = i - pre_end;
                if (wd == 8) x = ((const uint64_t*)src)[j];
                else if (wd == 4) x = ((const uint32_t*)src)[j];
                else x = ((const uint8_t*)src)[j];
            }
            v[r] = x;
        }
    };
    uint64_t cur[R], nxt[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = wbase + r * 64 + lane;
        uint32_t o;
        if (PRE && i < pre_end) o = 0x80000000u | (uint32_t)(i - hole);
        else if (a.orig_in) o = i < a.n ? a.orig_in[i - pre_end] : 0u;
        else o = (uint32_t)(i - pre_end + a.orig_base);
        cur[r] = (uint64_t)kreg[r] | ((uint64_t)o << 32);
    }
    for (int c = -1; c < a.ncols; ++c) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t i = wbase + r * 64 + lane;
            if (i < a.n && i >= hole) stage[sp_of(r)] = cur[r];
        }
        if (a.mono_col >= 0 && c == a.mono_col) {  // arrival-order timestamps: compare with row i - 1
            const uint64_t* src = (const uint64_t*)a.src[c];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int64_t i = wbase + r * 64 + lane;
                uint64_t prev = __shfl_up(cur[r], 1);
                const bool has_prev = i > 0 || a.mono_prev;
                if (lane == 0 && has_prev && i < a.n) prev = src[i - 1];
                if (has_prev && i < a.n && (int64_t)cur[r] < (int64_t)prev) *a.mono_flag = 1;
            }
        }
        __syncthreads();
        if (c + 1 < a.ncols) load_word(c + 1, nxt);
        const bool to32 = c >= 0 && c == a.ts32_col;
        const int wd = c < 0 ? 8 : to32 ? 4 : a.width[c];
        void* dst = c < 0 ? nullptr : a.dst[c];
        const int64_t tb = to32 ? *a.ts_base : 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = r * RX_THREADS + t;
            if (j < tile_v) {
                const uint32_t dj = sdig[j];
                const uint32_t o = gbase[dj] + (uint32_t)j - tstart[dj];
                const uint64_t v = stage[j];
                if (c < 0) {
                    if (a.lkey_out) a.lkey_out[o] = (uint8_t)((uint32_t)v >> a.lkey_shift);
                    else a.keys_out[o] = (uint32_t)v;
                    a.orig_out[o] = (uint32_t)(v >> 32);
                } else if (to32) {
                    const int64_t d = (int64_t)v - tb;
                    if ((uint64_t)d > 0xFFFFFFFFull) *a.mono_flag = 1;  // span past u32 (or time went back)
                    ((uint32_t*)dst)[o] = (uint32_t)d;
                } else if (wd == 8) {
                    ((uint64_t*)dst)[o] = v;
                } else if (wd == 4) {
                    ((uint32_t*)dst)[o] = (uint32_t)v;
                } else {
                    ((uint8_t*)dst)[o] = (uint8_t)v;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) cur[r] = nxt[r];
    }
}

// key segments of the sorted keys: 4 consecutive rows per thread (one 16-B load; the neighbours come from the
// adjacent lanes, the wave's edges from two scalar-sized loads)
__global__ __launch_bounds__(256) void rx_segments(const uint32_t* __restrict__ keys, int64_t n, uint32_t K,
                                                   uint32_t* __restrict__ seg_start, uint32_t* __restrict__ seg_end) {
    const int64_t p = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    const int lane = threadIdx.x & 63;
    uint32_t k[4];
    if (p + 4 <= n) {
        const uint4 x = *reinterpret_cast<const uint4*>(keys + p);
        k[0] = x.x; k[1] = x.y; k[2] = x.z; k[3] = x.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = p + j < n ? keys[p + j] : 0xFFFFFFFFu;
    }
    uint32_t prev = __shfl_up(k[3], 1), next = __shfl_down(k[0], 1);
    if (lane == 0) prev = p > 0 && p - 1 < n ? keys[p - 1] : 0xFFFFFFFFu;
    if (lane == 63) next = p + 4 < n ? keys[p + 4] : 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = p + j;
        if (i >= n) break;
        const uint32_t kk = k[j];
        if (kk >= K) continue;  // flagged by rx_hist
        const uint32_t before = j == 0 ? prev : k[j - 1];
        const uint32_t after = j == 3 ? next : k[j + 1];
        if (i == 0 || before != kk) seg_start[kk] = (uint32_t)i;
        if (i == n - 1 || after != kk) seg_end[kk] = (uint32_t)(i + 1);
    }
}

// blocks per CU the generic NFA without timers is compiled for. 4 (4 waves/SIMD, <= 128 VGPRs, a few spills) measured
// no faster than 1 (150 VGPRs, 3 waves/SIMD) on C3 (175 vs 171 ms per 10^8 events, r2ab): the kernel is bound by its
// uncoalesced per-key arena traffic (each lane walks its own key's arena), not by latency hiding
#ifndef SDG_NFA_MINB
#define SDG_NFA_MINB 1
#endif
// one lane per key: the key's arena is private to the lane, so the state machine runs without atomics; only
// the output slot and log reservations are shared
// a key's run overflowed its arena: the flag the host checks, and the key on the list it takes spilled keys from
__device__ __forceinline__ void note_overflow(const NfaArgs& a, int64_t k) {
    atomicOr(&a.flags[2], 1);
    if (a.ovf_keys) {
        const unsigned i = atomicAdd(a.ovf_count, 1u);
        if (i < (unsigned)a.ovf_cap) a.ovf_keys[i] = (uint32_t)k;
    }
}

template <bool TM>
__global__ __launch_bounds__(256, TM ? 1 : SDG_NFA_MINB) void nfa_k(const NfaArgs* __restrict__ pa) {
    // arguments from a device copy: indexing a by-value kernel argument (cols[col]) makes the compiler copy the
    // whole struct to scratch per lane
    const NfaArgs& a = *pa;
    __shared__ int64_t stack_mem[STACK * 256];
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    int64_t k;
    if (a.list) {
        if (idx >= a.nlist) return;
        k = a.list[idx];
    } else {
        if (idx >= a.K) return;
        k = idx;
    }
    int64_t b = 0, e = a.n;
    if (a.seg_start) {
        b = a.seg_start[k];
        e = a.seg_end[k];
    }
    const Plan* P = a.plan;
    const int64_t kb = a.L.bytes;
    int64_t s = k;  // arena slot
    uint8_t from = 0;
    if (a.slot_of) {
        s = a.slot_of[k];
        if (s < 0) return;  // no rows (reclaiming queries have no timers)
        from = a.init_from[s];
    }
    uint8_t* src = a.arena + s * kb;
    uint8_t* dst = src;
    if (a.arena2) {
        if (a.cur[s]) src = a.arena2 + s * kb;
        else dst = a.arena2 + s * kb;
    }
    if (!from && (((const nfa::KHead*)src)->flags & nfa::KH_HOST)) return;  // a spilled key: the host runs it
    if (!a.list && b >= e && P->partitioned) {
        // no event of this key: it runs only for its queued timers (initPartition happens at a first event)
        const nfa::KHead* h = (const nfa::KHead*)src;
        if (!(h->flags & 2) || P->n_sched == 0) return;
        bool queued = false;
        const nfa::TQ* tq = (const nfa::TQ*)(src + a.L.off_tq);
        for (int i = 0; i < a.L.n_sched; ++i) queued |= tq[i].n > 0;
        if (!queued) return;
    }
    if (from) {  // no committed arena: fresh (zeros), or rebuilt from the idle record below
        uint4* d4 = (uint4*)dst;
        for (int64_t i = 0; i < kb / 16; ++i) d4[i] = make_uint4(0, 0, 0, 0);
        if (dst != src) a.ran[s] = 1;
    } else if (dst != src) {  // work on the other copy: the committed state stays intact until nfa_commit
        const uint4* s4 = (const uint4*)src;
        uint4* d4 = (uint4*)dst;
        for (int64_t i = 0; i < kb / 16; ++i) d4[i] = s4[i];
        a.ran[s] = 1;
    }
    nfa::CtxT<TM> c;
    c.P = P;
    c.code = a.code;
    c.consts = a.consts;
    c.L = a.L;
    c.base = dst;
    c.stk = stack_mem + threadIdx.x;
    c.stride = 256;
    c.emit_ts = a.out_ts;
    c.emit_vals = a.out_vals;
    c.emit_nulls = a.out_nulls;
    c.emit_seq = a.out_emit_seq;
    c.emit_sub = a.out_sub;
    c.emit_key = a.out_key;
    c.emit_round = a.out_round;
    c.round = a.round;
    c.emit_count = a.out_count;
    c.emit_cap = a.out_cap;
    c.flags = &a.flags[0];
    c.key = (uint32_t)k;
    c.T = a.T;
    c.fires = nullptr;
    c.nfires = -1;  // ideal mode unless a rerun list gives the fires
    if (a.list) {
        c.fires = a.fires + a.fire_off[idx];
        c.nfires = (int32_t)(a.fire_off[idx + 1] - a.fire_off[idx]);
    }
    // last_seen is stored XOR INT64_MIN, so the zero-filled array reads as "never seen"
    if (a.last_seen) c.purge = nfa::PurgeIn{a.purge_clk, a.purge_from, a.purge_idle, a.last_seen_in[k] ^ INT64_MIN};
    c.emit_flags = a.out_flags;
    if (from == 2) nfa::from_idle(c, a.idle_rec + k * a.idle_bytes);
    nfa::KeyEvents ev{a.ts, a.qstream, a.orig, a.cols, a.nulls, b, e, a.seq_base, a.pos_off, a.vrank};
    nfa::run_key(c, ev);
    if (a.last_seen) a.last_seen[k] = c.purge.last ^ INT64_MIN;
    if (a.agg_reset && c.purge_pending) a.agg_reset[k] = 1;
    if (a.releasable) a.releasable[s] = nfa::to_idle(c, a.idle_out + s * a.idle_bytes) ? 1 : 0;
    if (c.ovf()) note_overflow(a, k);
}

// The same state machine with each key's arena staged in LDS (nfa_k walks it in HBM: one lane per key, every
// access a separate cache line of a ~1-10 KB arena, 50-100x the algorithmic bytes, r2g_c3_pmc). A block is one
// wave whose `lanes` first lanes each own a key: the wave copies the committed arenas of its keys into LDS
// cooperatively (64 lanes x 16 B on one arena at a time: coalesced), every lane runs its key against its LDS copy
// (the arena code addresses through CtxT::base, a generic pointer, so the same nfa.h code runs), and the wave
// writes the arenas back, coalesced, into the working copy (double-buffered: the committed copy stays intact until
// nfa_commit). Concurrency is bounded by LDS (keys in flight per CU = LDS / arena bytes); lanes per wave is sized
// so that four such waves fit a CU, one per SIMD.
// Lane stride of the LDS arenas: every lane walks the same arena offsets, so a stride that is a multiple of 256 B
// (or of 64 B: 4 banks apart) puts the lanes of one wave-instruction on a few of the 64 banks -- r3i's C3 pass
// counted 1.09e10 SQ_LDS_BANK_CONFLICT cycles against 2.09e9 LDS instructions. A stride of 2 (mod 4) dwords gives
// the 32 lanes of a ds_read_b64 group 32 distinct bank pairs (the arena code reads 8-byte fields).
__host__ __device__ __forceinline__ int64_t nfa_lds_stride(int64_t kb) { return ((kb >> 3) & 1) ? kb : kb + 8; }

template <bool TM>
__global__ __launch_bounds__(64) void nfa_lds_k(const NfaArgs* __restrict__ pa, int lanes) {
    const NfaArgs& a = *pa;
    extern __shared__ __align__(16) uint8_t lds_arena[];
    __shared__ int64_t stack_mem[STACK * 64];
    const int lane = threadIdx.x;
    const int64_t idx = (int64_t)blockIdx.x * lanes + lane;
    const Plan* P = a.plan;
    const int64_t kb = a.L.bytes;
    bool active = lane < lanes;
    int64_t k = 0;
    if (active) {
        if (a.list) {
            active = idx < a.nlist;
            if (active) k = a.list[idx];
        } else {
            active = idx < a.K;
            k = idx;
        }
    }
    int64_t b = 0, e = a.n;
    const uint8_t* src = nullptr;
    uint8_t* dst = nullptr;
    int64_t s = k;     // arena slot
    uint8_t from = 0;  // 1: a fresh key, 2: rebuilt from its idle record (no committed arena to stage)
    if (active) {
        if (a.seg_start) {
            b = a.seg_start[k];
            e = a.seg_end[k];
        }
        if (a.slot_of) {
            s = a.slot_of[k];
            if (s < 0) active = false;  // no rows (slots go to keys with rows; reclaiming queries have no timers)
            else from = a.init_from[s];
        }
    }
    if (active) {
        src = a.arena + s * kb;
        dst = a.arena + s * kb;
        if (a.arena2) {
            if (a.cur[s]) src = a.arena2 + s * kb;
            else dst = a.arena2 + s * kb;
        }
        if (!from && (((const nfa::KHead*)src)->flags & nfa::KH_HOST)) active = false;  // spilled: the host runs it
        if (active && !a.list && b >= e && P->partitioned) {
            // no event of this key: it runs only for its queued timers (initPartition happens at a first event)
            const nfa::KHead* h = (const nfa::KHead*)src;
            if (!(h->flags & 2) || P->n_sched == 0) {
                active = false;
            } else {
                bool queued = false;
                const nfa::TQ* tq = (const nfa::TQ*)(src + a.L.off_tq);
                for (int i = 0; i < a.L.n_sched; ++i) queued |= tq[i].n > 0;
                active = queued;
            }
        }
    }
    const int64_t n8 = kb / 8;
    const int64_t ks = nfa_lds_stride(kb);
    // stage: the committed arenas of the active keys, one arena per wave instruction sweep (zeros for a key that
    // has none: fresh, or rebuilt from its idle record below)
    for (uint64_t m = __ballot(active); m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        const uint2* s8 = (const uint2*)__shfl((long long)(uintptr_t)src, j);
        const int fj = __shfl((int)from, j);
        uint2* d8 = (uint2*)(lds_arena + (int64_t)j * ks);
        if (fj) for (int64_t i = lane; i < n8; i += 64) d8[i] = make_uint2(0, 0);
        else for (int64_t i = lane; i < n8; i += 64) d8[i] = s8[i];
    }
    __syncthreads();
    bool ovf = false;
    if (active) {
        nfa::CtxT<TM> c;
        c.P = P;
        c.code = a.code;
        c.consts = a.consts;
        c.L = a.L;
        c.base = lds_arena + (int64_t)lane * ks;
        c.stk = stack_mem + lane;
        c.stride = 64;
        c.emit_ts = a.out_ts;
        c.emit_vals = a.out_vals;
        c.emit_nulls = a.out_nulls;
        c.emit_seq = a.out_emit_seq;
        c.emit_sub = a.out_sub;
        c.emit_key = a.out_key;
        c.emit_round = a.out_round;
        c.round = a.round;
        c.emit_count = a.out_count;
        c.emit_cap = a.out_cap;
        c.flags = &a.flags[0];
        c.key = (uint32_t)k;
        c.T = a.T;
        c.fires = nullptr;
        c.nfires = -1;
        if (a.list) {
            c.fires = a.fires + a.fire_off[idx];
            c.nfires = (int32_t)(a.fire_off[idx + 1] - a.fire_off[idx]);
        }
        if (a.last_seen) c.purge = nfa::PurgeIn{a.purge_clk, a.purge_from, a.purge_idle, a.last_seen_in[k] ^ INT64_MIN};
        c.emit_flags = a.out_flags;
        if (from == 2) nfa::from_idle(c, a.idle_rec + k * a.idle_bytes);
        nfa::KeyEvents ev{a.ts, a.qstream, a.orig, a.cols, a.nulls, b, e, a.seq_base, a.pos_off, a.vrank};
        nfa::run_key(c, ev);
        if (a.last_seen) a.last_seen[k] = c.purge.last ^ INT64_MIN;
        if (a.agg_reset && c.purge_pending) a.agg_reset[k] = 1;
        if (a.releasable) a.releasable[s] = nfa::to_idle(c, a.idle_out + s * a.idle_bytes) ? 1 : 0;
        ovf = c.ovf();
        if (dst != src) a.ran[s] = 1;
    }
    if (ovf) note_overflow(a, k);
    __syncthreads();
    // write back into the working copy
    for (uint64_t m = __ballot(active); m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        uint2* d8 = (uint2*)__shfl((long long)(uintptr_t)dst, j);
        const uint2* s8 = (const uint2*)(lds_arena + (int64_t)j * ks);
        for (int64_t i = lane; i < n8; i += 64) d8[i] = s8[i];
    }
}

// arena growth: every key's committed state into the larger layout (nfa.h migrate_key)
__global__ __launch_bounds__(256) void nfa_migrate_k(const Plan* __restrict__ plan, const uint8_t* __restrict__ arena,
                                                     const uint8_t* __restrict__ arena2, const uint8_t* __restrict__ cur,
                                                     nfa::Layout Ls, uint8_t* __restrict__ dst, nfa::Layout Ld, int64_t K) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    const uint8_t* src = (arena2 && cur[k] ? arena2 : arena) + k * Ls.bytes;
    nfa::CtxT<true> c;
    c.P = plan;
    c.L = Ld;
    c.base = dst + k * Ld.bytes;
    nfa::migrate_key(c, src, Ls);
}

__device__ __forceinline__ bool has_rows(const uint32_t* seg_start, const uint32_t* seg_end, int64_t k) {
    return !seg_start || seg_end[k] > seg_start[k];
}
__global__ __launch_bounds__(256) void nfa_slots_need_k(SlotPool sp, const uint32_t* __restrict__ seg_start,
                                                        const uint32_t* __restrict__ seg_end, int64_t K) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    // (-1 never seen, -2 idle: a slot for a key with rows; -3: spilled, the host runs it)
    const bool need = k < K && (sp.slot_of[k] == -1 || sp.slot_of[k] == -2) && has_rows(seg_start, seg_end, k);
    const uint64_t m = __ballot(need);
    if (m && lane_id() == __ffsll((unsigned long long)m) - 1) atomicAdd(&sp.counters[1], (unsigned)__popcll(m));
}
__global__ __launch_bounds__(256) void nfa_slots_assign_k(SlotPool sp, const uint32_t* __restrict__ seg_start,
                                                          const uint32_t* __restrict__ seg_end, int64_t K) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    const int32_t cur = sp.slot_of[k];
    if ((cur != -1 && cur != -2) || !has_rows(seg_start, seg_end, k)) return;
    const unsigned top = atomicSub(&sp.counters[0], 1u);  // (the host grew the pool to cover every such key)
    const int32_t s = sp.free_slots[top - 1];
    sp.slot_of[k] = s;
    sp.slot_key[s] = (int32_t)k;
    sp.init_from[s] = cur == -2 ? 2 : 1;
}
__global__ __launch_bounds__(256) void nfa_commit_slots_k(SlotPool sp, uint8_t* __restrict__ cur, uint8_t* __restrict__ ran,
                                                          int64_t S) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= S || !ran[s]) return;
    cur[s] ^= 1;
    ran[s] = 0;
    sp.init_from[s] = 0;
    if (!sp.releasable[s]) return;
    sp.releasable[s] = 0;
    const int64_t k = sp.slot_key[s];
    const int ib = sp.idle_bytes;
    for (int i = 0; i < ib; i += 4) *(int32_t*)(sp.idle_rec + k * ib + i) = *(const int32_t*)(sp.idle_out + s * ib + i);
    sp.slot_of[k] = -2;
    const unsigned top = atomicAdd(&sp.counters[0], 1u);
    sp.free_slots[top] = (int32_t)s;
}

__global__ __launch_bounds__(256) void nfa_commit_k(uint8_t* __restrict__ cur, uint8_t* __restrict__ ran, int64_t K) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K || !ran[k]) return;
    cur[k] ^= 1;
    ran[k] = 0;
}

}  // namespace

// SDG_RX_TILE=8192 / 16384: the radix tile (A/B); the workspace is sized for the smaller one
static int rx_tile() {
    static const int t = [] {
        const char* e = getenv("SDG_RX_TILE");
        return e && atoi(e) == RX_TILE_BIG ? RX_TILE_BIG : e && atoi(e) == RX_TILE ? RX_TILE : RX_TILE_DEFAULT;
    }();
    return t;
}
// the fused path's single bucket pass (bucketize): 8192-row tiles, two blocks per CU (r5j: scatter 1.39 -> 1.31 ms
// per C2 step against 16384-row tiles on the same box; the multi-pass key sort keeps rx_tile()).
// SDG_RX_TILE_BK=16384 for A/B
static int rx_tile_bucket() {
    static const int t = [] {
        const char* e = getenv("SDG_RX_TILE_BK");
        return e && atoi(e) == RX_TILE_BIG ? RX_TILE_BIG : RX_TILE;
    }();
    return t;
}
static int g_tile_override = 0;  // set around bucketize's launches
static int rx_tile_now() { return g_tile_override ? g_tile_override : rx_tile(); }
static int64_t rx_ntiles(int64_t n, int tile = RX_TILE) { return n <= 0 ? 1 : (n + tile - 1) / tile; }
static void launch_rx_hist(int64_t nt, hipStream_t stream, const uint32_t* keys, int64_t n, int shift, uint32_t mask,
                           int nb, uint32_t* counts, uint32_t kcheck, int* kflag, const uint32_t* pre_keys = nullptr,
                           int64_t pre_n = 0, int64_t hole = 0) {
    if (rx_tile_now() == RX_TILE_BIG)
        hipLaunchKernelGGL((rx_hist<RX_TILE_BIG, RX_THREADS_BIG>), dim3((unsigned)nt), dim3(RX_THREADS_BIG), 0, stream,
                           keys, n, shift, mask, nb, counts, kcheck, kflag, pre_keys, pre_n, hole);
    else
        hipLaunchKernelGGL((rx_hist<RX_TILE, RX_THREADS>), dim3((unsigned)nt), dim3(RX_THREADS), 0, stream, keys, n,
                           shift, mask, nb, counts, kcheck, kflag, pre_keys, pre_n, hole);
}
template <int BITS>
static void launch_rx_scatter_b(int64_t grid, hipStream_t stream, const RxPass& rp) {
    if (rp.pre_n > 0) {  // (prefix rows exist on the sorted-view path alone)
        if (rx_tile_now() == RX_TILE_BIG)
            hipLaunchKernelGGL((rx_scatter<RX_TILE_BIG, RX_THREADS_BIG, true, BITS>), dim3((unsigned)grid),
                               dim3(RX_THREADS_BIG), 0, stream, rp);
        else
            hipLaunchKernelGGL((rx_scatter<RX_TILE, RX_THREADS, true, BITS>), dim3((unsigned)grid), dim3(RX_THREADS), 0,
                               stream, rp);
    } else if (rx_tile_now() == RX_TILE_BIG) {
        hipLaunchKernelGGL((rx_scatter<RX_TILE_BIG, RX_THREADS_BIG, false, BITS>), dim3((unsigned)grid),
                           dim3(RX_THREADS_BIG), 0, stream, rp);
    } else {
        hipLaunchKernelGGL((rx_scatter<RX_TILE, RX_THREADS, false, BITS>), dim3((unsigned)grid), dim3(RX_THREADS), 0,
                           stream, rp);
    }
}
static void launch_rx_scatter(int64_t nt, hipStream_t stream, RxPass rp) {
    static const bool no_xcd = getenv("SDG_RX_NOXCD") != nullptr;  // A/B: tiles in block order
    static const bool no_b8 = getenv("SDG_RX_NO_B8") != nullptr;    // A/B: the run-time digit width for 8-bit passes
    static const bool no_split = getenv("SDG_RX_NO_SPLIT") != nullptr;  // A/B: one PRE launch over every tile
    rp.xcds = no_xcd ? 1 : g_xcds;
    if (rp.pre_n > 0 && !no_split) {
        // the tiles with prefix rows (or the alignment hole) take the PRE build; the ones past them -- nearly all --
        // the plain build, reading the batch columns through pointers moved back by the prefix (row i of the pass is
        // batch row i - pre_end there)
        const int tile = rx_tile_now();
        const int64_t pre_end = rp.hole + rp.pre_n;
        const int64_t t1 = std::min<int64_t>(nt, (pre_end + tile - 1) / tile);
        RxPass b = rp;
        rp.ntiles = (int)t1;
        rp.tile_off = 0;
        if (t1 > 0) launch_rx_scatter_b<0>(no_xcd ? t1 : xcd_round(t1), stream, rp);
        if (t1 < nt) {
            b.pre_n = 0;
            b.hole = 0;
            b.keys_in = b.keys_in - pre_end;
            if (b.orig_in) b.orig_in = b.orig_in - pre_end;
            else b.orig_base -= pre_end;
            for (int c = 0; c < b.ncols; ++c) b.src[c] = (const uint8_t*)b.src[c] - pre_end * (int64_t)b.width[c];
            b.ntiles = (int)(nt - t1);
            b.tile_off = (int32_t)t1;
            const int64_t g2 = no_xcd ? nt - t1 : xcd_round(nt - t1);
            if (b.bits == 8 && !no_b8) launch_rx_scatter_b<8>(g2, stream, b);
            else launch_rx_scatter_b<0>(g2, stream, b);
        }
        return;
    }
    rp.ntiles = (int)nt;
    const int64_t grid = no_xcd ? nt : xcd_round(nt);
    // (the 8192-row tile only: the bucket pass. C2 scatter 1.375 -> 1.350 ms, r6l; the key sort's 16384-row passes
    // measured no gain)
    if (rp.bits == 8 && !no_b8 && rx_tile_now() != RX_TILE_BIG) launch_rx_scatter_b<8>(grid, stream, rp);
    else launch_rx_scatter_b<0>(grid, stream, rp);
}

size_t keygroup_workspace(int64_t n, int32_t K, int32_t ncols, const uint8_t* widths) {
    int64_t nt = rx_ntiles(n + 64);  // (+ the first pass's alignment hole)
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
    int64_t nt = rx_ntiles(a.n + 64);
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
    // the first pass reads the prefix rows (the sorted view's carried partials) ahead of the batch; a hole of < 64
    // virtual rows in front of them puts the batch rows at a 64-row boundary, so the batch's loads stay aligned
    const int64_t hole = a.pre_n > 0 ? (64 - a.pre_n % 64) % 64 : 0;
    if (marks) (void)hipEventRecord(marks[0], stream);
    for (int p = 0; p < npass; ++p) {
        int shift = p * bits;
        int b = min(bits, kbits - shift);
        int nb = 1 << b;
        uint32_t mask = (uint32_t)nb - 1;
        const uint32_t* kin = p == 0 ? a.keys : a.tmp_keys[(p - 1) & 1];
        bool last = p == npass - 1;
        const int64_t np = p == 0 ? a.n + hole : a.n;  // rows of this pass (virtual: with the hole)
        const int64_t nt = rx_ntiles(np, rx_tile());
        const int ng = (int)((nt + KG_GROUP - 1) / KG_GROUP);
        launch_rx_hist(nt, stream, kin, np, shift, mask, nb, a.counts, p == 0 && a.key_flag ? (uint32_t)a.K : 0u,
                       a.key_flag, p == 0 ? a.pre_keys : nullptr, p == 0 ? a.pre_n : 0, p == 0 ? hole : 0);
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
        rp.orig_in = p == 0 ? a.orig_in : a.tmp_orig[(p - 1) & 1];
        rp.orig_out = last ? a.orig_sorted : a.tmp_orig[p & 1];
        rp.ncols = a.ncols;
        for (int c = 0; c < a.ncols; ++c) {
            rp.src[c] = p == 0 ? a.src[c] : a.tmp_cols[(p - 1) & 1][c];
            rp.dst[c] = last ? a.dst[c] : a.tmp_cols[p & 1][c];
            rp.width[c] = a.width[c];
        }
        rp.offsets = a.counts;
        rp.n = np;
        rp.shift = shift;
        rp.mask = mask;
        rp.nb = nb;
        rp.bits = b;
        rp.mono_col = -1;
        rp.ts32_col = -1;
        if (a.ts32_col >= 0) {  // the first pass converts the int64 ts to u32 offsets, the later ones move u32
            if (p == 0) {
                rp.ts32_col = a.ts32_col;
                rp.ts_base = a.ts_base;
                rp.mono_flag = a.ts32_flag;
            } else {
                rp.width[a.ts32_col] = 4;
            }
        }
        if (p == 0 && a.pre_n > 0) {
            rp.pre_n = a.pre_n;
            rp.hole = hole;
            rp.pre_keys = a.pre_keys;
            for (int c = 0; c < a.ncols; ++c) rp.pre_src[c] = a.pre_src[c];
        }
        launch_rx_scatter(nt, stream, rp);
    }
    if (marks) (void)hipEventRecord(marks[2], stream);
    if (!a.no_segments) {
        (void)hipMemsetAsync(a.seg_start, 0, (size_t)a.K * 4, stream);
        (void)hipMemsetAsync(a.seg_end, 0, (size_t)a.K * 4, stream);
        hipLaunchKernelGGL(rx_segments, dim3((unsigned)((a.n + 1023) / 1024)), dim3(256), 0, stream, a.keys_sorted, a.n,
                           (uint32_t)a.K, a.seg_start, a.seg_end);
    }
    if (marks) (void)hipEventRecord(marks[3], stream);
}

namespace {
// bucket row ranges and the fused matcher's block plan (one block, nb <= 256)
// tm: the time-major order (kernels.h ChainArgs::tm), when the buckets are balanced enough that enumerating
// (segment index, bucket) costs little (S * nb <= 2 * segments + 256) and it fits tm_cap
__global__ __launch_bounds__(256) void bk_plan(const uint32_t* __restrict__ tot, int64_t n, int nb, int seg_rows,
                                               uint32_t* __restrict__ bstart, uint32_t* __restrict__ bseg,
                                               uint32_t* __restrict__ tm, int64_t tm_cap,
                                               const uint32_t* __restrict__ offs = nullptr, int64_t halo_tile = 0,
                                               int64_t ntiles = 0, uint32_t* __restrict__ bown = nullptr) {
    __shared__ uint32_t part[256], sg[256], smax, smin;
    const int d = threadIdx.x;
    uint32_t s0 = 0, len = 0;
    if (d < nb) {
        s0 = tot[d];
        const uint32_t s1 = d + 1 < nb ? tot[d + 1] : (uint32_t)n;
        len = s1 - s0;
        bstart[d] = s0;
        if (bown) {  // sub-batch: the bucket's own rows end where the first halo tile's run of it starts (the scan's
                     // rewritten counts are each (tile, digit) run's output offset)
            const uint32_t oe = halo_tile < ntiles ? offs[halo_tile * nb + d] : s1;
            bown[d] = oe;
            len = oe - s0;  // segments over the own rows only
        }
    }
    const uint32_t segs = (len + (uint32_t)seg_rows - 1) / (uint32_t)seg_rows;
    part[d] = segs;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const uint32_t x = d >= off ? part[d - off] : 0u;
        __syncthreads();
        part[d] += x;
        __syncthreads();
    }
    if (d < nb) bseg[d] = part[d] - segs;
    if (d == 255) {
        bstart[nb] = (uint32_t)n;
        bseg[nb] = part[255];
    }
    if (!tm) return;
    sg[d] = segs;
    if (d == 0) {
        smax = 0;
        smin = 0xFFFFFFFFu;
    }
    __syncthreads();
    atomicMax(&smax, segs);
    if (d < nb) atomicMin(&smin, segs);
    __syncthreads();
    const uint32_t S = smax, total = part[255];
    const bool on = S > 0 && (uint64_t)S * (uint64_t)nb <= 2ull * total + 256 && (int64_t)S + 3 <= tm_cap;
    if (d == 0) {
        tm[0] = on ? S : 0u;
        tm[1] = smin;
    }
    if (!on) return;
    for (uint32_t s = d; s <= S; s += 256) {
        uint32_t acc = 0;
        for (int b = 0; b < nb; ++b) acc += min(sg[b], s);
        tm[2 + s] = acc;
    }
}
}  // namespace

void bucketize(const KeyGroupArgs& a, int bits, int ts_col, int* mono_flag, uint32_t* bstart, uint32_t* bseg,
               int seg_rows, hipStream_t stream, hipEvent_t* marks, uint32_t* tm, int64_t tm_cap) {
    const int nb = 1 << bits;
    const uint32_t mask = (uint32_t)nb - 1;
    g_tile_override = rx_tile_bucket();
    const int64_t nt = rx_ntiles(a.n, g_tile_override);
    const int ng = (int)((nt + KG_GROUP - 1) / KG_GROUP);
    if (marks) (void)hipEventRecord(marks[0], stream);
    launch_rx_hist(nt, stream, a.keys, a.n, 0, mask, nb, a.counts, a.key_flag ? (uint32_t)a.K : 0u, a.key_flag);
    const int64_t gk = (int64_t)ng * nb;
    hipLaunchKernelGGL(rx_p1, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, (int)nt, nb, a.gsum);
    hipLaunchKernelGGL(rx_p2, dim3(1), dim3(256), 0, stream, a.gsum, ng, nb, a.tot);
    hipLaunchKernelGGL(rx_p3, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, a.gsum, a.tot,
                       (int)nt, nb);
    if (marks) (void)hipEventRecord(marks[1], stream);
    RxPass rp;
    std::memset(&rp, 0, sizeof rp);
    rp.keys_in = a.keys;
    rp.keys_out = a.keys_sorted;
    rp.orig_in = a.orig_in;
    rp.orig_out = a.orig_sorted;
    rp.ncols = a.ncols;
    for (int c = 0; c < a.ncols; ++c) {
        rp.src[c] = a.src[c];
        rp.dst[c] = a.dst[c];
        rp.width[c] = a.width[c];
    }
    rp.offsets = a.counts;
    rp.n = a.n;
    rp.shift = 0;
    rp.mask = mask;
    rp.nb = nb;
    rp.bits = bits;
    rp.mono_col = ts_col;
    rp.mono_flag = mono_flag;
    rp.ts32_col = a.ts32_col;
    rp.ts_base = a.ts_base;
    rp.lkey_out = a.lkey_out;
    rp.lkey_shift = bits;
    launch_rx_scatter(nt, stream, rp);
    g_tile_override = 0;
    if (marks) (void)hipEventRecord(marks[2], stream);
    hipLaunchKernelGGL(bk_plan, dim3(1), dim3(256), 0, stream, a.tot, a.n, nb, seg_rows, bstart, bseg, tm, tm_cap);
    if (marks) (void)hipEventRecord(marks[3], stream);
}

int bucket_tile() { return rx_tile_bucket(); }

void bucketize_sub(const KeyGroupArgs& a, int bits, int ts_col, int* mono_flag, int64_t row0, int64_t n, int64_t own,
                   uint32_t* bstart, uint32_t* bseg, uint32_t* bown, int seg_rows, hipStream_t stream) {
    const int nb = 1 << bits;
    const uint32_t mask = (uint32_t)nb - 1;
    g_tile_override = rx_tile_bucket();
    const int64_t tile = g_tile_override;
    const int64_t nt = rx_ntiles(n, tile);
    const int ng = (int)((nt + KG_GROUP - 1) / KG_GROUP);
    launch_rx_hist(nt, stream, a.keys + row0, n, 0, mask, nb, a.counts, a.key_flag ? (uint32_t)a.K : 0u, a.key_flag);
    const int64_t gk = (int64_t)ng * nb;
    hipLaunchKernelGGL(rx_p1, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, (int)nt, nb, a.gsum);
    hipLaunchKernelGGL(rx_p2, dim3(1), dim3(256), 0, stream, a.gsum, ng, nb, a.tot);
    hipLaunchKernelGGL(rx_p3, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, a.gsum, a.tot,
                       (int)nt, nb);
    RxPass rp;
    std::memset(&rp, 0, sizeof rp);
    rp.keys_in = a.keys + row0;
    rp.keys_out = a.keys_sorted;
    rp.orig_in = nullptr;
    rp.orig_out = a.orig_sorted;
    rp.orig_base = row0;
    rp.mono_prev = row0 > 0;
    rp.ncols = a.ncols;
    for (int c = 0; c < a.ncols; ++c) {
        rp.src[c] = (const uint8_t*)a.src[c] + row0 * a.width[c];
        rp.dst[c] = a.dst[c];
        rp.width[c] = a.width[c];
    }
    rp.offsets = a.counts;
    rp.n = n;
    rp.shift = 0;
    rp.mask = mask;
    rp.nb = nb;
    rp.bits = bits;
    rp.mono_col = ts_col;
    rp.mono_flag = mono_flag;
    rp.ts32_col = a.ts32_col;
    rp.ts_base = a.ts_base;
    rp.lkey_out = a.lkey_out;
    rp.lkey_shift = bits;
    launch_rx_scatter(nt, stream, rp);
    g_tile_override = 0;
    hipLaunchKernelGGL(bk_plan, dim3(1), dim3(256), 0, stream, a.tot, n, nb, seg_rows, bstart, bseg, (uint32_t*)nullptr,
                       (int64_t)0, (const uint32_t*)a.counts, own / tile, nt, bown);
}

namespace {
__global__ void sub_halo_check_k(const int64_t* __restrict__ ts, int64_t n, int64_t S, int64_t H, int64_t within,
                                 int64_t J, int* __restrict__ flags) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 >= J) return;  // the last sub-batch has no halo
    const int64_t last_own = (j + 1) * S - 1, after = (j + 1) * S + H;
    if (after < n && !(ts[after] - ts[last_own] > within)) flags[5] = 1;
}
}  // namespace

void sub_halo_check(const int64_t* ts, int64_t n, int64_t S, int64_t H, int64_t within_ms, int* flags, hipStream_t st) {
    const int64_t J = (n + S - 1) / S;
    if (J <= 1) return;
    hipLaunchKernelGGL(sub_halo_check_k, dim3((unsigned)((J + 255) / 256)), dim3(256), 0, st, ts, n, S, H, within_ms, J,
                       flags);
}

void nfa_migrate(const Plan* plan, const uint8_t* arena, const uint8_t* arena2, const uint8_t* cur,
                 const nfa::Layout& Ls, uint8_t* dst, const nfa::Layout& Ld, int64_t K, hipStream_t stream) {
    if (K <= 0) return;
    hipLaunchKernelGGL(nfa_migrate_k, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, plan, arena, arena2, cur,
                       Ls, dst, Ld, K);
}

int nfa_lds_lanes(const nfa::Layout& L) {
    static const char* off = getenv("SDG_NFA_HBM");  // A/B: the arena-in-HBM kernel
    if (off) return 0;
    static const char* bud = getenv("SDG_NFA_LDS");  // A/B: LDS bytes per block (wave)
    const int64_t budget = bud ? atoll(bud) : NFA_LDS_BUDGET;
    const int64_t lanes = budget / nfa_lds_stride(L.bytes);
    return lanes >= NFA_LDS_MIN_LANES ? (int)(lanes < 64 ? lanes : 64) : 0;
}

void nfa_run(const NfaArgs& a, const NfaArgs* d_a, hipStream_t stream) {
    const int64_t keys = a.list ? a.nlist : a.K;
    if (keys <= 0) return;
    const int lanes = nfa_lds_lanes(a.L);
    if (lanes > 0) {
        const unsigned grid = (unsigned)((keys + lanes - 1) / lanes);
        const size_t lds = (size_t)lanes * (size_t)nfa_lds_stride(a.L.bytes);
        if (a.T.log) hipLaunchKernelGGL(nfa_lds_k<true>, dim3(grid), dim3(64), lds, stream, d_a, lanes);
        else hipLaunchKernelGGL(nfa_lds_k<false>, dim3(grid), dim3(64), lds, stream, d_a, lanes);
        return;
    }
    if (a.T.log) hipLaunchKernelGGL(nfa_k<true>, dim3((unsigned)((keys + 255) / 256)), dim3(256), 0, stream, d_a);
    else hipLaunchKernelGGL(nfa_k<false>, dim3((unsigned)((keys + 255) / 256)), dim3(256), 0, stream, d_a);
}

void nfa_slots_need(const SlotPool& sp, const uint32_t* seg_start, const uint32_t* seg_end, int64_t K, hipStream_t st) {
    if (K > 0) hipLaunchKernelGGL(nfa_slots_need_k, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, st, sp, seg_start, seg_end, K);
}
void nfa_slots_assign(const SlotPool& sp, const uint32_t* seg_start, const uint32_t* seg_end, int64_t K, hipStream_t st) {
    if (K > 0) hipLaunchKernelGGL(nfa_slots_assign_k, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, st, sp, seg_start, seg_end, K);
}
void nfa_commit_slots(const SlotPool& sp, uint8_t* cur, uint8_t* ran, int64_t slots, hipStream_t st) {
    if (slots > 0) hipLaunchKernelGGL(nfa_commit_slots_k, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, st, sp, cur, ran, slots);
}

int g_xcds = 8;
int g_cus = 256;

namespace {
__global__ void ts_window_base_k(const int64_t* __restrict__ ts, int64_t* __restrict__ out) {
    if (threadIdx.x == 0) out[0] = ts[0] - ((int64_t)1 << 31);
}
}  // namespace
void ts_window_base(const int64_t* ts, int64_t* out, hipStream_t stream) {
    hipLaunchKernelGGL(ts_window_base_k, dim3(1), dim3(64), 0, stream, ts, out);
}

void nfa_commit(uint8_t* cur, uint8_t* ran, int64_t K, hipStream_t stream) {
    if (K <= 0) return;
    hipLaunchKernelGGL(nfa_commit_k, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, cur, ran, K);
}

}  // namespace sdg
