// Delivery order of a flush's match records on the device: records come out of the matchers in arbitrary order
// (wave-aggregated appends), and the reference delivers them by emitting event, then by the partial's place in
// the pending list (StateMultiProcessStreamReceiver.processAndClear :47-68, QuerySelector.processNoGroupBy
// :161-205). One LSD radix sort of a record index by the emitting event's position (rocPRIM: a library sort for a
// bookkeeping pass, not the matching path) over the bits the flush's records use, then each run of one event's
// records (short: the partials one event completed) insertion-sorted by its ordinal; a run over RUN_MAX records
// falls back to two sorts (by the ordinal, then stably by the event). The columns follow through one packed
// gather, so the host / the gather reads the records already in order.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "../engine/eval.h"
#include "kernels.h"

namespace sdg {
namespace {

// the key ranges: max of emit - emit_base (u32), min / max of sub - sub_bias (u64); r[0] = max emit, r[1] = min sub,
// r[2] = max sub (the host sized the sorts by them: the ordinal / e1 position spans far fewer bits than its type)
__global__ __launch_bounds__(256) void order_range_k(const int64_t* __restrict__ emit, const int64_t* __restrict__ sub,
                                                     int64_t n, int64_t emit_base, int64_t sub_bias,
                                                     unsigned long long* __restrict__ r) {
    unsigned long long emx = 0, smn = ~0ull, smx = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const unsigned long long e = (unsigned long long)(uint32_t)(emit[i] - emit_base);
        const unsigned long long s = (unsigned long long)(sub[i] - sub_bias);
        emx = e > emx ? e : emx;
        smn = s < smn ? s : smn;
        smx = s > smx ? s : smx;
    }
    for (int o = 32; o > 0; o >>= 1) {  // wave reduction, then one atomic per wave
        const unsigned long long e2 = __shfl_xor(emx, o), n2 = __shfl_xor(smn, o), x2 = __shfl_xor(smx, o);
        emx = e2 > emx ? e2 : emx;
        smn = n2 < smn ? n2 : smn;
        smx = x2 > smx ? x2 : smx;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&r[0], emx);
        atomicMin(&r[1], smn);
        atomicMax(&r[2], smx);
    }
}

__global__ __launch_bounds__(256) void order_emit_keys_k(const int64_t* __restrict__ emit, int64_t n, int64_t emit_base,
                                                         uint32_t* __restrict__ ek, uint32_t* __restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    ek[i] = (uint32_t)(emit[i] - emit_base);
    idx[i] = (uint32_t)i;
}

template <typename SK>
__global__ __launch_bounds__(256) void order_keys_k(const int64_t* __restrict__ emit, const int64_t* __restrict__ sub,
                                                    int64_t n, int64_t emit_base, int64_t sub_bias, uint32_t* __restrict__ ek,
                                                    SK* __restrict__ sk, uint32_t* __restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    ek[i] = (uint32_t)(emit[i] - emit_base);
    sk[i] = (SK)(sub[i] - sub_bias);
    idx[i] = (uint32_t)i;
}

// after the sort by the emitting event: each run of records with one emitting event, in ordinal order. A run is
// short (the partials one event completes / the records one event emits); its first record's thread insertion-sorts
// the run's record indices by sub. A run longer than RUN_MAX is left to the two-sort ordering (*long_run set).
constexpr int RUN_MAX = 256;
__global__ __launch_bounds__(256) void order_runs_k(const uint32_t* __restrict__ ek, uint32_t* __restrict__ perm,
                                                    const int64_t* __restrict__ sub, int64_t n, int* __restrict__ long_run) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t e = ek[i];
    if (i > 0 && ek[i - 1] == e) return;  // not the first record of its run
    int64_t j = i + 1;
    while (j < n && ek[j] == e && j - i <= RUN_MAX) ++j;
    const int64_t len = j - i;
    if (len < 2) return;
    if (len > RUN_MAX) {
        atomicOr(long_run, 1);
        return;
    }
    for (int64_t x = i + 1; x < j; ++x) {  // insertion sort by sub (the run's records are few)
        const uint32_t v = perm[x];
        const int64_t kv = sub[v];
        int64_t y = x - 1;
        while (y >= i && sub[perm[y]] > kv) {
            perm[y + 1] = perm[y];
            --y;
        }
        perm[y + 1] = v;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void gather_k(const T* __restrict__ src, const uint32_t* __restrict__ perm, int64_t n,
                                                T* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}

// packed-record gather: the columns are first written row-major (one record = ncol consecutive int64s, a
// sequential pass), then each output slot reads its record's bytes in one place instead of ncol random 8-byte
// reads from ncol columns (a random 8-byte read costs a whole memory transaction)
struct ColSet {
    const int64_t* src[GATHER_MAX_COLS];
    int64_t* dst[GATHER_MAX_COLS];
};
__global__ __launch_bounds__(256) void pack_k(ColSet cs, int ncol, int64_t n, int64_t* __restrict__ rec) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    for (int c = 0; c < ncol; ++c) rec[i * ncol + c] = cs.src[c][i];
}
__global__ __launch_bounds__(256) void unpack_k(ColSet cs, int ncol, const int64_t* __restrict__ rec,
                                                const uint32_t* __restrict__ perm, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t* r = rec + (int64_t)perm[i] * ncol;
    for (int c = 0; c < ncol; ++c) cs.dst[c][i] = r[c];
}

// the same result as order_runs_k, written to a second index array: each record finds its run of equal emitting
// events around it (a few coalesced reads of the sorted keys), counts the run's records that precede it by
// (sub, sorted index) and writes its index at run start + that rank. No thread walks a whole run serially, and no
// record moves twice (order_runs_k insertion-sorted each run in place, one thread per run: 0.62 ms per 40M records)
// Each record's sub is read once (the one random read); the run's other subs come from the neighbouring lanes by
// shuffles (a wave holds 64 consecutive sorted records, and runs are short), from memory only past the wave's edge.
__global__ __launch_bounds__(256) void order_runs_rank_k(const uint32_t* __restrict__ ek, const uint32_t* __restrict__ ix,
                                                         const int64_t* __restrict__ sub, int64_t n,
                                                         uint32_t* __restrict__ perm, int* __restrict__ long_run) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool in = i < n;
    const uint32_t e = in ? ek[i] : 0u;
    int64_t s = i, t = i + 1;
    if (in) {
        while (s > 0 && i - s <= RUN_MAX && ek[s - 1] == e) --s;
        while (t < n && t - s <= RUN_MAX && ek[t] == e) ++t;
    }
    const bool lng = in && t - s > RUN_MAX;  // (left to the two-sort ordering)
    if (lng) atomicOr(long_run, 1);
    const bool multi = in && !lng && t - s > 1;
    const uint32_t me = in ? ix[i] : 0u;
    const int64_t my = multi ? sub[me] : 0;
    int64_t rank = 0;
    // offsets d = 1 .. the wave's longest run: lane + d / lane - d by shuffle when inside the wave
    int span = multi ? (int)(t - s) : 0;
    for (int o = 32; o > 0; o >>= 1) span = max(span, __shfl_xor(span, o));
    for (int d = 1; d < span; ++d) {
        const int64_t fw = __shfl(my, min(lane + d, 63));
        const int64_t bw = __shfl(my, max(lane - d, 0));
        if (!multi) continue;
        if (i + d < t) {  // a later record of the run: before me only with a smaller sub
            const int64_t o = lane + d < 64 ? fw : sub[ix[i + d]];
            rank += o < my;
        }
        if (i - d >= s) {  // an earlier one: before me unless its sub is larger (equal subs keep the sorted order)
            const int64_t o = lane - d >= 0 ? bw : sub[ix[i - d]];
            rank += o <= my;
        }
    }
    if (in && !lng) perm[multi ? s + rank : i] = me;
}

// The export's ordering pass in one kernel (export_ordered): the run rank of order_runs_rank_k, then the record's
// columns gathered straight to their final slot -- no index array written and read back. The emitting position is
// not gathered at all: in delivery order it is the sorted key + emit_base (seq_dst).
__global__ __launch_bounds__(256) void order_runs_gather_k(const uint32_t* __restrict__ ek, const uint32_t* __restrict__ ix,
                                                           const int64_t* __restrict__ sub, int64_t n, ColSet cs,
                                                           int ncol, int64_t* __restrict__ seq_dst, int64_t emit_base,
                                                           int* __restrict__ long_run, uint32_t xcds) {
    const uint32_t vb = xcd_block(blockIdx.x, gridDim.x, xcds);
    const int64_t i = (int64_t)vb * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool in = i < n;
    const uint32_t e = in ? ek[i] : 0u;
    int64_t s = i, t = i + 1;
    if (in) {
        while (s > 0 && i - s <= RUN_MAX && ek[s - 1] == e) --s;
        while (t < n && t - s <= RUN_MAX && ek[t] == e) ++t;
    }
    const bool lng = in && t - s > RUN_MAX;
    if (lng) atomicOr(long_run, 1);
    const bool multi = in && !lng && t - s > 1;
    const uint32_t me = in ? ix[i] : 0u;
    const int64_t my = multi ? sub[me] : 0;
    int64_t rank = 0;
    int span = multi ? (int)(t - s) : 0;
    for (int o = 32; o > 0; o >>= 1) span = max(span, __shfl_xor(span, o));
    for (int d = 1; d < span; ++d) {
        const int64_t fw = __shfl(my, min(lane + d, 63));
        const int64_t bw = __shfl(my, max(lane - d, 0));
        if (!multi) continue;
        if (i + d < t) rank += (lane + d < 64 ? fw : sub[ix[i + d]]) < my;
        if (i - d >= s) rank += (lane - d >= 0 ? bw : sub[ix[i - d]]) <= my;
    }
    if (!in || lng) return;
    const int64_t f = multi ? s + rank : i;
    int64_t x[GATHER_MAX_COLS];
#pragma unroll
    for (int c = 0; c < GATHER_MAX_COLS; ++c)
        if (c < ncol) x[c] = cs.src[c][me];
#pragma unroll
    for (int c = 0; c < GATHER_MAX_COLS; ++c)
        if (c < ncol) cs.dst[c][f] = x[c];
    if (seq_dst) seq_dst[f] = emit_base + (int64_t)e;
}

// order_runs_gather_k with the run bounds from wave ballots (a record's neighbours by shuffles; only a run that
// crosses the wave's edge scans HBM) and the column gathers issued right after the index load, so they overlap the
// run / rank work: two dependent memory waits per record instead of five or more
#ifndef SDG_OG_THREADS
#define SDG_OG_THREADS 256
#endif
constexpr int OG_T = SDG_OG_THREADS;  // order_runs_gather_w_k block size
__global__ __launch_bounds__(OG_T) void order_runs_gather_w_k(const uint32_t* __restrict__ ek, const uint32_t* __restrict__ ix,
                                                             const int64_t* __restrict__ sub, int64_t n, ColSet cs,
                                                             int ncol, int64_t* __restrict__ seq_dst, int64_t emit_base,
                                                             int* __restrict__ long_run, uint32_t xcds) {
    const uint32_t vb = xcd_block(blockIdx.x, gridDim.x, xcds);
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)vb * OG_T + threadIdx.x;
    const int64_t i0 = i - lane;  // the wave's first record
    const bool in = i < n;
    const uint32_t e = in ? ek[i] : 0xFFFFFFFFu;  // (positions < 2^32 - 1: the sentinel never equals a key)
    const uint32_t me = in ? ix[i] : 0u;
    uint32_t edge = 0xFFFFFFFEu;
    if (lane == 0 && in && i > 0) edge = ek[i - 1];
    if (lane == 63 && i + 1 < n) edge = ek[i + 1];
    int64_t x[GATHER_MAX_COLS];
#pragma unroll
    for (int c = 0; c < GATHER_MAX_COLS; ++c)
        if (c < ncol && in) x[c] = cs.src[c][me];
    uint32_t prev = __shfl_up(e, 1), next = __shfl_down(e, 1);
    if (lane == 0) prev = edge;
    if (lane == 63) next = edge;
    const uint64_t H = __ballot(in && e != prev), T = __ballot(in && e != next);
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);  // lanes 0..lane
    const uint64_t hm = H & upto, tm = T & ~(upto >> 1);              // heads at or below / tails at or above
    int64_t s = hm ? i0 + (63 - __clzll(hm)) : -1;
    int64_t t = tm ? i0 + (__ffsll((unsigned long long)tm) - 1) + 1 : -1;
    if (in && s < 0) {  // the run began in an earlier wave
        s = i0;
        while (s > 0 && i - s <= RUN_MAX && ek[s - 1] == e) --s;
    }
    if (in && t < 0) {  // it continues past this wave
        t = i0 + 64;
        while (t < n && t - s <= RUN_MAX && ek[t] == e) ++t;
    }
    const bool lng = in && t - s > RUN_MAX;
    if (lng) atomicOr(long_run, 1);
    const bool multi = in && !lng && t - s > 1;
    const int64_t my = multi ? sub[me] : 0;
    int64_t rank = 0;
    int span = multi ? (int)(t - s) : 0;
    for (int o = 32; o > 0; o >>= 1) span = max(span, __shfl_xor(span, o));
    for (int d = 1; d < span; ++d) {
        const int64_t fw = __shfl(my, min(lane + d, 63));
        const int64_t bw = __shfl(my, max(lane - d, 0));
        if (!multi) continue;
        if (i + d < t) rank += (lane + d < 64 ? fw : sub[ix[i + d]]) < my;
        if (i - d >= s) rank += (lane - d >= 0 ? bw : sub[ix[i - d]]) <= my;
    }
    if (!in || lng) return;
    const int64_t f = multi ? s + rank : i;
#pragma unroll
    for (int c = 0; c < GATHER_MAX_COLS; ++c)
        if (c < ncol) cs.dst[c][f] = x[c];
    if (seq_dst) seq_dst[f] = emit_base + (int64_t)e;
}

// every column of a record through one index read: dst[c][i] = src[c][perm[i]]. Blocks are mapped XCD-contiguous
// (kernels.h xcd_block): consecutive output records come from a few hundred emission streams (the matcher's blocks),
// each read forward, so one XCD's slice of the output keeps those streams' lines in its own L2
__global__ __launch_bounds__(256) void gather_rows_k(ColSet cs, int ncol, const uint32_t* __restrict__ perm, int64_t n,
                                                     uint32_t xcds) {
    const uint32_t v = xcd_block(blockIdx.x, gridDim.x, xcds);
    const int64_t i = (int64_t)v * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = perm[i];
    int64_t x[GATHER_MAX_COLS];
#pragma unroll
    for (int c = 0; c < GATHER_MAX_COLS; ++c)
        if (c < ncol) x[c] = cs.src[c][p];
#pragma unroll
    for (int c = 0; c < GATHER_MAX_COLS; ++c)
        if (c < ncol) cs.dst[c][i] = x[c];
}

// the sort by the emitting event: RADIX_BITS per onesweep pass (the flush's positions need ~27 bits: 3 passes of 9
// instead of 4 of rocPRIM's default 8)
#ifndef SDG_ORDER_RADIX_BITS
#define SDG_ORDER_RADIX_BITS 9
#endif
// onesweep blocks of 1024 threads x 8 keys: export 2.52 -> 2.29 ms per 40M records against 512 x 16 (r5os2 same box;
// 256 x 16: 3.16, 512 x 8: 2.78, 512 x 24: 2.81, 1024 x 12: 2.51, 1024 x 16: 2.53 ms)
#ifndef SDG_ORDER_BLOCK
#define SDG_ORDER_BLOCK 1024
#endif
#ifndef SDG_ORDER_IPT
#define SDG_ORDER_IPT 8
#endif
using EkSortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<SDG_ORDER_BLOCK, SDG_ORDER_IPT>,
                                        rocprim::kernel_config<SDG_ORDER_BLOCK, SDG_ORDER_IPT>,
                                        SDG_ORDER_RADIX_BITS, rocprim::block_radix_rank_algorithm::match>>;

void temp_sizes(int64_t n, size_t& a, size_t& b) {
    uint64_t* k64 = nullptr;
    uint32_t* k32 = nullptr;
    uint32_t* v = nullptr;
    a = b = 0;
    size_t c = 0;
    rocprim::radix_sort_pairs(nullptr, a, k64, k64, v, v, (size_t)n, 0, 64);
    rocprim::radix_sort_pairs(nullptr, b, k32, k32, v, v, (size_t)n, 0, 32);
    rocprim::radix_sort_pairs<EkSortCfg>(nullptr, c, k32, k32, v, v, (size_t)n, 0, 32);
    b = std::max(b, c);
}

int bits_for(unsigned long long v) {  // bits to hold 0..v
    int b = 0;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

}  // namespace

size_t order_workspace(int64_t n) {
    size_t a = 0, b = 0;
    temp_sizes(n, a, b);
    const size_t sort_tmp = ((a > b ? a : b) + 255) & ~size_t(255);
    // keys: sub (2 x 8n) + emit (2 x 4n), index (2 x 4n), the range (3 x 8)
    return sort_tmp + (size_t)n * (16 + 8 + 8) + 1024;
}

void order_records(const int64_t* emit, const int64_t* sub, int64_t n, int64_t emit_base, int64_t emit_span,
                   int64_t sub_bias, int sub_bits, void* work, size_t work_bytes, uint32_t** perm_out, hipStream_t stream) {
    if (n <= 0) return;
    size_t a = 0, b = 0;
    temp_sizes(n, a, b);
    size_t sort_tmp = ((a > b ? a : b) + 255) & ~size_t(255);
    uint8_t* p = (uint8_t*)work;
    void* tmp = p;
    p += sort_tmp;
    uint64_t* sk0 = (uint64_t*)p; p += (size_t)n * 8;
    uint64_t* sk1 = (uint64_t*)p; p += (size_t)n * 8;
    uint32_t* ek0 = (uint32_t*)p; p += (size_t)n * 4;
    uint32_t* ek1 = (uint32_t*)p; p += (size_t)n * 4;
    uint32_t* ix0 = (uint32_t*)p; p += (size_t)n * 4;
    uint32_t* ix1 = (uint32_t*)p; p += (size_t)n * 4;
    unsigned long long* rng = (unsigned long long*)p;
    (void)work_bytes;
    const unsigned grid = (unsigned)((n + 255) / 256);
    // the keys' actual ranges (one small read-back): both sorts cover only the bits the flush's records use --
    // an e1 position / ordinal spans ~30 bits, not the 48 or 64 of its encoding, and then fits a 32-bit key
    static const bool full = getenv("SDG_ORDER_FULL") != nullptr;  // A/B: the fixed-width sorts
    static const bool two = getenv("SDG_ORDER_TWO") != nullptr;    // A/B: always the two sorts
    int eb = 32, sb = sub_bits;
    unsigned long long smin = 0;
    // one sort by the emitting event, then each run of one event's records put in ordinal order (order_runs_k);
    // runs longer than RUN_MAX (an event that completed hundreds of partials) take the two-sort ordering below.
    // The emitting events lie in the flush's positions, so that sort needs no range pass
    if (!full && !two && emit_span > 0) {
        eb = std::max(1, bits_for((unsigned long long)(emit_span - 1)));
        hipLaunchKernelGGL(order_emit_keys_k, dim3(grid), dim3(256), 0, stream, emit, n, emit_base, ek0, ix0);
        static const bool dflt = getenv("SDG_ORDER_DEFAULT_CFG") != nullptr;  // A/B: rocPRIM's default digits
        if (dflt) rocprim::radix_sort_pairs(tmp, b, ek0, ek1, ix0, ix1, (size_t)n, 0, eb, stream);
        else rocprim::radix_sort_pairs<EkSortCfg>(tmp, b, ek0, ek1, ix0, ix1, (size_t)n, 0, eb, stream);
        int* flag = (int*)(rng + 3);
        (void)hipMemsetAsync(flag, 0, 4, stream);
        static const bool serial_runs = getenv("SDG_ORDER_SERIAL_RUNS") != nullptr;  // A/B: order_runs_k
        if (serial_runs) hipLaunchKernelGGL(order_runs_k, dim3(grid), dim3(256), 0, stream, ek1, ix1, sub, n, flag);
        else hipLaunchKernelGGL(order_runs_rank_k, dim3(grid), dim3(256), 0, stream, ek1, ix1, sub, n, ix0, flag);
        int hf = 0;
        (void)hipMemcpyAsync(&hf, flag, 4, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        if (!hf) {
            *perm_out = serial_runs ? ix1 : ix0;
            return;
        }
    }
    if (!full) {
        const unsigned long long init[3] = {0ull, ~0ull, 0ull};
        (void)hipMemcpyAsync(rng, init, sizeof init, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(order_range_k, dim3((unsigned)std::min<int64_t>(grid, 2048)), dim3(256), 0, stream, emit, sub, n,
                           emit_base, sub_bias, rng);
        unsigned long long h[3];
        (void)hipMemcpyAsync(h, rng, sizeof h, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        eb = std::max(1, bits_for(h[0]));
        smin = h[1];
        sb = std::max(1, bits_for(h[2] - h[1]));
    }
    uint32_t* perm1 = nullptr;
    if (!full && sb <= 32) {  // the ordinal as a 32-bit key relative to its minimum
        uint32_t* s32a = (uint32_t*)sk0;
        uint32_t* s32b = (uint32_t*)sk1;
        hipLaunchKernelGGL(order_keys_k<uint32_t>, dim3(grid), dim3(256), 0, stream, emit, sub, n, emit_base,
                           sub_bias + (int64_t)smin, ek0, s32a, ix0);
        rocprim::radix_sort_pairs(tmp, b, s32a, s32b, ix0, ix1, (size_t)n, 0, sb, stream);
    } else {
        hipLaunchKernelGGL(order_keys_k<uint64_t>, dim3(grid), dim3(256), 0, stream, emit, sub, n, emit_base,
                           sub_bias + (int64_t)smin, ek0, sk0, ix0);
        rocprim::radix_sort_pairs(tmp, a, sk0, sk1, ix0, ix1, (size_t)n, 0, full ? sub_bits : sb, stream);
    }
    perm1 = ix1;
    // then (stable) by the emitting event
    hipLaunchKernelGGL(gather_k<uint32_t>, dim3(grid), dim3(256), 0, stream, ek0, perm1, n, ek1);
    rocprim::radix_sort_pairs(tmp, b, ek1, ek0, perm1, ix0, (size_t)n, 0, eb, stream);
    *perm_out = ix0;
}

bool order_export(const int64_t* emit, const int64_t* sub, int64_t n, int64_t emit_base, int64_t emit_span,
                  const int64_t* const* src, int64_t* const* dst, int ncol, int64_t* seq_dst, void* work,
                  hipStream_t stream) {
    if (n <= 0) return true;
    if (emit_span <= 0 || ncol > GATHER_MAX_COLS) return false;
    size_t a = 0, b = 0;
    temp_sizes(n, a, b);
    const size_t sort_tmp = ((a > b ? a : b) + 255) & ~size_t(255);
    uint8_t* p = (uint8_t*)work;
    void* tmp = p;
    p += sort_tmp;
    p += (size_t)n * 16;  // (order_records' 64-bit key buffers: unused here)
    uint32_t* ek0 = (uint32_t*)p; p += (size_t)n * 4;
    uint32_t* ek1 = (uint32_t*)p; p += (size_t)n * 4;
    uint32_t* ix0 = (uint32_t*)p; p += (size_t)n * 4;
    uint32_t* ix1 = (uint32_t*)p; p += (size_t)n * 4;
    int* flag = (int*)p;
    const unsigned grid = (unsigned)((n + 255) / 256);
    const int eb = std::max(1, bits_for((unsigned long long)(emit_span - 1)));
    hipLaunchKernelGGL(order_emit_keys_k, dim3(grid), dim3(256), 0, stream, emit, n, emit_base, ek0, ix0);
    rocprim::radix_sort_pairs<EkSortCfg>(tmp, b, ek0, ek1, ix0, ix1, (size_t)n, 0, eb, stream);
    (void)hipMemsetAsync(flag, 0, 4, stream);
    ColSet cs{};
    for (int c = 0; c < ncol; ++c) {
        cs.src[c] = src[c];
        cs.dst[c] = dst[c];
    }
    const unsigned g8 = (unsigned)xcd_round(grid);
    static const bool scan_runs = getenv("SDG_ORDER_SCAN_RUNS") != nullptr;  // A/B: per-thread HBM run scans
    if (scan_runs)
        hipLaunchKernelGGL(order_runs_gather_k, dim3(g8), dim3(256), 0, stream, ek1, ix1, sub, n, cs, ncol, seq_dst,
                           emit_base, flag, (uint32_t)g_xcds);
    else
        hipLaunchKernelGGL(order_runs_gather_w_k, dim3((unsigned)xcd_round((n + OG_T - 1) / OG_T)), dim3(OG_T), 0, stream,
                           ek1, ix1, sub, n, cs, ncol, seq_dst,
                           emit_base, flag, (uint32_t)g_xcds);
    int hf = 0;
    (void)hipMemcpyAsync(&hf, flag, 4, hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    return hf == 0;  // false: a run longer than RUN_MAX. The short runs' records are ALREADY written to dst /
                     // seq_dst; the caller's fallback (order_records) overwrites all n slots
}

size_t gather_cols_workspace(int64_t n, int ncol) { return (size_t)std::max<int64_t>(n, 1) * ncol * 8 + 256; }

void gather_cols_i64(const int64_t* const* src, int64_t* const* dst, int ncol, const uint32_t* perm, int64_t n,
                     void* work, hipStream_t stream) {
    if (n <= 0 || ncol <= 0) return;
    static const bool cols = getenv("SDG_GATHER_COLS") != nullptr;  // A/B: one random-read gather per column
    static const bool packed = getenv("SDG_GATHER_PACKED") != nullptr;  // A/B: pack_k + unpack_k (round 4)
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (!cols && !packed) {  // one pass, every column of a record per thread, XCD-contiguous output slices
        const unsigned g8 = (unsigned)xcd_round(grid);
        for (int c0 = 0; c0 < ncol; c0 += GATHER_MAX_COLS) {
            const int nc = std::min(GATHER_MAX_COLS, ncol - c0);
            ColSet cs{};
            for (int c = 0; c < nc; ++c) {
                cs.src[c] = src[c0 + c];
                cs.dst[c] = dst[c0 + c];
            }
            hipLaunchKernelGGL(gather_rows_k, dim3(g8), dim3(256), 0, stream, cs, nc, perm, n, (uint32_t)g_xcds);
        }
        return;
    }
    if (cols || ncol == 1) {
        for (int c = 0; c < ncol; ++c) hipLaunchKernelGGL(gather_k<int64_t>, dim3(grid), dim3(256), 0, stream, src[c], perm, n, dst[c]);
        return;
    }
    for (int c0 = 0; c0 < ncol; c0 += GATHER_MAX_COLS) {
        const int nc = std::min(GATHER_MAX_COLS, ncol - c0);
        ColSet cs{};
        for (int c = 0; c < nc; ++c) {
            cs.src[c] = src[c0 + c];
            cs.dst[c] = dst[c0 + c];
        }
        int64_t* rec = (int64_t*)work;
        hipLaunchKernelGGL(pack_k, dim3(grid), dim3(256), 0, stream, cs, nc, n, rec);
        hipLaunchKernelGGL(unpack_k, dim3(grid), dim3(256), 0, stream, cs, nc, (const int64_t*)rec, perm, n);
    }
}

void gather_i64(const int64_t* src, const uint32_t* perm, int64_t n, int64_t* dst, hipStream_t stream) {
    if (n > 0) hipLaunchKernelGGL(gather_k<int64_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, src, perm, n, dst);
}
void gather_u32(const uint32_t* src, const uint32_t* perm, int64_t n, uint32_t* dst, hipStream_t stream) {
    if (n > 0) hipLaunchKernelGGL(gather_k<uint32_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, src, perm, n, dst);
}
void gather_u8(const uint8_t* src, const uint32_t* perm, int64_t n, uint8_t* dst, hipStream_t stream) {
    if (n > 0) hipLaunchKernelGGL(gather_k<uint8_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, src, perm, n, dst);
}

// ---- the selector's post pass (QuerySelector.processNoGroupBy :161-205 for aggregators and having) ------------
// Records arrive in delivery order. Attribute aggregators keep their state per partition key and see that key's
// records in delivery order, so the records are stably sorted by key (a record index, rocPRIM) and one lane walks
// each key's run sequentially -- float sums must add in the reference's order to be bit-exact. Per record: the
// aggregators (arguments were evaluated at emission into hidden columns), then the select items over them, then
// the having condition.
namespace {

__device__ __forceinline__ double as_f64(int64_t v, uint8_t k) {
    return k == VK_I32 ? (double)(int32_t)v : k == VK_I64 ? (double)v : k == VK_F32 ? (double)bits_f32(v) : bits_f64(v);
}

// state per (key, aggregator): {count, value}; value = long sum | double sum bits | min/max payload
__device__ __forceinline__ void agg_step(const AggSpec& g, int64_t* st, int64_t arg, bool arg_null, int64_t* out,
                                         bool* out_null) {
    int64_t& cnt = st[0];
    int64_t& v = st[1];
    switch (g.kind) {
        case AG_COUNT:  // CountAttributeAggregatorExecutor.processAdd
            ++cnt;
            *out = cnt;
            *out_null = false;
            return;
        case AG_SUM:  // SumAttributeAggregatorExecutor: Int -> Long state, Float -> Double state; null -> currentValue
            if (!arg_null) {
                if (g.out_kind == VK_I64) v = (int64_t)((uint64_t)v + (uint64_t)(g.arg_kind == VK_I32 ? (int64_t)(int32_t)arg : arg));
                else v = f64_bits(bits_f64(v) + as_f64(arg, g.arg_kind));
                ++cnt;
            }
            *out = v;
            *out_null = cnt == 0;
            return;
        case AG_AVG: {  // AvgAttributeAggregatorExecutor: double value / long count
            if (!arg_null) {
                ++cnt;
                v = f64_bits(bits_f64(v) + as_f64(arg, g.arg_kind));
            }
            *out = f64_bits(bits_f64(v) / (double)cnt);
            *out_null = cnt == 0;
            return;
        }
        default: {  // Min/MaxAttributeAggregatorExecutor: minValue == null || minValue > value
            if (!arg_null) {
                bool take = cnt == 0;
                if (!take) {
                    const bool mn = g.kind == AG_MIN;
                    switch (g.arg_kind) {
                        case VK_I32: take = mn ? (int32_t)v > (int32_t)arg : (int32_t)v < (int32_t)arg; break;
                        case VK_I64: take = mn ? v > arg : v < arg; break;
                        case VK_F32: take = mn ? bits_f32(v) > bits_f32(arg) : bits_f32(v) < bits_f32(arg); break;
                        default: take = mn ? bits_f64(v) > bits_f64(arg) : bits_f64(v) < bits_f64(arg); break;
                    }
                }
                if (take) {
                    v = arg;
                    cnt = 1;
                }
            }
            *out = v;
            *out_null = cnt == 0;
            return;
        }
    }
}

// the post pass's view of one record: its columns, and its key's aggregator states
struct PostAcc {
    const Plan* P;
    const int64_t* vals;
    int64_t vstride;
    int64_t i;
    uint32_t nm;
    int64_t* st;
    __device__ void load(int, int col, int, uint8_t, int64_t* v, bool* null) {
        *v = vals[(int64_t)col * vstride + i];
        *null = (nm >> col) & 1u;
    }
    __device__ bool slot_empty(int, int) { return false; }
    __device__ void agg(int g, int64_t* v, bool* n) {
        const AggSpec& s = P->agg[g];
        int64_t arg = 0;
        bool an = true;
        if (s.arg_col >= 0) {
            arg = vals[(int64_t)s.arg_col * vstride + i];
            an = (nm >> s.arg_col) & 1u;
        }
        agg_step(s, st + 2 * g, arg, an, v, n);
    }
};

__global__ __launch_bounds__(256) void sel_post_k(SelPostArgs a) {
    __shared__ int64_t stk_mem[STACK * 256];
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= a.n) return;
    const uint32_t k = a.key_sorted ? a.key_sorted[p] : 0u;
    if (p > 0 && a.key_sorted && a.key_sorted[p - 1] == k) return;  // not the head of its key's run
    if (p > 0 && !a.key_sorted) return;                               // one run: lane 0
    const Plan* P = a.plan;
    const int na = P->n_agg;
    int64_t* st = a.agg_state + (int64_t)k * na * 2;
    int64_t* stk = stk_mem + threadIdx.x;
    for (int64_t q = p; q < a.n && (!a.key_sorted || a.key_sorted[q] == k); ++q) {
        const int64_t i = a.perm ? (int64_t)a.perm[q] : q;
        if (a.reset && a.reset[i])  // @purge destroyed the key's aggregator states before this record
            for (int g = 0; g < 2 * na; ++g) st[g] = 0;
        const uint32_t nm0 = a.nulls[i];
        PostAcc acc{P, a.vals, a.vstride, i, nm0, st};
        for (int j = 0; j < P->n_user_out; ++j) {  // select items over aggregators, in order, then having
            if (!P->out_post[j]) continue;
            int64_t v;
            bool nl;
            run(a.code, P->post_prog[j], a.consts, acc, stk, 256, &v, &nl);
            a.vals[(int64_t)j * a.vstride + i] = v;
            acc.nm = nl ? (acc.nm | (1u << j)) : (acc.nm & ~(1u << j));
        }
        a.nulls[i] = acc.nm;
        a.pass[i] = P->having.len == 0 ? 1 : (uint8_t)pass(a.code, P->having, a.consts, acc, stk, 256);
    }
}

// keys purged after their last record of the flush: their aggregator states restart (zero = fresh)
__global__ __launch_bounds__(256) void agg_reset_k(int64_t* __restrict__ st, int na, uint8_t* __restrict__ flag, int64_t K) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K || !flag[k]) return;
    for (int g = 0; g < 2 * na; ++g) st[k * 2 * na + g] = 0;
    flag[k] = 0;
}

__global__ __launch_bounds__(256) void iota_k(uint32_t* __restrict__ x, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = (uint32_t)i;
}

}  // namespace

size_t select_post_workspace(int64_t n) {
    size_t t = 0;
    uint32_t* k = nullptr;
    rocprim::radix_sort_pairs(nullptr, t, k, k, k, k, (size_t)n, 0, 32);
    return ((t + 255) & ~size_t(255)) + (size_t)n * 12 + 1024;
}

void select_post(SelPostArgs a, const uint32_t* key, int kbits, void* work, hipStream_t stream) {
    if (a.n <= 0) return;
    const unsigned grid = (unsigned)((a.n + 255) / 256);
    a.perm = nullptr;
    a.key_sorted = nullptr;
    if (key && kbits > 0) {  // stable sort of the record index by key: each key's records stay in delivery order
        size_t t = 0;
        uint32_t* kk = nullptr;
        rocprim::radix_sort_pairs(nullptr, t, kk, kk, kk, kk, (size_t)a.n, 0, kbits);
        uint8_t* p = (uint8_t*)work;
        void* tmp = p;
        p += (t + 255) & ~size_t(255);
        uint32_t* ks = (uint32_t*)p; p += (size_t)a.n * 4;
        uint32_t* ix0 = (uint32_t*)p; p += (size_t)a.n * 4;
        uint32_t* ix1 = (uint32_t*)p;
        hipLaunchKernelGGL(iota_k, dim3(grid), dim3(256), 0, stream, ix0, a.n);
        rocprim::radix_sort_pairs(tmp, t, key, ks, ix0, ix1, (size_t)a.n, 0, kbits, stream);
        a.perm = ix1;
        a.key_sorted = ks;
    }
    hipLaunchKernelGGL(sel_post_k, dim3(a.key_sorted ? grid : 1u), dim3(256), 0, stream, a);
}

void agg_reset(int64_t* agg_state, int n_agg, uint8_t* flags, int64_t K, hipStream_t stream) {
    if (K > 0) hipLaunchKernelGGL(agg_reset_k, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, agg_state,
                                  n_agg > 0 ? n_agg : 1, flags, K);
}

}  // namespace sdg
