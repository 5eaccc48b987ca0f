// gfx950 kernels of the pattern/sequence path: key grouping and the chain matcher.
//
// Wave64 throughout: ballots are 64-bit, lane masks use __lanemask_lt(), compaction is ballot + mbcnt with one
// atomic per wave. Everything is integer/byte work bound by HBM, so no MFMA.
#include <hip/hip_runtime.h>

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
// key grouping

__global__ __launch_bounds__(256) void kg_hist(const uint32_t* __restrict__ keys, int64_t n, int K,
                                               uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t h[];
    for (int k = threadIdx.x; k < K; k += blockDim.x) h[k] = 0;
    __syncthreads();
    int64_t s = (int64_t)blockIdx.x * KG_CHUNK;
    int64_t e = s + KG_CHUNK < n ? s + KG_CHUNK : n;
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) atomicAdd(&h[keys[i]], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < K; k += blockDim.x) counts[(int64_t)blockIdx.x * K + k] = h[k];
}

// group sums over KG_GROUP chunks: thread (g, k)
__global__ __launch_bounds__(256) void kg_p1(const uint32_t* __restrict__ counts, int nchunks, int K,
                                             uint32_t* __restrict__ gsum) {
    int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int ng = (nchunks + KG_GROUP - 1) / KG_GROUP;
    if (idx >= (int64_t)ng * K) return;
    int g = (int)(idx / K), k = (int)(idx % K);
    int b0 = g * KG_GROUP, b1 = min(nchunks, b0 + KG_GROUP);
    uint32_t s = 0;
    for (int b = b0; b < b1; ++b) s += counts[(int64_t)b * K + k];
    gsum[idx] = s;
}

// per key: exclusive scan over groups (in place); totals to tot[k]
__global__ __launch_bounds__(256) void kg_p2(uint32_t* __restrict__ gsum, int ng, int K, uint32_t* __restrict__ tot) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    uint32_t run = 0;
    for (int g = 0; g < ng; ++g) {
        uint32_t c = gsum[(int64_t)g * K + k];
        gsum[(int64_t)g * K + k] = run;
        run += c;
    }
    tot[k] = run;
}

// exclusive scan of tot[0..K) in place (K <= KG_MAXK), one 1024-thread block; tot[K] = n
__global__ __launch_bounds__(1024) void kg_kscan(uint32_t* __restrict__ tot, int K, int64_t n) {
    __shared__ uint32_t part[1024];
    constexpr int PER = KG_MAXK / 1024;
    int t = threadIdx.x;
    uint32_t v[PER];
    uint32_t s = 0;
    for (int j = 0; j < PER; ++j) {
        int k = t * PER + j;
        v[j] = k < K ? tot[k] : 0;
        s += v[j];
    }
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
        uint32_t x = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (int j = 0; j < PER; ++j) {
        int k = t * PER + j;
        if (k < K) tot[k] = run;
        run += v[j];
    }
    if (t == 0) tot[K] = (uint32_t)n;
}

// per (group, key): rewrite the group's chunk counts as absolute start offsets
__global__ __launch_bounds__(256) void kg_p3(uint32_t* __restrict__ counts, const uint32_t* __restrict__ gsum,
                                             const uint32_t* __restrict__ seg_start, int nchunks, int K) {
    int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int ng = (nchunks + KG_GROUP - 1) / KG_GROUP;
    if (idx >= (int64_t)ng * K) return;
    int g = (int)(idx / K), k = (int)(idx % K);
    uint32_t run = seg_start[k] + gsum[idx];
    int b0 = g * KG_GROUP, b1 = min(nchunks, b0 + KG_GROUP);
    for (int b = b0; b < b1; ++b) {
        uint32_t c = counts[(int64_t)b * K + k];
        counts[(int64_t)b * K + k] = run;
        run += c;
    }
}

// stable scatter: one wave per chunk, LDS cursor per key; equal keys inside one wave step are ranked by a
// ballot match over the key bits (lane order == arrival order).
__global__ __launch_bounds__(64) void kg_scatter(KeyGroupArgs a, int kbits) {
    extern __shared__ uint32_t cur[];
    const int K = a.K;
    const int lane = threadIdx.x;
    for (int k = lane; k < K; k += 64) cur[k] = a.counts[(int64_t)blockIdx.x * K + k];
    __syncthreads();
    int64_t s = (int64_t)blockIdx.x * KG_CHUNK;
    int64_t e = s + KG_CHUNK < a.n ? s + KG_CHUNK : a.n;
    const uint64_t lt = lanemask_lt();
    for (int64_t base = s; base < e; base += 64) {
        int64_t i = base + lane;
        bool valid = i < e;
        uint32_t k = valid ? a.keys[i] : 0u;
        uint64_t peers = __ballot(valid);
        for (int bit = 0; bit < kbits; ++bit) {
            bool on = (k >> bit) & 1u;
            uint64_t b = __ballot(on);
            peers &= on ? b : ~b;
        }
        int leader = peers ? __ffsll((unsigned long long)peers) - 1 : lane;
        uint32_t kb = 0;
        if (valid && lane == leader) {
            kb = cur[k];
            cur[k] = kb + (uint32_t)__popcll(peers);
        }
        kb = __shfl(kb, leader);
        if (valid) {
            uint32_t dest = kb + (uint32_t)__popcll(peers & lt);
            a.keys_sorted[dest] = k;
            a.orig_sorted[dest] = (uint32_t)i;
            for (int c = 0; c < a.ncols; ++c) {
                switch (a.width[c]) {
                    case 8: ((int64_t*)a.dst[c])[dest] = ((const int64_t*)a.src[c])[i]; break;
                    case 4: ((uint32_t*)a.dst[c])[dest] = ((const uint32_t*)a.src[c])[i]; break;
                    default: ((uint8_t*)a.dst[c])[dest] = ((const uint8_t*)a.src[c])[i]; break;
                }
            }
        }
    }
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
            if (pass(a.code, c1, a.consts, acc, stk, stride)) return q;
            acc.r1 = -1;
        }
    }
    return -2;
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
        run(a.code, P->out_prog[j], a.consts, acc, stk, stride, &v, &nl);
        a.out_vals[(int64_t)j * a.out_cap + slot] = v;
        if (nl) nm |= 1u << j;
    }
    a.out_nulls[slot] = nm;
}

__global__ __launch_bounds__(256) void chain_match_k(ChainArgs a) {
    __shared__ int64_t stack_mem[STACK * 256];
    int64_t* stk = stack_mem + threadIdx.x;
    const int stride = 256;
    const Plan* P = a.plan;
    int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool active = p < a.n;
    bool has = false, carry = false;
    int64_t qhit = -1;
    ChainAcc acc{&a, p, -1, -1};
    uint32_t key = 0;
    if (active) {
        key = a.key ? a.key[p] : 0u;
        if (p > 0 && a.ts[p] < a.ts[p - 1] && (!a.key || a.key[p - 1] == key)) atomicOr(&a.flags[1], 1);
        if (qstream_of(a, p) == a.s0 && pass(a.code, P->st[0].filter, a.consts, acc, stk, stride)) {
            if (P->n_states == 1) {
                has = true;
                qhit = p;
            } else {
                int64_t end = a.key ? (int64_t)a.seg_start[key + 1] : a.n;
                int64_t r = chain_scan(a, acc, p + 1, end, a.ts[p], stk, stride);
                if (r >= 0) { has = true; qhit = r; }
                else if (r == -2) carry = true;
            }
        }
    }
    int64_t slot = wave_reserve(has, a.out_count);
    if (has) {
        if (slot >= a.out_cap) atomicOr(&a.flags[0], 1);
        else emit_match(a, acc, slot, qhit, key, a.seq_base + (a.orig ? (int64_t)a.orig[p] : p), stk, stride);
    }
    int64_t cs = wave_reserve(carry, a.carry_count);
    if (carry) {
        if (cs >= a.carry_cap) {
            atomicOr(&a.flags[0], 1);
        } else {
            a.carry_key[cs] = key;
            a.carry_ts[cs] = a.ts[p];
            a.carry_seq[cs] = a.seq_base + (a.orig ? (int64_t)a.orig[p] : p);
            uint32_t nm = 0;
            for (int c = 0; c < P->n_cols; ++c) {
                a.carry_vals[(int64_t)c * a.carry_cap + cs] = load_col(a.cols[c], P->col_kind[c], p);
                if (a.nulls[c] && a.nulls[c][p]) nm |= 1u << c;
            }
            a.carry_nulls[cs] = nm;
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
        int64_t b = a.key ? (int64_t)a.seg_start[key] : 0;
        int64_t e = a.key ? (int64_t)a.seg_start[key + 1] : a.n;
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

}  // namespace

size_t keygroup_workspace(int64_t n, int32_t K, int32_t* nchunks, size_t* counts_bytes, size_t* gsum_bytes) {
    int32_t nc = (int32_t)((n + KG_CHUNK - 1) / KG_CHUNK);
    if (nc < 1) nc = 1;
    int32_t ng = (nc + KG_GROUP - 1) / KG_GROUP;
    *nchunks = nc;
    *counts_bytes = (size_t)nc * K * 4;
    *gsum_bytes = (size_t)ng * K * 4;
    return *counts_bytes + *gsum_bytes;
}

void keygroup(const KeyGroupArgs& a, hipStream_t stream, hipEvent_t* marks) {
    const int K = a.K;
    const int nc = a.nchunks;
    const int ng = (nc + KG_GROUP - 1) / KG_GROUP;
    int kbits = 0;
    while ((1 << kbits) < K) ++kbits;
    if (marks) (void)hipEventRecord(marks[0], stream);
    hipLaunchKernelGGL(kg_hist, dim3(nc), dim3(256), K * 4, stream, a.keys, a.n, K, a.counts);
    if (marks) (void)hipEventRecord(marks[1], stream);
    int64_t gk = (int64_t)ng * K;
    hipLaunchKernelGGL(kg_p1, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, nc, K, a.gsum);
    hipLaunchKernelGGL(kg_p2, dim3((K + 255) / 256), dim3(256), 0, stream, a.gsum, ng, K, a.seg_start);
    hipLaunchKernelGGL(kg_kscan, dim3(1), dim3(1024), 0, stream, a.seg_start, K, a.n);
    hipLaunchKernelGGL(kg_p3, dim3((unsigned)((gk + 255) / 256)), dim3(256), 0, stream, a.counts, a.gsum,
                       a.seg_start, nc, K);
    if (marks) (void)hipEventRecord(marks[2], stream);
    hipLaunchKernelGGL(kg_scatter, dim3(nc), dim3(64), K * 4, stream, a, kbits);
    if (marks) (void)hipEventRecord(marks[3], stream);
}

void chain_match(const ChainArgs& a, hipStream_t stream) {
    if (a.n <= 0) return;
    hipLaunchKernelGGL(chain_match_k, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, stream, a);
}

void chain_carry(const ChainArgs& a, hipStream_t stream) {
    if (a.cin_n <= 0) return;
    hipLaunchKernelGGL(chain_carry_k, dim3((unsigned)((a.cin_n + 255) / 256)), dim3(256), 0, stream, a);
}

}  // namespace sdg
