// G-way merge of sorted runs on the device: the ordered result gather's merge on rank 0 (the
// reference delivers one ordered stream per input event, StateMultiProcessStreamReceiver.java:47-68,
// StreamCallback.java:93-129). Each rank's export is already a run sorted by its key (sdg_export_ordered), so rank 0
// merges G runs instead of re-sorting their concatenation.
//
// Order: (key, run, index in run) -- equal keys keep run order, then their order inside the run (a stable merge).
// Regular sampling (PSRS) gives every output bucket a hard size bound, so one workgroup merges one bucket in LDS:
//  1. samples: every MG_S-th record of every run, in (run, index) order, keys radix-sorted (rocPRIM, stable: ties
//     stay in (run, index) order = the composite order);
//  2. splitters: every MG_M-th sorted sample. A splitter's position in each run: its own index in its own run, the
//     upper bound of its key in earlier runs, the lower bound in later runs (binary searches, one lane per (splitter,
//     run)). The bucket between two consecutive splitters then holds, from run r, the records between them in the
//     composite order: at most (c_r + 1) * MG_S where c_r samples of run r lie between them, sum c_r <= MG_M, so a
//     bucket holds <= (MG_M + G) * MG_S records;
//  3. one workgroup per bucket: the bucket's key slices into LDS, each record's rank inside the bucket = its index
//     in its slice + its bounds in the other slices (LDS binary searches), then the records leave in output order:
//     keys from LDS, payload columns read from the runs (G nearly sequential streams), all stores contiguous.
// HBM traffic: the keys read once and written once, every payload byte read once and written once, plus the
// samples (1 / MG_S of the keys) and the splitter bounds (G x 4 B per MG_M x MG_S records).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>

#include <rocprim/device/device_radix_sort.hpp>

#include "kernels.h"

namespace sdg {
namespace {

constexpr int MG_S = 128;                              // sample stride (records of one run per sample)
constexpr int MG_M = 16;                               // samples per bucket
constexpr int MG_THREADS = 512;

struct MergeRuns {
    const int64_t* keys[MG_MAX_RUNS];
    const void* cols[MG_MAX_RUNS][MG_MAX_COLS];
    int64_t len[MG_MAX_RUNS];
    int64_t sbase[MG_MAX_RUNS + 1];  // first sample id of each run (run-major)
    void* out_cols[MG_MAX_COLS];
    int64_t* out_keys;
    uint8_t width[MG_MAX_COLS];
    int G;
    int ncols;
    int64_t nsamples;
    int64_t nbuckets;
    int64_t kmin;                    // samples are sorted as key - kmin (u64, non-negative)
    int* flag;                       // set if a bucket broke the sampling bound (never expected)
    int pairwise;                    // buckets whose keys span < 2^32 take the pairwise LDS merge (SDG_MG_PAIR)
};

// the runs' first / last keys (they are sorted: the extremes of the whole input)
__global__ void mg_ends_k(const MergeRuns a, int64_t* __restrict__ ends) {
    const int r = threadIdx.x;
    if (r < a.G && a.len[r] > 0) {
        ends[2 * r] = a.keys[r][0];
        ends[2 * r + 1] = a.keys[r][a.len[r] - 1];
    }
}

// samples: key - kmin and the sample id (run-major ids: the input order of the stable sort)
__global__ __launch_bounds__(256) void mg_samples_k(const MergeRuns a, uint64_t* __restrict__ skey,
                                                    uint32_t* __restrict__ sid) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.nsamples) return;
    int r = 0;
    while (r + 1 < a.G && a.sbase[r + 1] <= i) ++r;
    const int64_t idx = (i - a.sbase[r]) * MG_S;
    skey[i] = (uint64_t)(a.keys[r][idx] - a.kmin);
    sid[i] = (uint32_t)i;
}

// records of run `r` with key < k (lower) or <= k (upper)
__device__ __forceinline__ int64_t mg_bound(const int64_t* __restrict__ keys, int64_t n, int64_t k, bool upper) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int64_t v = keys[mid];
        if (v < k || (upper && v == k)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// bounds[b * G + r]: the first record of run r in bucket b (b = 0: all zero; b = nbuckets: the run lengths)
__global__ __launch_bounds__(256) void mg_bounds_k(const MergeRuns a, const uint32_t* __restrict__ sorted_sid,
                                                   int64_t* __restrict__ bounds) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int G = a.G;
    if (t >= (a.nbuckets + 1) * G) return;
    const int64_t b = t / G;
    const int r = (int)(t - b * G);
    int64_t v;
    if (b == 0) {
        v = 0;
    } else if (b == a.nbuckets) {
        v = a.len[r];
    } else {
        const uint32_t s = sorted_sid[b * MG_M];  // the splitter: a sample (run rs, index is)
        int rs = 0;
        while (rs + 1 < G && a.sbase[rs + 1] <= (int64_t)s) ++rs;
        const int64_t is = ((int64_t)s - a.sbase[rs]) * MG_S;
        if (r == rs) v = is;
        else v = mg_bound(a.keys[r], a.len[r], a.keys[rs][is], r < rs);
    }
    bounds[t] = v;
}

// the payload of a bucket's records in output order, one column (width W) at a time: each lane gathers up to 4 records
// (issued together, then stored: the loads of one batch never wait for its stores)
template <int W, int GMAX>
__device__ __forceinline__ void mg_out_col(const void* const* __restrict__ src, void* __restrict__ dst, int64_t off,
                                          int L, const uint16_t* s_src, const uint8_t* s_run, const int64_t* s_start,
                                          const int* s_pre) {
    using U = typename std::conditional<W == 8, uint64_t, typename std::conditional<W == 4, uint32_t,
                                        typename std::conditional<W == 2, uint16_t, uint8_t>::type>::type>::type;
    constexpr int B = 4;
    for (int p0 = threadIdx.x; p0 < L; p0 += B * MG_THREADS) {
        U v[B];
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const int p = p0 + k * MG_THREADS;
            if (p < L) {
                const int i = s_src[p];
                const int r = s_run[i];
                v[k] = ((const U*)src[r])[s_start[r] + (i - s_pre[r])];
            }
        }
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const int p = p0 + k * MG_THREADS;
            if (p < L) ((U*)dst)[off + p] = v[k];
        }
    }
}

// payload columns in output order: one column at a time, its runs' pointers in LDS
template <int GMAX>
__device__ __forceinline__ void mg_out_cols(const MergeRuns& a, int t, int G, int64_t off, int L, const void** s_ptr,
                                            const uint16_t* s_src, const uint8_t* s_run, const int64_t* s_start,
                                            const int* s_pre) {
    for (int c = 0; c < a.ncols; ++c) {
        __syncthreads();  // (s_ptr is rewritten per column)
        if (t < G) s_ptr[t] = a.cols[t][c];
        __syncthreads();
        switch (a.width[c]) {
            case 8: mg_out_col<8, GMAX>(s_ptr, a.out_cols[c], off, L, s_src, s_run, s_start, s_pre); break;
            case 4: mg_out_col<4, GMAX>(s_ptr, a.out_cols[c], off, L, s_src, s_run, s_start, s_pre); break;
            case 2: mg_out_col<2, GMAX>(s_ptr, a.out_cols[c], off, L, s_src, s_run, s_start, s_pre); break;
            default: mg_out_col<1, GMAX>(s_ptr, a.out_cols[c], off, L, s_src, s_run, s_start, s_pre); break;
        }
    }
}

// the bucket's G sorted slices merged pairwise in LDS (slices r and r + w, then 2w, ...: log2(G) rounds; the lower
// run first on equal keys, so the merge is stable in (key, run, index)), each round by merge paths: every lane
// produces E consecutive outputs of its pair after one co-rank binary search. Keys as u32 offsets from kmin (the
// int64 keys in s_key are rewritten in place: its bytes hold the two u32 key buffers); s_src / s_src2 the LDS slot
// each output came from. Leaves the merged offsets at the front of s_key and the slots in s_src.
template <int GMAX, int CAP>
__device__ __forceinline__ void mg_pairwise(int L, int G, int64_t* s_key, uint16_t* s_src, uint16_t* s_src2,
                                            const int* s_pre, int64_t kmin) {
    constexpr int E = (CAP + MG_THREADS - 1) / MG_THREADS;
    const int t = threadIdx.x;
    uint32_t* ka = reinterpret_cast<uint32_t*>(s_key);
    uint32_t* kb = ka + CAP;
    // int64 -> u32 offsets (in registers first: the u32 buffers overlay the int64 keys)
    uint32_t kv[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
        const int i = t + k * MG_THREADS;
        kv[k] = i < L ? (uint32_t)(s_key[i] - kmin) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < E; ++k) {
        const int i = t + k * MG_THREADS;
        if (i < L) {
            ka[i] = kv[k];
            s_src[i] = (uint16_t)i;
        }
    }
    __syncthreads();
    int gp = 1;
    while (gp < G) gp <<= 1;
    uint32_t *ks = ka, *kd = kb;
    uint16_t *is = s_src, *id = s_src2;
    for (int w = 1; w < gp; w <<= 1) {
        // lane t: outputs [t E, t E + E); the pair (r, r + w) with r a multiple of 2w holding them
        int p = t * E;
        const int pe = min(p + E, L);
        while (p < pe) {
            int r = 0;
            while (r + 2 * w < gp && s_pre[min(r + 2 * w, G)] <= p) r += 2 * w;
            const int a0 = s_pre[min(r, G)], a1 = s_pre[min(r + w, G)], a2 = s_pre[min(r + 2 * w, G)];
            const int na = a1 - a0, nb = a2 - a1, q = p - a0;
            // co-rank: i elements of A and q - i of B precede output q (A first on equal keys)
            int lo = max(0, q - nb), hi = min(q, na);
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (ks[a0 + mid] <= ks[a1 + q - 1 - mid]) lo = mid + 1;
                else hi = mid;
            }
            int i = lo, j = q - lo;
            const int stop = min(pe, a2);
            for (; p < stop; ++p) {
                const bool take_a = j >= nb || (i < na && ks[a0 + i] <= ks[a1 + j]);
                const int src = take_a ? a0 + i : a1 + j;
                kd[p] = ks[src];
                id[p] = is[src];
                i += take_a;
                j += !take_a;
            }
        }
        __syncthreads();
        uint32_t* tk = ks; ks = kd; kd = tk;
        uint16_t* ti = is; is = id; id = ti;
    }
    if (ks != ka) {  // the result at the front of s_key and in s_src
        for (int i = t; i < L; i += MG_THREADS) {
            ka[i] = ks[i];
            s_src[i] = is[i];
        }
    }
}

// one workgroup per bucket. GMAX: the runs it is compiled for (register pointers), CAP: the bucket bound
// (MG_M + GMAX) * MG_S records in LDS -- 3072 for up to 8 runs: ~35 KB, four workgroups per CU
template <int GMAX>
__global__ __launch_bounds__(MG_THREADS) void mg_merge_k(const MergeRuns a, const int64_t* __restrict__ bounds) {
    constexpr int CAP = (MG_M + GMAX) * MG_S;
    constexpr int E = 4;  // consecutive records of one slice per chunk: bounds walked forward, not searched again
    __shared__ int64_t s_key[CAP];
    __shared__ uint16_t s_src[CAP];  // output rank -> LDS slot
    __shared__ uint16_t s_src2[CAP];  // (the pairwise merge's second index buffer)
    __shared__ int64_t s_kmin;
    __shared__ int s_fit;
    __shared__ uint8_t s_run[CAP];   // LDS slot -> run
    __shared__ int64_t s_start[GMAX];
    __shared__ int s_pre[GMAX + 1];
    __shared__ const void* s_ptr[GMAX];  // the runs' key / column pointers (an LDS read, not a kernel-argument load per lane)
    const int t = threadIdx.x;
    const int G = a.G;
    const int64_t b = blockIdx.x;
    if (t < G) {  // the bucket's slice of each run (one lane per run)
        const int64_t lo = bounds[b * G + t], hi = bounds[(b + 1) * G + t];
        s_start[t] = lo;
        s_pre[t + 1] = (int)(hi - lo);
        s_ptr[t] = a.keys[t];
    }
    __syncthreads();
    if (t == 0) {
        s_pre[0] = 0;
        for (int r = 0; r < G; ++r) s_pre[r + 1] += s_pre[r];
    }
    __syncthreads();
    const int L = s_pre[G];
    int64_t off = 0;  // the bucket's first output position: every record below its splitter
    for (int r = 0; r < G; ++r) off += s_start[r];
    if (L > CAP) {  // cannot happen (the sampling bound); never write past the LDS
        if (t == 0) atomicOr(a.flag, 1);
        return;
    }
    // the bucket's key slices into LDS (slice r at s_pre[r]); all of a lane's loads issued before the stores
    {
        constexpr int B = CAP / MG_THREADS;
        int64_t kv[B];
        int r = 0;  // the slice of record i (i grows with k: continue the walk)
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const int i = t + k * MG_THREADS;
            if (i < L) {
                while (r + 1 < G && s_pre[r + 1] <= i) ++r;
                kv[k] = ((const int64_t*)s_ptr[r])[s_start[r] + (i - s_pre[r])];
                s_run[i] = (uint8_t)r;
            }
        }
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const int i = t + k * MG_THREADS;
            if (i < L) s_key[i] = kv[k];
        }
    }
    __syncthreads();
    // buckets whose keys span less than 2^32 (every slice is sorted: the extremes are slice ends) merge pairwise
    // with merge paths on u32 offsets (mg_pairwise); the others rank every record against the other slices
    if (t == 0) {
        int64_t mn = INT64_MAX, mx = INT64_MIN;
        for (int r = 0; r < G; ++r)
            if (s_pre[r + 1] > s_pre[r]) {
                mn = min(mn, s_key[s_pre[r]]);
                mx = max(mx, s_key[s_pre[r + 1] - 1]);
            }
        s_kmin = mn;
        s_fit = a.pairwise && L > 0 && (uint64_t)mx - (uint64_t)mn < 0xFFFFFFFFull;
    }
    __syncthreads();
    if (s_fit) {  // (block-uniform)
        mg_pairwise<GMAX, CAP>(L, G, s_key, s_src, s_src2, s_pre, s_kmin);
        __syncthreads();
        const uint32_t* kk = reinterpret_cast<const uint32_t*>(s_key);
        for (int p = t; p < L; p += MG_THREADS) a.out_keys[off + p] = s_kmin + (int64_t)kk[p];
        mg_out_cols<GMAX>(a, t, G, off, L, s_ptr, s_src, s_run, s_start, s_pre);
        return;
    }
    // each record's rank inside the bucket: its index in its slice + its bound in every other slice (earlier runs
    // first on equal keys). A chunk of E consecutive records of one slice searches the bounds for its first record
    // and walks them forward for the next ones (keys ascend inside a slice). (Interleaving the G searches of a
    // chunk's first record, branch-free, measured slower: 25.4 against 20.5 ms for 8 x 10^8 wide-span records.)
    for (int c = t; c * E < L; c += MG_THREADS) {
        const int i0 = c * E, i1 = min(i0 + E, L);
        int cur = -1;
        int ptr[GMAX];
        for (int i = i0; i < i1; ++i) {
            const int r = s_run[i];
            const int64_t k = s_key[i];
            int rank = i - s_pre[r];
#pragma unroll
            for (int r2 = 0; r2 < GMAX; ++r2) {
                if (r2 >= G || r2 == r) continue;
                const bool upper = r2 < r;
                const int hi = s_pre[r2 + 1];
                int lo;
                if (r != cur) {  // a new slice: binary search
                    lo = s_pre[r2];
                    int h = hi;
                    while (lo < h) {
                        const int mid = (lo + h) >> 1;
                        const int64_t v = s_key[mid];
                        if (v < k || (upper && v == k)) lo = mid + 1;
                        else h = mid;
                    }
                } else {  // the same slice: forward from the previous record's bound
                    lo = ptr[r2];
                    while (lo < hi) {
                        const int64_t v = s_key[lo];
                        if (!(v < k || (upper && v == k))) break;
                        ++lo;
                    }
                }
                ptr[r2] = lo;
                rank += lo - s_pre[r2];
            }
            cur = r;
            s_src[rank] = (uint16_t)i;
        }
    }
    __syncthreads();
    // keys in output order (contiguous stores)
    for (int p = t; p < L; p += MG_THREADS) a.out_keys[off + p] = s_key[s_src[p]];
    mg_out_cols<GMAX>(a, t, G, off, L, s_ptr, s_src, s_run, s_start, s_pre);
}

struct MergeWs {
    void* p = nullptr;
    size_t n = 0;
    void* ensure(size_t bytes) {
        if (bytes <= n) return p;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) throw std::runtime_error("merge workspace: hipMalloc failed");
        n = bytes;
        return p;
    }
};

}  // namespace

void merge_runs_device(int G, const int64_t* const* keys, const int64_t* lens, int ncols, const void* const* cols,
                       const uint8_t* widths, int64_t* out_keys, void* const* out_cols, hipStream_t stream) {
    if (G < 1 || G > MG_MAX_RUNS) throw std::invalid_argument("merge: 1 to " + std::to_string(MG_MAX_RUNS) + " runs");
    if (ncols < 0 || ncols > MG_MAX_COLS) throw std::invalid_argument("merge: too many columns");
    MergeRuns a;
    std::memset(&a, 0, sizeof a);
    a.G = G;
    a.ncols = ncols;
    {
        const char* e = getenv("SDG_MG_PAIR");
        a.pairwise = e ? atoi(e) : 1;
    }
    a.out_keys = out_keys;
    int64_t total = 0, ns = 0;
    for (int r = 0; r < G; ++r) {
        if (lens[r] < 0) throw std::invalid_argument("merge: negative run length");
        a.keys[r] = keys[r];
        a.len[r] = lens[r];
        a.sbase[r] = ns;
        ns += (lens[r] + MG_S - 1) / MG_S;
        total += lens[r];
        for (int c = 0; c < ncols; ++c) a.cols[r][c] = cols[(size_t)r * ncols + c];
    }
    a.sbase[G] = ns;
    for (int c = 0; c < ncols; ++c) {
        if (widths[c] != 1 && widths[c] != 2 && widths[c] != 4 && widths[c] != 8)
            throw std::invalid_argument("merge: column widths are 1, 2, 4 or 8 bytes");
        a.width[c] = widths[c];
        a.out_cols[c] = out_cols[c];
    }
    if (total == 0) return;
    if (ns >= (int64_t)0xFFFFFFF0) throw std::invalid_argument("merge: too many records");
    a.nsamples = ns;
    a.nbuckets = (ns + MG_M - 1) / MG_M;
    static MergeWs ws;
    static int64_t* h_ends = nullptr;  // pinned: the runs' end keys, then the bound flag
    if (!h_ends && hipHostMalloc((void**)&h_ends, (2 * MG_MAX_RUNS + 2) * 8) != hipSuccess)
        throw std::runtime_error("merge: hipHostMalloc failed");
    size_t tmp_bytes = 0;  // (sized for 64 key bits: at least what fewer bits need)
    if (rocprim::radix_sort_pairs(nullptr, tmp_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)ns, 0, 64, stream) != hipSuccess)
        throw std::runtime_error("merge: sample sort workspace");
    const size_t tmp_cap = tmp_bytes;
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t nb1 = (size_t)(a.nbuckets + 1) * G;
    const size_t need = 1024 + 2 * al((size_t)ns * 8) + 2 * al((size_t)ns * 4) + al(nb1 * 8) + al(tmp_bytes);
    uint8_t* w = (uint8_t*)ws.ensure(need);
    int64_t* d_ends = (int64_t*)w;  // 2G end keys + the flag word
    a.flag = (int*)(d_ends + 2 * MG_MAX_RUNS);
    w += 1024;
    // key bits the sample sort needs: keys relative to their minimum (one small read-back)
    if (hipMemsetAsync(a.flag, 0, 8, stream) != hipSuccess) throw std::runtime_error("merge: memset failed");
    hipLaunchKernelGGL(mg_ends_k, dim3(1), dim3(64), 0, stream, a, d_ends);
    if (hipMemcpyAsync(h_ends, d_ends, 2 * G * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        throw std::runtime_error("merge: reading the run ends failed");
    int64_t kmin = INT64_MAX, kmax = INT64_MIN;
    for (int r = 0; r < G; ++r)
        if (lens[r] > 0) {
            kmin = std::min(kmin, h_ends[2 * r]);
            kmax = std::max(kmax, h_ends[2 * r + 1]);
        }
    a.kmin = kmin;
    const uint64_t span = (uint64_t)kmax - (uint64_t)kmin;
    int bits = 1;
    while (bits < 64 && (span >> bits) != 0) ++bits;
    if (rocprim::radix_sort_pairs(nullptr, tmp_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)ns, 0, bits, stream) != hipSuccess || tmp_bytes > tmp_cap)
        throw std::runtime_error("merge: sample sort workspace");
    uint64_t* sk0 = (uint64_t*)w;
    w += al((size_t)ns * 8);
    uint64_t* sk1 = (uint64_t*)w;
    w += al((size_t)ns * 8);
    uint32_t* si0 = (uint32_t*)w;
    w += al((size_t)ns * 4);
    uint32_t* si1 = (uint32_t*)w;
    w += al((size_t)ns * 4);
    int64_t* bounds = (int64_t*)w;
    w += al(nb1 * 8);
    void* tmp = w;
    hipLaunchKernelGGL(mg_samples_k, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, stream, a, sk0, si0);
    if (rocprim::radix_sort_pairs(tmp, tmp_bytes, sk0, sk1, si0, si1, (size_t)ns, 0, bits, stream) != hipSuccess)
        throw std::runtime_error("merge: sample sort failed");
    hipLaunchKernelGGL(mg_bounds_k, dim3((unsigned)((nb1 + 255) / 256)), dim3(256), 0, stream, a, si1, bounds);
    if (G <= 8) hipLaunchKernelGGL(mg_merge_k<8>, dim3((unsigned)a.nbuckets), dim3(MG_THREADS), 0, stream, a, bounds);
    else if (G <= 16) hipLaunchKernelGGL(mg_merge_k<16>, dim3((unsigned)a.nbuckets), dim3(MG_THREADS), 0, stream, a, bounds);
    else hipLaunchKernelGGL(mg_merge_k<MG_MAX_RUNS>, dim3((unsigned)a.nbuckets), dim3(MG_THREADS), 0, stream, a, bounds);
    if (hipGetLastError() != hipSuccess) throw std::runtime_error("merge: kernel launch failed");
    if (hipMemcpyAsync(h_ends + 2 * MG_MAX_RUNS, a.flag, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        throw std::runtime_error("merge: kernels failed");
    if (*(int*)(h_ends + 2 * MG_MAX_RUNS)) throw std::runtime_error("merge: a bucket broke the sampling bound");
}

}  // namespace sdg
