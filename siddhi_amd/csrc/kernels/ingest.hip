// Device-side batch view of mixed pushes (sdg_push_mixed: InputHandler.send calls of several streams, interleaved,
// attributes as 64-bit slots): a query's view rows -- the rows of its streams, in arrival order, null partition keys
// dropped (PartitionStreamReceiver.java:262-272) -- with its physical columns at their widths, the query-stream
// index of each row, the row's batch position and the partition key value, built on the GPU by a stable compaction
// (per-tile counts, one scan, per-tile writes with wave ballot ranks) instead of a per-row host loop.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"
#include "wave.h"

namespace sdg {
namespace {

constexpr int MV_TILE = 4096;  // rows per block (256 threads x 16)

struct MvRow {
    bool keep;
    int qp;
};

__device__ __forceinline__ MvRow mv_row(const MixedViewArgs& a, int64_t r) {  // (a: device memory)
    MvRow x{false, -1};
    if (r >= a.n) return x;
    const int32_t s = a.streams[r];
    const int qp = (s >= 0 && s < MV_MAX_STREAMS) ? a.qpos[s] : -1;
    if (qp < 0) return x;
    if (a.partitioned) {
        const int ka = a.key_attr[qp];
        if (ka < 0) return x;
        if (a.slot_nulls[ka] && a.slot_nulls[ka][r]) return x;  // null partition key: dropped
    }
    x.keep = true;
    x.qp = qp;
    return x;
}

// arguments from a device copy: indexing a by-value kernel argument (slots[attr]) copies the struct to scratch
__global__ __launch_bounds__(256) void mv_count_k(const MixedViewArgs* __restrict__ pa, uint32_t* __restrict__ cnt) {
    const MixedViewArgs& a = *pa;
    __shared__ uint32_t s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * MV_TILE;
    uint32_t c = 0;
    for (int j = 0; j < MV_TILE / 256; ++j) c += mv_row(a, base + j * 256 + threadIdx.x).keep;
    atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void mv_scan_k(const uint32_t* __restrict__ cnt, int64_t ntiles, int64_t* __restrict__ off,
                                                  int64_t* __restrict__ total) {
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t per = (ntiles + 1023) / 1024;
    const int64_t lo = t * per, hi = lo + per < ntiles ? lo + per : ntiles;
    int64_t s = 0;
    for (int64_t i = lo; i < hi; ++i) s += cnt[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int64_t x = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    int64_t run = part[t] - s;
    for (int64_t i = lo; i < hi; ++i) {
        off[i] = run;
        run += cnt[i];
    }
    if (t == 1023) *total = part[1023];
}

// the key's value as the device key table encodes it (keytab.hip kt_value): integral sign-extended, real bit
// patterns with one canonical NaN, bool 0 / 1; string ids as they are
__device__ __forceinline__ int64_t mv_key_value(int64_t slot, uint8_t kind) {
    switch (kind) {
        case VK_I32: return (int64_t)(int32_t)slot;
        case VK_F64: return (slot & 0x7FFFFFFFFFFFFFFFll) > 0x7FF0000000000000ll ? 0x7FF8000000000000ll : slot;
        case VK_F32: {
            const int32_t b = (int32_t)slot;
            return (b & 0x7FFFFFFF) > 0x7F800000 ? 0x7FC00000ll : (int64_t)(uint32_t)b;
        }
        case VK_BOOL: return slot ? 1 : 0;
        case VK_STR: return (int64_t)(uint32_t)slot;
        default: return slot;
    }
}

__global__ __launch_bounds__(256) void mv_write_k(const MixedViewArgs* __restrict__ pa, const int64_t* __restrict__ off) {
    const MixedViewArgs& a = *pa;
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * MV_TILE;
    const int64_t out0 = off[blockIdx.x];
    for (int j = 0; j < MV_TILE / 256; ++j) {
        const int64_t r = base + j * 256 + threadIdx.x;
        const MvRow x = mv_row(a, r);
        const uint64_t b = __ballot(x.keep);
        const uint32_t below = (uint32_t)__popcll(b & lanemask_lt());
        if (lane == 0) wsum[w] = (uint32_t)__popcll(b);
        __syncthreads();
        uint32_t pre = carry;
        for (int y = 0; y < w; ++y) pre += wsum[y];
        if (x.keep) {
            const int64_t o = out0 + pre + below;
            a.out_ts[o] = a.ts[r];
            a.out_pos[o] = (uint32_t)(a.pos0 + r);
            if (a.out_qs) a.out_qs[o] = (uint8_t)x.qp;
            if (a.partitioned) {
                const int ka = a.key_attr[x.qp];
                a.out_key[o] = mv_key_value(a.slots[ka][r], a.key_kind[x.qp]);
            }
            for (int k = 0; k < a.n_cols; ++k) {
                const int ai = a.col_attr[x.qp][k];
                const int64_t v = ai >= 0 ? a.slots[ai][r] : 0;  // a column of another stream: zeros, not null
                switch (a.col_width[k]) {
                    case 8: ((int64_t*)a.out_cols[k])[o] = v; break;
                    case 4: ((int32_t*)a.out_cols[k])[o] = (int32_t)v; break;
                    default: ((uint8_t*)a.out_cols[k])[o] = (uint8_t)v; break;
                }
                if (a.out_nulls[k]) a.out_nulls[k][o] = (ai >= 0 && a.slot_nulls[ai]) ? a.slot_nulls[ai][r] : 0;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void narrow_k(const int64_t* __restrict__ src, int64_t n, uint32_t* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = (uint32_t)src[i];
}

}  // namespace

void narrow_u32(const int64_t* src, int64_t n, uint32_t* dst, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(narrow_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, n, dst);
}

size_t mixed_view_workspace(int64_t n) {
    const int64_t nt = (n + MV_TILE - 1) / MV_TILE;
    return (size_t)nt * 4 + (size_t)nt * 8 + 64;
}

void mixed_view_count(const MixedViewArgs& a, const MixedViewArgs* d_a, void* work, int64_t* d_total, hipStream_t st) {
    const int64_t nt = (a.n + MV_TILE - 1) / MV_TILE;
    if (nt == 0) {
        (void)hipMemsetAsync(d_total, 0, 8, st);
        return;
    }
    uint32_t* cnt = (uint32_t*)work;
    int64_t* off = (int64_t*)((uint8_t*)work + ((nt * 4 + 15) & ~15ll));
    hipLaunchKernelGGL(mv_count_k, dim3((unsigned)nt), dim3(256), 0, st, d_a, cnt);
    hipLaunchKernelGGL(mv_scan_k, dim3(1), dim3(1024), 0, st, cnt, nt, off, d_total);
}

void mixed_view_write(const MixedViewArgs& a, const MixedViewArgs* d_a, void* work, hipStream_t st) {
    const int64_t nt = (a.n + MV_TILE - 1) / MV_TILE;
    if (nt == 0) return;
    const int64_t* off = (const int64_t*)((uint8_t*)work + ((nt * 4 + 15) & ~15ll));
    hipLaunchKernelGGL(mv_write_k, dim3((unsigned)nt), dim3(256), 0, st, d_a, off);
}

// ---- broadcast rows (kernels.h BcastExpandArgs) ---------------------------------------------------------------
namespace {
__device__ __forceinline__ void bx_copy_cols(const BcastExpandArgs& a, int64_t from, int64_t to) {
    for (int c = 0; c < a.ncols; ++c) {
        const int w = a.width[c];
        if (w == 8) ((int64_t*)a.o_cols[c])[to] = ((const int64_t*)a.cols[c])[from];
        else if (w == 4) ((uint32_t*)a.o_cols[c])[to] = ((const uint32_t*)a.cols[c])[from];
        else ((uint8_t*)a.o_cols[c])[to] = ((const uint8_t*)a.cols[c])[from];
        if (a.o_nulls[c]) a.o_nulls[c][to] = a.nulls[c] ? a.nulls[c][from] : 0;
    }
}
// every compact row moves to off[r]; a placeholder's slot is written by bx_expand_k
__global__ __launch_bounds__(256) void bx_move_k(BcastExpandArgs a) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= a.n) return;
    if (a.key[r] == BX_PLACEHOLDER) return;  // a placeholder: bx_expand_k writes its rows
    const uint32_t o = a.off[r];
    a.o_ts[o] = a.ts[r];
    a.o_vpos[o] = a.vpos[r];
    if (a.o_qs) a.o_qs[o] = a.qs[r];
    a.o_key[o] = a.key[r];
    if (a.o_vrank) a.o_vrank[o] = a.vrank ? a.vrank[r] : 0u;
    bx_copy_cols(a, r, o);
}
// placeholder p (grid y, strided) x key x of its order (grid x): the event's row for that key, ranked x
__global__ __launch_bounds__(256) void bx_expand_k(BcastExpandArgs a) {
    const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (int64_t p = blockIdx.y; p < a.nph; p += gridDim.y) {
        const uint32_t k = a.ph_k[p];
        if (x >= k) continue;
        const uint32_t r = a.ph_row[p];
        const int64_t o = (int64_t)a.off[r] + x;
        a.o_ts[o] = a.ts[r];
        a.o_vpos[o] = a.vpos[r];
        if (a.o_qs) a.o_qs[o] = a.qs[r];
        a.o_key[o] = a.ord[(int64_t)a.ph_ord[p] + x];
        if (a.o_vrank) a.o_vrank[o] = (uint32_t)x;
        bx_copy_cols(a, r, o);
    }
}
}  // namespace

void bcast_expand(const BcastExpandArgs& a, int64_t kmax, hipStream_t st) {
    if (a.n > 0) hipLaunchKernelGGL(bx_move_k, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
    if (a.nph > 0 && kmax > 0)
        hipLaunchKernelGGL(bx_expand_k, dim3((unsigned)((kmax + 255) / 256), (unsigned)std::min<int64_t>(a.nph, 65535)),
                           dim3(256), 0, st, a);
}

}  // namespace sdg
