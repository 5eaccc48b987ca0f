// Wave64 / block helpers shared by the gfx950 kernels: lane masks, ballot + mbcnt compaction, block-wide
// reservation of output ranges (one global atomic per block).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdg {

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

// inclusive scan of one value per thread over threads 0..255 (waves 0-3: shuffles, then one barrier for the wave
// totals). Every thread of the block must call it (threads >= 256 pass anything and get garbage); wsum: 4 words of
// LDS. Replaces the 8-step Hillis-Steele loop over an LDS array (16 block barriers).
__device__ __forceinline__ uint32_t scan256_incl(uint32_t x, uint32_t* wsum) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (w < 4 && lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t pre = 0;
    if (w < 4)
        for (int v = 0; v < w; ++v) pre += wsum[v];
    return x + pre;
}

// block-wide exclusive scan of two per-thread counts; one atomic per block and counter reserves the block's
// output ranges (per-wave reservations on one global counter serialise in L2 at ~10^8/s). Every thread of the
// block must call it.
template <int THREADS>
__device__ __forceinline__ void block_reserve2(uint32_t c0, uint32_t c1, unsigned long long* ctr0,
                                               unsigned long long* ctr1, int64_t* off0, int64_t* off1) {
    __shared__ uint32_t wtot[2][THREADS / 64];
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
        for (int v = 0; v < THREADS / 64; ++v) {
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

}  // namespace sdg
