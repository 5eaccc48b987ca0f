// Synthetic C5 stream generator on the GPU ("10^10 events, 10^8 keys (seed 17), ts_i = T0 +
// floor(i / 10^6), generated on-device per shard in batches of 2^28"). Benchmark / test infrastructure, not part of
// the engine: it produces the columns a caller then hands to sdg_push_device, exactly as an application would.
//
// Global event i (0-based) of the stream:
//   key   k_i  = splitmix64(seed, i) mod nkeys        (the partition key is the string "S%08d" % k_i)
//   price p_i  = rint((10 + 20 u) * 100) / 100, u = (splitmix64(seed + 1, i) >> 11) * 2^-53
//   ts_i       = T0 + floor(i / per_ms),  id_i = i,  volume_i = i mod 1000
// where splitmix64(s, i) is the (i+1)-th output of the splitmix64 sequence seeded with s (siddhi_amd/workloads.py
// splitmix64). Rank r of N owns key k iff fnv1a64("S%08d" % k) mod N == r (siddhi_amd/shard.py owner), so every
// rank generates the events of its own keys, in global order, with no exchange.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ double c5_price(uint64_t seed, uint64_t i) {
    const double u = (double)(splitmix64(seed + 1, i) >> 11) * (1.0 / 9007199254740992.0);
    // separate roundings (the build has -ffp-contract=off): numpy's rint((10 + 20 u) * 100) / 100
    const double x = __dadd_rn(10.0, __dmul_rn(20.0, u));
    return __ddiv_rn(rint(__dmul_rn(x, 100.0)), 100.0);
}

// fnv1a64 of the decimal key string "S%08d" (keys < 10^8)
__device__ __forceinline__ uint64_t key_hash(uint64_t k) {
    uint64_t h = 0xcbf29ce484222325ull;
    h = (h ^ (uint64_t)'S') * 0x100000001b3ull;
    uint64_t div = 10000000ull;
    for (int d = 0; d < 8; ++d) {
        const uint64_t digit = (k / div) % 10ull;
        h = (h ^ (uint64_t)('0' + digit)) * 0x100000001b3ull;
        div /= 10ull;
    }
    return h;
}

__global__ __launch_bounds__(256) void owner_k(int64_t nkeys, int32_t world, uint8_t* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < nkeys) out[k] = (uint8_t)(key_hash((uint64_t)k) % (uint64_t)world);
}

constexpr int TILE = 4096;  // global indices per block (256 threads x 16)

// pass 1: kept events per tile
__global__ __launch_bounds__(256) void count_k(uint64_t seed, int64_t nkeys, const int32_t* __restrict__ map, int64_t g0,
                                               int64_t g1, uint32_t* __restrict__ tile_cnt) {
    __shared__ uint32_t s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    const int64_t base = g0 + (int64_t)blockIdx.x * TILE;
    uint32_t c = 0;
    for (int j = 0; j < TILE / 256; ++j) {
        const int64_t i = base + j * 256 + threadIdx.x;
        if (i < g1) c += map[splitmix64(seed, (uint64_t)i) % (uint64_t)nkeys] >= 0;
    }
    atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = s;
}

// pass 2: exclusive prefix over the tiles (one block)
__global__ __launch_bounds__(1024) void scan_k(const uint32_t* __restrict__ cnt, int64_t ntiles, int64_t* __restrict__ off,
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

// pass 3: the kept events of each tile, in global order (stable: wave ballot ranks + per-wave prefix in LDS)
__global__ __launch_bounds__(256) void write_k(uint64_t seed, int64_t nkeys, const int32_t* __restrict__ map, int64_t g0,
                                               int64_t g1, int64_t t0, int64_t per_ms, const int64_t* __restrict__ off,
                                               int64_t cap, int64_t* __restrict__ ts, int64_t* __restrict__ id,
                                               uint32_t* __restrict__ sym, double* __restrict__ price,
                                               int32_t* __restrict__ volume) {
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = g0 + (int64_t)blockIdx.x * TILE;
    const int64_t out0 = off[blockIdx.x];
    for (int j = 0; j < TILE / 256; ++j) {
        const int64_t i = base + j * 256 + threadIdx.x;
        int32_t m = -1;
        if (i < g1) m = map[splitmix64(seed, (uint64_t)i) % (uint64_t)nkeys];
        const bool keep = m >= 0;
        const uint64_t b = __ballot(keep);
        const uint32_t below = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = (uint32_t)__popcll(b);
        __syncthreads();
        uint32_t pre = carry;
        for (int x = 0; x < w; ++x) pre += wsum[x];
        if (keep) {
            const int64_t o = out0 + pre + below;
            if (o < cap) {
                ts[o] = t0 + i / per_ms;
                id[o] = i;
                sym[o] = (uint32_t)m;
                price[o] = c5_price(seed, (uint64_t)i);
                volume[o] = (int32_t)(i % 1000);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void key_of_k(uint64_t seed, int64_t nkeys, const int64_t* __restrict__ ids, int64_t n,
                                                const int32_t* __restrict__ map, int64_t* __restrict__ out) {
    const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (x >= n) return;
    const uint64_t k = splitmix64(seed, (uint64_t)ids[x]) % (uint64_t)nkeys;
    out[x] = map ? (int64_t)map[k] : (int64_t)k;
}

__global__ __launch_bounds__(256) void price_of_k(uint64_t seed, const int64_t* __restrict__ ids, int64_t n,
                                                  double* __restrict__ out) {
    const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (x < n) out[x] = c5_price(seed, (uint64_t)ids[x]);
}

inline unsigned blocks(int64_t n, int64_t per) { return (unsigned)((n + per - 1) / per); }

// every entry point is synchronous: its callers (torch tensors on another HIP runtime instance, the engine's own
// stream) see the results as soon as it returns
inline int done(hipStream_t st) {
    if (hipGetLastError() != hipSuccess) return 1;
    return hipStreamSynchronize(st) != hipSuccess;
}

}  // namespace

extern "C" {

// owner[k] = fnv1a64("S%08d" % k) mod world, for k < nkeys
int sdg_synth_owner(int64_t nkeys, int32_t world, uint8_t* d_out, hipStream_t st) {
    if (nkeys > 100000000ll || world < 1) return 1;
    if (nkeys > 0) hipLaunchKernelGGL(owner_k, dim3(blocks(nkeys, 256)), dim3(256), 0, st, nkeys, world, d_out);
    return done(st);
}

// workspace bytes for a batch of global indices [g0, g1)
int64_t sdg_synth_workspace(int64_t g0, int64_t g1) {
    const int64_t nt = (g1 - g0 + TILE - 1) / TILE;
    return nt * 4 + nt * 8 + 64;
}

// the events of [g0, g1) whose key k has d_map[k] >= 0 (the caller's id for the key: an sdg_intern id), in global
// order, into the columns (cap rows each). *d_count (device) and *h_count (host, optional) = the number kept (may
// exceed cap: nothing past cap is written)
int sdg_synth_batch(uint64_t seed, int64_t nkeys, const int32_t* d_map, int64_t g0, int64_t g1, int64_t t0,
                    int64_t per_ms, void* d_work, int64_t cap, int64_t* d_ts, int64_t* d_id, uint32_t* d_sym,
                    double* d_price, int32_t* d_volume, int64_t* d_count, int64_t* h_count, hipStream_t st) {
    if (g1 < g0 || per_ms <= 0 || nkeys <= 0) return 1;
    const int64_t nt = (g1 - g0 + TILE - 1) / TILE;
    if (nt > 0x7FFFFFFF) return 1;
    uint32_t* cnt = (uint32_t*)d_work;
    int64_t* off = (int64_t*)((uint8_t*)d_work + ((nt * 4 + 15) & ~15ll));
    if (nt == 0) {
        (void)hipMemsetAsync(d_count, 0, 8, st);
    } else {
        hipLaunchKernelGGL(count_k, dim3((unsigned)nt), dim3(256), 0, st, seed, nkeys, d_map, g0, g1, cnt);
        hipLaunchKernelGGL(scan_k, dim3(1), dim3(1024), 0, st, cnt, nt, off, d_count);
        hipLaunchKernelGGL(write_k, dim3((unsigned)nt), dim3(256), 0, st, seed, nkeys, d_map, g0, g1, t0, per_ms, off, cap,
                           d_ts, d_id, d_sym, d_price, d_volume);
    }
    if (h_count && hipMemcpyAsync(h_count, d_count, 8, hipMemcpyDeviceToHost, st) != hipSuccess) return 1;
    return done(st);
}

// per event id: d_map[key] (d_map != nullptr) or the key index itself
int sdg_synth_key_of(uint64_t seed, int64_t nkeys, const int64_t* d_ids, int64_t n, const int32_t* d_map, int64_t* d_out,
                     hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(key_of_k, dim3(blocks(n, 256)), dim3(256), 0, st, seed, nkeys, d_ids, n, d_map, d_out);
    return done(st);
}

// per event id: its price (the generator's formula; `seed` is the key seed, the price stream uses seed + 1)
int sdg_synth_price_of(uint64_t seed, const int64_t* d_ids, int64_t n, double* d_out, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(price_of_k, dim3(blocks(n, 256)), dim3(256), 0, st, seed, d_ids, n, d_out);
    return done(st);
}

}  // extern "C"
