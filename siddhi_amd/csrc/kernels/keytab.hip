// Device-resident partition key table for int / long / float / double / bool partition attributes: an open-addressed HBM hash
// table from the key value to the dense key id the rest of the engine indexes its per-key state with (arenas,
// carries, segments). ValuePartitionExecutor keys a partition by the attribute's toString (reference:
// core/partition/executor/ValuePartitionExecutor.java, PartitionStreamReceiver.java:262-272); Java's toString is
// injective on int / long and prints equal values of either type alike, so the sign-extended 64-bit value stands
// for the key. Ids are dense and assigned in order of a key's first row, as the host dictionary assigns them
// (engine.cpp host_key), so a batch maps to the same ids whichever side it was pushed from.
//
// Slots (kernels.h KtSlot, 16 B): key (KT_EMPTY = free; the value KT_EMPTY itself lives in the extra slot cap, key =
// 1 when used), id (id + 1, 0 = new in this batch), first (smallest row of a new key). Linear probing; a
// probe sequence longer than KT_MAX_PROBE, or a batch whose new keys would fill the table over half, stops the pass
// early (flags) and the host grows the table (at least 8x) and probes again.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sdg {
namespace {

constexpr int64_t KT_EMPTY = INT64_MIN;
constexpr uint32_t KT_MAX_PROBE = 4096;
constexpr uint32_t KT_NEW = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t kt_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// the 64-bit value standing for a key's toString. A query's table holds one class of key attribute (integral,
// float, double or bool: engine.cpp key_class), so the encodings never meet: int / long sign-extended (equal values
// print alike); double / float bit patterns -- Double/Float.toString is injective on them (-0.0 prints "-0.0", 0.0
// "0.0") except that every NaN prints "NaN", so NaNs map to the canonical NaN; bool 0 / 1
__device__ __forceinline__ int64_t kt_value(const void* col, int kind, int64_t r) {
    switch (kind) {
        case VK_I32: return (int64_t)((const int32_t*)col)[r];
        case VK_F64: {
            const int64_t b = ((const int64_t*)col)[r];
            return (b & 0x7FFFFFFFFFFFFFFFll) > 0x7FF0000000000000ll ? 0x7FF8000000000000ll : b;
        }
        case VK_F32: {
            const int32_t b = ((const int32_t*)col)[r];
            return (b & 0x7FFFFFFF) > 0x7F800000 ? 0x7FC00000ll : (int64_t)(uint32_t)b;
        }
        case VK_BOOL: return ((const uint8_t*)col)[r] ? 1 : 0;
        default: return ((const int64_t*)col)[r];
    }
}

// a new key: counted; once the table would be over half full, flags[1] stops the pass (the host grows the table)
__device__ __forceinline__ void kt_count_new(unsigned long long* new_count, unsigned long long limit, int* flags) {
    if (!new_count) return;
    if (atomicAdd(new_count, 1ull) >= limit) atomicOr(&flags[1], 1);
}

// the slot of v, inserting it when absent; -1: probe limit hit, or the pass was stopped
__device__ __forceinline__ int64_t kt_slot(const KeyTab& t, int64_t v, unsigned long long* new_count,
                                           unsigned long long limit, int* flags) {
    if (v == KT_EMPTY) {
        const unsigned long long was = atomicCAS((unsigned long long*)&t.slots[t.cap].key, 0ull, 1ull);
        if (was == 0ull) kt_count_new(new_count, limit, flags);
        return t.cap;
    }
    uint64_t h = kt_mix((uint64_t)v) & t.mask;
    for (uint32_t i = 0; i < KT_MAX_PROBE && i <= t.mask; ++i) {
        if ((i & 31) == 31 && flags && *(volatile int*)&flags[1]) return -1;
        int64_t cur = t.slots[h].key;
        if (cur == KT_EMPTY) {  // a stale read can only show a slot as still free: the CAS decides
            cur = (int64_t)atomicCAS((unsigned long long*)&t.slots[h].key, (unsigned long long)KT_EMPTY, (unsigned long long)v);
            if (cur == KT_EMPTY) {
                kt_count_new(new_count, limit, flags);
                return (int64_t)h;
            }
        }
        if (cur == v) return (int64_t)h;
        h = (h + 1) & t.mask;
    }
    return -1;
}

__global__ __launch_bounds__(256) void kt_clear_k(KeyTab t) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > (int64_t)t.cap) return;
    t.slots[i].key = i == (int64_t)t.cap ? 0 : KT_EMPTY;
    t.slots[i].id = 0;
    t.slots[i].first = 0xFFFFFFFFu;
}

// known keys (the host dictionary's, id order)
__global__ __launch_bounds__(256) void kt_load_k(KeyTab t, const int64_t* __restrict__ vals, uint32_t id0, int64_t n,
                                                 int* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t s = kt_slot(t, vals[i], nullptr, 0, nullptr);
    if (s < 0) {
        atomicOr(&flags[0], 1);
        return;
    }
    t.slots[s].id = id0 + (uint32_t)i + 1u;
}

// per row: the key id, or KT_NEW (first sighting in this batch: the row's index competes for the key's first row).
// KT_RPT rows per thread (a block's rows strided by 256, loads coalesced): the rows' values, the stop flag and then
// the rows' home slots (16 B: key and id in one load) are all in flight together; a row whose home slot holds its key
// is done (the common case once the table knows the keys), the others take the probing / inserting walk (kt_slot).
constexpr int KT_RPT = 4;
__global__ __launch_bounds__(256) void kt_probe_k(KeyTab t, const void* __restrict__ col, int kind, int64_t n,
                                                  uint32_t* __restrict__ out, unsigned long long* __restrict__ new_count,
                                                  unsigned long long limit, int* __restrict__ flags) {
    const int64_t r0 = (int64_t)blockIdx.x * (256 * KT_RPT) + threadIdx.x;
    int64_t v[KT_RPT];
#pragma unroll
    for (int j = 0; j < KT_RPT; ++j) {
        const int64_t r = r0 + j * 256;
        v[j] = r < n ? kt_value(col, kind, r) : KT_EMPTY;
    }
    const int stop = *(volatile int*)&flags[1];
    uint4 home[KT_RPT];
#pragma unroll
    for (int j = 0; j < KT_RPT; ++j) {
        const uint64_t h = kt_mix((uint64_t)v[j]) & t.mask;
        home[j] = r0 + j * 256 < n && v[j] != KT_EMPTY ? *reinterpret_cast<const uint4*>(&t.slots[h]) : make_uint4(0, 0, 0, 0);
    }
    if (stop) return;  // stopped: the table is being outgrown
#pragma unroll
    for (int j = 0; j < KT_RPT; ++j) {
        const int64_t r = r0 + j * 256;
        if (r >= n) break;
        const int64_t hk = (int64_t)(((uint64_t)home[j].y << 32) | home[j].x);
        uint32_t id;
        if (v[j] != KT_EMPTY && hk == v[j]) {
            id = home[j].z;
            if (!id) atomicMin(&t.slots[kt_mix((uint64_t)v[j]) & t.mask].first, (uint32_t)r);
        } else {
            const int64_t sl = kt_slot(t, v[j], new_count, limit, flags);
            if (sl < 0) {
                atomicOr(&flags[0], 1);
                out[r] = 0;
                continue;
            }
            id = t.slots[sl].id;
            if (!id) atomicMin(&t.slots[sl].first, (uint32_t)r);
        }
        out[r] = id ? id - 1u : KT_NEW;
    }
}

// the slots of the batch's new keys: (first row << 32 | slot) and the key values
__global__ __launch_bounds__(256) void kt_collect_k(KeyTab t, unsigned long long* __restrict__ pairs,
                                                    int64_t* __restrict__ vals, unsigned long long* __restrict__ cnt,
                                                    int64_t cap_out) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s > (int64_t)t.cap) return;
    const bool used = s == (int64_t)t.cap ? t.slots[s].key != 0 : t.slots[s].key != KT_EMPTY;
    if (!used || t.slots[s].id != 0) return;
    const unsigned long long o = atomicAdd(cnt, 1ull);
    if ((int64_t)o >= cap_out) return;  // the host sized pairs by the probe's count
    pairs[o] = ((unsigned long long)t.slots[s].first << 32) | (unsigned long long)s;
    vals[o] = s == (int64_t)t.cap ? KT_EMPTY : t.slots[s].key;
}

__global__ __launch_bounds__(256) void kt_assign_k(KeyTab t, const uint32_t* __restrict__ slots, uint32_t id0, int64_t m) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    t.slots[slots[i]].id = id0 + (uint32_t)i + 1u;
}

__global__ __launch_bounds__(256) void kt_fix_k(KeyTab t, const void* __restrict__ col, int kind, int64_t n,
                                                uint32_t* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n || out[r] != KT_NEW) return;
    const int64_t s = kt_slot(t, kt_value(col, kind, r), nullptr, 0, nullptr);  // present: inserted by the probe
    out[r] = s >= 0 ? t.slots[s].id - 1u : 0u;
}

dim3 blocks(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

void kt_clear(const KeyTab& t, hipStream_t st) { hipLaunchKernelGGL(kt_clear_k, blocks((int64_t)t.cap + 1), dim3(256), 0, st, t); }
void kt_load(const KeyTab& t, const int64_t* vals, uint32_t id0, int64_t n, int* flags, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(kt_load_k, blocks(n), dim3(256), 0, st, t, vals, id0, n, flags);
}
void kt_probe(const KeyTab& t, const void* col, int kind, int64_t n, uint32_t* out, unsigned long long* new_count,
              unsigned long long limit, int* flags, hipStream_t st) {
    if (n > 0)
        hipLaunchKernelGGL(kt_probe_k, dim3((unsigned)((n + 256 * KT_RPT - 1) / (256 * KT_RPT))), dim3(256), 0, st, t, col,
                           kind, n, out, new_count, limit, flags);
}
void kt_collect(const KeyTab& t, unsigned long long* pairs, int64_t* vals, unsigned long long* cnt, int64_t cap_out,
                hipStream_t st) {
    hipLaunchKernelGGL(kt_collect_k, blocks((int64_t)t.cap + 1), dim3(256), 0, st, t, pairs, vals, cnt, cap_out);
}
void kt_assign(const KeyTab& t, const uint32_t* slots, uint32_t id0, int64_t m, hipStream_t st) {
    if (m > 0) hipLaunchKernelGGL(kt_assign_k, blocks(m), dim3(256), 0, st, t, slots, id0, m);
}
void kt_fix(const KeyTab& t, const void* col, int kind, int64_t n, uint32_t* out, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(kt_fix_k, blocks(n), dim3(256), 0, st, t, col, kind, n, out);
}

}  // namespace sdg
