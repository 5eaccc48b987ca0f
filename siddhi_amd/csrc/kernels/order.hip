// Delivery order of a flush's match records on the device: records come out of the matchers in arbitrary order
// (wave-aggregated appends), and the reference delivers them by emitting event, then by the partial's place in
// the pending list (StateMultiProcessStreamReceiver.processAndClear :47-68, QuerySelector.processNoGroupBy
// :161-205). Two stable LSD radix sorts of a record index (rocPRIM: a library sort for a bookkeeping pass, not
// the matching path) -- by the ordinal, then by the emitting event's position -- and one gather per column, so
// the host reads the records back already in order.
#include <hip/hip_runtime.h>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "kernels.h"

namespace sdg {
namespace {

__global__ __launch_bounds__(256) void order_keys_k(const int64_t* __restrict__ emit, const int64_t* __restrict__ sub,
                                                    int64_t n, int64_t emit_base, int64_t sub_bias, uint32_t* __restrict__ ek,
                                                    uint64_t* __restrict__ sk, uint32_t* __restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    ek[i] = (uint32_t)(emit[i] - emit_base);
    sk[i] = (uint64_t)(sub[i] - sub_bias);
    idx[i] = (uint32_t)i;
}

template <typename T>
__global__ __launch_bounds__(256) void gather_k(const T* __restrict__ src, const uint32_t* __restrict__ perm, int64_t n,
                                                T* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}

void temp_sizes(int64_t n, size_t& a, size_t& b) {
    uint64_t* k64 = nullptr;
    uint32_t* k32 = nullptr;
    uint32_t* v = nullptr;
    a = b = 0;
    rocprim::radix_sort_pairs(nullptr, a, k64, k64, v, v, (size_t)n, 0, 48);
    rocprim::radix_sort_pairs(nullptr, b, k32, k32, v, v, (size_t)n, 0, 32);
}

}  // namespace

size_t order_workspace(int64_t n) {
    size_t a = 0, b = 0;
    temp_sizes(n, a, b);
    const size_t sort_tmp = ((a > b ? a : b) + 255) & ~size_t(255);
    // keys: sub (2 x 8n) + emit (2 x 4n), index (2 x 4n)
    return sort_tmp + (size_t)n * (16 + 8 + 8) + 1024;
}

void order_records(const int64_t* emit, const int64_t* sub, int64_t n, int64_t emit_base, int64_t sub_bias, void* work,
                   size_t work_bytes, uint32_t** perm_out, hipStream_t stream) {
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
    (void)work_bytes;
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(order_keys_k, dim3(grid), dim3(256), 0, stream, emit, sub, n, emit_base, sub_bias, ek0, sk0, ix0);
    // by the ordinal, then (stable) by the emitting event
    rocprim::radix_sort_pairs(tmp, a, sk0, sk1, ix0, ix1, (size_t)n, 0, 48, stream);
    hipLaunchKernelGGL(gather_k<uint32_t>, dim3(grid), dim3(256), 0, stream, ek0, ix1, n, ek1);
    rocprim::radix_sort_pairs(tmp, b, ek1, ek0, ix1, ix0, (size_t)n, 0, 32, stream);
    *perm_out = ix0;
}

void gather_i64(const int64_t* src, const uint32_t* perm, int64_t n, int64_t* dst, hipStream_t stream) {
    if (n > 0) hipLaunchKernelGGL(gather_k<int64_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, src, perm, n, dst);
}
void gather_u32(const uint32_t* src, const uint32_t* perm, int64_t n, uint32_t* dst, hipStream_t stream) {
    if (n > 0) hipLaunchKernelGGL(gather_k<uint32_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, src, perm, n, dst);
}

}  // namespace sdg
