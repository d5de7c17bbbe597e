// table_prims.hpp — small device primitives shared by the table builders (wq_table.hip,
// wq_delta.hip): grid sizing, iota / gather kernels and rocPRIM radix-sort / scan wrappers whose
// temporary storage lives in h->sort_tmp. Everything is TU-local (anonymous namespace).
#pragma once
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "wq_internal.hpp"

namespace wq {
namespace {

constexpr int kBlock = 256;

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

__global__ void k_iota(uint32_t* a, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) a[i] = (uint32_t)i;
}

template <typename T>
__global__ void k_gather(const T* __restrict__ src, const uint32_t* __restrict__ idx, T* dst,
                         uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}

// ---- rocPRIM wrappers (temp storage in h->sort_tmp) ----

template <typename K, typename V = uint32_t>
int sort_pairs(wq_router* h, const K* kin, K* kout, const V* vin, V* vout, uint64_t n, int end_bit) {
    size_t bytes = 0;
    WQ_HIP(h, rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, (size_t)n, 0, end_bit,
                                        h->stream));
    WQ_ALLOC(h, h->sort_tmp, bytes);
    WQ_HIP(h, rocprim::radix_sort_pairs(h->sort_tmp.p, bytes, kin, kout, vin, vout, (size_t)n, 0,
                                        end_bit, h->stream));
    return WQ_OK;
}

int sort_keys_u64(wq_router* h, const uint64_t* kin, uint64_t* kout, uint64_t n) {
    size_t bytes = 0;
    WQ_HIP(h, rocprim::radix_sort_keys(nullptr, bytes, kin, kout, (size_t)n, 0, 64, h->stream));
    WQ_ALLOC(h, h->sort_tmp, bytes);
    WQ_HIP(h, rocprim::radix_sort_keys(h->sort_tmp.p, bytes, kin, kout, (size_t)n, 0, 64, h->stream));
    return WQ_OK;
}

int scan_u32(wq_router* h, const uint32_t* in, uint32_t* out, uint64_t n, bool inclusive) {
    size_t bytes = 0;
    if (inclusive) {
        WQ_HIP(h, rocprim::inclusive_scan(nullptr, bytes, in, out, (size_t)n, rocprim::plus<uint32_t>(),
                                          h->stream));
        WQ_ALLOC(h, h->sort_tmp, bytes);
        WQ_HIP(h, rocprim::inclusive_scan(h->sort_tmp.p, bytes, in, out, (size_t)n,
                                          rocprim::plus<uint32_t>(), h->stream));
    } else {
        WQ_HIP(h, rocprim::exclusive_scan(nullptr, bytes, in, out, 0u, (size_t)n,
                                          rocprim::plus<uint32_t>(), h->stream));
        WQ_ALLOC(h, h->sort_tmp, bytes);
        WQ_HIP(h, rocprim::exclusive_scan(h->sort_tmp.p, bytes, in, out, 0u, (size_t)n,
                                          rocprim::plus<uint32_t>(), h->stream));
    }
    return WQ_OK;
}

// n-th element of a device u32 array (synchronous read; build path only).
int read_u32(wq_router* h, const uint32_t* a, uint64_t i, uint32_t* out) {
    WQ_HIP(h, hipMemcpyAsync(out, a + i, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
    WQ_HIP(h, hipStreamSynchronize(h->stream));
    return WQ_OK;
}

int ensure_state(wq_router* h, State& s, uint64_t n) {
    const uint64_t m = n ? n : 1;
    WQ_ALLOC(h, s.h, m * 8);
    WQ_ALLOC(h, s.w, m * 4);
    WQ_ALLOC(h, s.kx, m * 8);
    WQ_ALLOC(h, s.ky, m * 8);
    WQ_ALLOC(h, s.kz, m * 8);
    WQ_ALLOC(h, s.p, m * 4);
    return WQ_OK;
}

}  // namespace
}  // namespace wq
