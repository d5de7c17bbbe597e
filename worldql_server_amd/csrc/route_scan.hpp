// route_scan.hpp — pass 2 of the tick: exclusive scan of the count pass's per-block totals.
//
// The count pass reduces e_m per block of 256*IPT messages; this single 1024-thread block scans
// those few thousand totals (C2: 1,954) into tile_prefix[], writes offsets[M] = P and the
// counters. The emit pass turns tile_prefix + a block-local scan into every CSR offset, so no
// 1M-element global scan and no inter-block look-back is needed anywhere in the tick.
#pragma once
#include "route_common.hpp"

namespace wq {

constexpr int kScanThreads = 1024;
constexpr int kScanWaves = kScanThreads / 64;

struct TileScanParams {
    const uint32_t* tile_total;
    const uint32_t* tile_F;
    uint32_t* tile_prefix;
    uint32_t n_tiles;
    uint32_t* offsets;  // offsets[M] = P
    uint32_t M;
    uint64_t capacity;
    wq_route_counters* cnt;
    uint32_t* health;  // sticky {error, overflow} words (flag_route)
};

__device__ __forceinline__ uint64_t wave_incl_scan_add64(uint64_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

static __global__ __launch_bounds__(kScanThreads) void tile_scan_kernel(TileScanParams p) {
    __shared__ uint64_t s_wave[kScanWaves];
    __shared__ uint64_t s_F[kScanWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t carry = 0, F = 0;
    for (uint32_t i = tid; i < p.n_tiles; i += kScanThreads) F += p.tile_F[i];
    F = wave_sum_u64(F);
    if (lane == 0) s_F[wave] = F;
    for (uint32_t b = 0; b < p.n_tiles; b += kScanThreads) {
        const uint32_t i = b + tid;
        const uint64_t x = i < p.n_tiles ? p.tile_total[i] : 0u;
        const uint64_t incl = wave_incl_scan_add64(x, lane);
        if (lane == 63) s_wave[wave] = incl;
        __syncthreads();
        uint64_t before = carry, tot = 0;
#pragma unroll
        for (int u = 0; u < kScanWaves; ++u) {
            const uint64_t t = s_wave[u];
            if (u < wave) before += t;
            tot += t;
        }
        if (i < p.n_tiles) p.tile_prefix[i] = (uint32_t)(before + incl - x);
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) {
        uint64_t Ft = 0;
#pragma unroll
        for (int u = 0; u < kScanWaves; ++u) Ft += s_F[u];
        p.cnt->n_candidates = Ft;
        const uint64_t P = carry;
        p.offsets[p.M] = (uint32_t)P;
        p.cnt->n_pairs = P;
        // u32 CSR offsets cannot hold more than 2^32-1 pairs: error bit 2
        flag_route(p.cnt, p.health, P > 0xFFFFFFFFull ? 2u : 0u, P > p.capacity ? 1u : 0u);
    }
}

}  // namespace wq
