// route_scan.hpp — pass 2 of the tick: exclusive scan of the count pass's per-block totals.
//
// The count pass reduces e_m per block of 256*IPT messages; this single 1024-thread block scans
// those few thousand totals (C2: 3,907; C3: 39,063) into tile_prefix[], writes offsets[M] = P and the
// counters. The emit pass turns tile_prefix + a block-local scan into every CSR offset, so no
// 1M-element global scan and no inter-block look-back is needed anywhere in the tick.
#pragma once
#include <cstdlib>
#include <cstring>  // rocPRIM's host code needs memset declared first

#include <rocprim/rocprim.hpp>

#include "route_common.hpp"
#include "route_async.hpp"

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
    const uint32_t* stale = nullptr;  // the table's stale word (check_stale)
    // a tick scanned in chunks (wq_route.hip's pipelined heavy tick): bit 0 = start from carry[0..1]
    // ({P, F} of the chunks before), bit 1 = hand {P, F} on in carry (not the last chunk: no
    // offsets[M], no counters)
    uint64_t* carry = nullptr;
    uint32_t chunk = 0;
    // an asynchronous sharded tick's end (route_async.hpp), run by the one-block scan after its counters
    AsyncResultParams ar{};
    bool async_end = false;
    // the caller's counters (wq_route_tick_device), copied from cnt once final (the emit after the
    // scan sets no counter bit), nullable
    wq_route_counters* out = nullptr;
};

// Inclusive wave64 prefix sum of u32 by DPP row shifts and row broadcasts (no LDS round trips).
__device__ __forceinline__ uint32_t wave_incl_scan_u32_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// One pass of the block covers 16,384 tiles (C3's 39,063 take three): wave w scans its 1,024-tile
// chunk as 16 coalesced rows of 64 (row k = tiles chunk + 64k + lane) with a running carry, the
// chunk totals are scanned across the 16 waves in LDS, and the rows are written with the wave's
// offset. Every load and store is one contiguous 256-byte wave access. The prefixes are u32 (as
// the CSR offsets are; they wrap only when P > 2^32 - 1, which error bit 2 reports) and are scanned
// by DPP; P itself is summed exactly in u64. (The first version scanned 64-bit values with
// __shfl_up, 12 LDS permutes per row: 21 us for C2's 3,907 tiles.)
constexpr int kScanRows = 16;

static __global__ __launch_bounds__(kScanThreads) void tile_scan_kernel(TileScanParams p) {
    __shared__ uint32_t s_wave[kScanWaves];
    __shared__ uint64_t s_tot[kScanWaves];
    __shared__ uint64_t s_F[kScanWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t carry = 0, F = 0, F0 = 0;
    if (p.chunk & 1u) {
        carry = p.carry[0];
        F0 = p.carry[1];
    }
    for (uint32_t base = 0; base < p.n_tiles; base += kScanThreads * kScanRows) {
        const uint32_t c0 = base + (uint32_t)wave * (64 * kScanRows) + lane;
        uint32_t v[kScanRows];
        uint64_t lane_sum = 0;
#pragma unroll
        for (int k = 0; k < kScanRows; ++k) {
            const uint32_t i = c0 + 64u * k;
            const bool in = i < p.n_tiles;
            v[k] = in ? p.tile_total[i] : 0u;
            F += in ? p.tile_F[i] : 0u;
        }
        uint32_t run = 0;  // wave-local exclusive prefix of each row element (u32, wrapping)
        uint32_t ex[kScanRows];
#pragma unroll
        for (int k = 0; k < kScanRows; ++k) {
            const uint32_t incl = wave_incl_scan_u32_dpp(v[k]);
            ex[k] = run + incl - v[k];
            run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            lane_sum += v[k];
        }
        const uint64_t wtot = wave_sum_u64(lane_sum);  // exact
        if (lane == 0) {
            s_wave[wave] = run;
            s_tot[wave] = wtot;
        }
        __syncthreads();
        uint32_t before = (uint32_t)carry;
        uint64_t tot = 0;
#pragma unroll
        for (int u = 0; u < kScanWaves; ++u) {
            if (u < wave) before += s_wave[u];
            tot += s_tot[u];
        }
#pragma unroll
        for (int k = 0; k < kScanRows; ++k) {
            const uint32_t i = c0 + 64u * k;
            if (i < p.n_tiles) p.tile_prefix[i] = before + ex[k];
        }
        carry += tot;
        __syncthreads();
    }
    F = wave_sum_u64(F);
    if (lane == 0) s_F[wave] = F;
    __syncthreads();
    if (tid == 0) {
        uint64_t Ft = F0;
#pragma unroll
        for (int u = 0; u < kScanWaves; ++u) Ft += s_F[u];
        if (p.chunk & 2u) {  // a chunk before the last: {P, F} so far to the next chunk's scan
            p.carry[0] = carry;
            p.carry[1] = Ft;
            return;
        }
        p.cnt->n_candidates = Ft;
        const uint64_t P = carry;
        p.offsets[p.M] = (uint32_t)P;
        p.cnt->n_pairs = P;
        // u32 CSR offsets cannot hold more than 2^32-1 pairs: error bit 2
        flag_route(p.cnt, p.health, P > 0xFFFFFFFFull ? 2u : 0u, P > p.capacity ? 1u : 0u);
        if (p.stale && *p.stale) flag_route(p.cnt, p.health, kErrStale, 0u);
        if (p.out) *p.out = *p.cnt;
    }
    if (p.async_end) {  // (never with chunks) the counters above are final: the tick's end, here
        __syncthreads();
        async_result_block(p.ar);
    }
}

// Many tiles (C3: 39,063): one block cannot keep up (the single-block scan above took ~60-76 us
// there whatever its load pattern), so the prefix is rocPRIM's single-pass decoupled look-back
// scan over every CU and this kernel adds what tile_scan_kernel adds: F (candidates) by block
// partial sums into the call's counters, P from the last tile, the overflow / error flags.
static __global__ __launch_bounds__(kBlock) void tile_finish_kernel(TileScanParams p) {
    __shared__ uint64_t s_F[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t F = 0;
    for (uint32_t i = blockIdx.x * kBlock + tid; i < p.n_tiles; i += gridDim.x * kBlock) F += p.tile_F[i];
    F = wave_sum_u64(F);
    if (lane == 0) s_F[wave] = F;
    lds_barrier();
    if (tid == 0) {
        uint64_t Fb = 0;
#pragma unroll
        for (int u = 0; u < kWaves; ++u) Fb += s_F[u];
        atomicAdd(reinterpret_cast<unsigned long long*>(&p.cnt->n_candidates), (unsigned long long)Fb);
    }
    if (blockIdx.x == 0 && tid == 0) {
        const uint32_t last = p.n_tiles - 1;
        const uint64_t P = (uint64_t)p.tile_prefix[last] + p.tile_total[last];  // no u32 wrap below 2^32
        p.offsets[p.M] = (uint32_t)P;
        p.cnt->n_pairs = P;
        flag_route(p.cnt, p.health, P > 0xFFFFFFFFull ? 2u : 0u, P > p.capacity ? 1u : 0u);
        if (p.stale && *p.stale) flag_route(p.cnt, p.health, kErrStale, 0u);
    }
}

// Many tiles in ONE launch: block b scans tiles [4096 b, 4096 b + 4096) (16 consecutive per thread,
// 16-byte loads), publishes its exact {E, F} aggregates as tagged granules, sums every lower block's
// aggregates itself (blocks wait only on lower, already dispatched blocks; C3's 39,063 tiles are 10
// blocks) and writes its prefixes; the last block writes P, F and the flags. It replaces rocPRIM's
// look-back scan + tile_finish_kernel (init, scan and finish: three launches, ~18 us on C3).
constexpr int kMScanThreads = 256;
constexpr int kMScanPer = 16;
constexpr uint32_t kMScanTile = kMScanThreads * kMScanPer;
constexpr uint32_t kSGranTagBits = 24;
constexpr uint32_t kSpinLimitScan = 1u << 21;  // x s_sleep(2) ~ 0.1 s (route_tick.hpp's bound)
constexpr uint32_t kErrSpinScan = 4u;          // error bit 4: a bounded spin gave up (WQ_E_TIMEOUT)

__device__ __forceinline__ uint64_t sgranule(uint32_t tag, uint64_t v) {
    return ((uint64_t)tag << (64 - kSGranTagBits)) | (v & ((1ull << (64 - kSGranTagBits)) - 1ull));
}

static __global__ __launch_bounds__(kMScanThreads) void tile_scan_multi_kernel(TileScanParams p, uint64_t* gran,
                                                                                uint32_t tag) {
    constexpr int NW = kMScanThreads / 64;
    __shared__ uint32_t s_wave[NW];
    __shared__ uint64_t s_e[NW], s_f[NW], s_pe[NW], s_pf[NW];
    __shared__ uint32_t s_gave;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x, n = p.n_tiles;
    const uint32_t t0 = b * kMScanTile + (uint32_t)tid * kMScanPer;
    uint32_t v[kMScanPer];
    uint64_t f = 0;
    if (t0 + kMScanPer <= n) {  // 64-byte aligned runs (t0 is a multiple of 16 tiles)
        const uint4* tv = reinterpret_cast<const uint4*>(p.tile_total + t0);
        const uint4* fv = reinterpret_cast<const uint4*>(p.tile_F + t0);
        uint4 a[kMScanPer / 4], c[kMScanPer / 4];
#pragma unroll
        for (int k = 0; k < kMScanPer / 4; ++k) {
            a[k] = tv[k];
            c[k] = fv[k];
        }
#pragma unroll
        for (int k = 0; k < kMScanPer / 4; ++k) {
            v[4 * k] = a[k].x;
            v[4 * k + 1] = a[k].y;
            v[4 * k + 2] = a[k].z;
            v[4 * k + 3] = a[k].w;
            f += (uint64_t)c[k].x + c[k].y + c[k].z + c[k].w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kMScanPer; ++k) {
            const bool in = t0 + k < n;
            v[k] = in ? p.tile_total[t0 + k] : 0u;
            f += in ? p.tile_F[t0 + k] : 0u;
        }
    }
    uint32_t run = 0;
    uint64_t esum = 0;
#pragma unroll
    for (int k = 0; k < kMScanPer; ++k) {
        const uint32_t x = v[k];
        v[k] = run;  // exclusive within the thread (u32, wrapping like the CSR offsets)
        run += x;
        esum += x;
    }
    const uint32_t incl = wave_incl_scan_u32_dpp(run);
    const uint64_t we = wave_sum_u64(esum), wf = wave_sum_u64(f);
    if (lane == 63) s_wave[wave] = incl;
    if (lane == 0) {
        s_e[wave] = we;
        s_f[wave] = wf;
    }
    if (tid == 0) s_gave = 0;
    __syncthreads();
    uint32_t before = incl - run;
    uint64_t E = 0, F = 0;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        if (u < wave) before += s_wave[u];
        E += s_e[u];
        F += s_f[u];
    }
    if (tid == 0) {  // this block's aggregates, for the blocks above it
        __hip_atomic_store(gran + 2 * b, sgranule(tag, E), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gran + 2 * b + 1, sgranule(tag, F), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the lower blocks' aggregates: thread j polls block j (and j + 256, ...)
    uint64_t pe = 0, pf = 0;
    bool gave = false;
    for (uint32_t j = tid; j < b; j += kMScanThreads) {
        for (int h = 0; h < 2; ++h) {
            const uint64_t* g = gran + 2 * j + h;
            uint64_t x = 0;
            for (uint32_t it = 0;; ++it) {
                x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(x >> (64 - kSGranTagBits)) == tag) break;
                if (it >= kSpinLimitScan) {
                    gave = true;
                    x = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            const uint64_t val = x & ((1ull << (64 - kSGranTagBits)) - 1ull);
            if (h == 0) pe += val;
            else pf += val;
        }
    }
    pe = wave_sum_u64(pe);
    pf = wave_sum_u64(pf);
    if (lane == 0) {
        s_pe[wave] = pe;
        s_pf[wave] = pf;
    }
    if (gave) s_gave = 1;
    __syncthreads();
    uint64_t PE = 0, PF = 0;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        PE += s_pe[u];
        PF += s_pf[u];
    }
    const uint32_t base = (uint32_t)PE + before;
    if (t0 + kMScanPer <= n) {
        uint4* o = reinterpret_cast<uint4*>(p.tile_prefix + t0);
#pragma unroll
        for (int k = 0; k < kMScanPer / 4; ++k)
            o[k] = make_uint4(base + v[4 * k], base + v[4 * k + 1], base + v[4 * k + 2], base + v[4 * k + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < kMScanPer; ++k)
            if (t0 + k < n) p.tile_prefix[t0 + k] = base + v[k];
    }
    if (tid == 0) {
        if (s_gave) flag_route(p.cnt, p.health, kErrSpinScan, 0u);
        if (b == gridDim.x - 1) {
            const uint64_t P = PE + E;
            p.cnt->n_candidates = PF + F;
            p.offsets[p.M] = (uint32_t)P;
            p.cnt->n_pairs = P;
            flag_route(p.cnt, p.health, P > 0xFFFFFFFFull ? 2u : 0u, P > p.capacity ? 1u : 0u);
            if (p.stale && *p.stale) flag_route(p.cnt, p.health, kErrStale, 0u);
            if (p.out) *p.out = *p.cnt;
        }
    }
}

// The same decoupled shape for a plain u32 exclusive scan (out[i] = sum of in[0 .. i), wrapping):
// 4,096 elements per block, each block summing every lower block's tagged total itself. One launch
// instead of rocPRIM's scan (its state init, the scan and its temporary storage).
static __global__ __launch_bounds__(kMScanThreads) void scan_u32_multi_kernel(const uint32_t* __restrict__ in,
                                                                               uint32_t* __restrict__ out, uint32_t n,
                                                                               uint64_t* gran, uint32_t tag,
                                                                               wq_route_counters* err) {
    constexpr int NW = kMScanThreads / 64;
    __shared__ uint32_t s_wave[NW], s_pre[NW];
    __shared__ uint32_t s_gave;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t t0 = b * kMScanTile + (uint32_t)tid * kMScanPer;
    uint32_t v[kMScanPer];
    if (t0 + kMScanPer <= n && (reinterpret_cast<uintptr_t>(in) & 15) == 0) {
        const uint4* iv = reinterpret_cast<const uint4*>(in + t0);
        uint4 a[kMScanPer / 4];
#pragma unroll
        for (int k = 0; k < kMScanPer / 4; ++k) a[k] = iv[k];
#pragma unroll
        for (int k = 0; k < kMScanPer / 4; ++k) {
            v[4 * k] = a[k].x;
            v[4 * k + 1] = a[k].y;
            v[4 * k + 2] = a[k].z;
            v[4 * k + 3] = a[k].w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kMScanPer; ++k) v[k] = t0 + k < n ? in[t0 + k] : 0u;
    }
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < kMScanPer; ++k) {
        const uint32_t x = v[k];
        v[k] = run;
        run += x;
    }
    const uint32_t incl = wave_incl_scan_u32_dpp(run);
    if (lane == 63) s_wave[wave] = incl;
    if (tid == 0) s_gave = 0;
    __syncthreads();
    uint32_t before = incl - run, tot = 0;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
        if (u < wave) before += s_wave[u];
        tot += s_wave[u];
    }
    if (tid == 0) __hip_atomic_store(gran + b, sgranule(tag, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t pe = 0;
    bool gave = false;
    for (uint32_t j = tid; j < b; j += kMScanThreads) {
        uint64_t x = 0;
        for (uint32_t it = 0;; ++it) {
            x = __hip_atomic_load(gran + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(x >> (64 - kSGranTagBits)) == tag) break;
            if (it >= kSpinLimitScan) {
                gave = true;
                x = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        pe += (uint32_t)x;
    }
    pe = (uint32_t)wave_sum_u64(pe);
    if (lane == 0) s_pre[wave] = pe;
    if (gave) s_gave = 1;
    __syncthreads();
    uint32_t base = before;
#pragma unroll
    for (int u = 0; u < NW; ++u) base += s_pre[u];
    if (t0 + kMScanPer <= n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
        uint4* o = reinterpret_cast<uint4*>(out + t0);
#pragma unroll
        for (int k = 0; k < kMScanPer / 4; ++k)
            o[k] = make_uint4(base + v[4 * k], base + v[4 * k + 1], base + v[4 * k + 2], base + v[4 * k + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < kMScanPer; ++k)
            if (t0 + k < n) out[t0 + k] = base + v[k];
    }
    if (tid == 0 && s_gave && err) atomicOr(&err->error, kErrSpinScan);
}

// The multi-block scans' tagged granules (RouteWs::sgran): room for `words`, zeroed when fresh or
// when the tags wrap; returns this launch's tag.
inline int scan_granules(wq_router* h, uint64_t words, uint32_t* tag) {
    RouteWs& rw = h->rws;
    WQ_ALLOC(h, rw.sgran, words * 8);
    const uint64_t period = (1ull << kSGranTagBits) - 1;
    // fresh granules (tag 0 never matches), and all of them again when the tags wrap, so a granule
    // left by a scan 2^24 - 1 calls back can never pass for this call's
    if (rw.sgran_zeroed < words || (rw.scan_calls && rw.scan_calls % period == 0)) {
        WQ_HIP(h, hipMemsetAsync(rw.sgran.p, 0, rw.sgran.bytes, h->stream));
        rw.sgran_zeroed = rw.sgran.bytes / 8;
    }
    *tag = (uint32_t)(rw.scan_calls++ % period) + 1u;
    return WQ_OK;
}

// out[i] = sum of in[0 .. i) (u32, wrapping) in one launch on the handle's stream; a spin that gave
// up (never in practice) sets error bit 4 in *err when given.
inline int launch_scan_u32(wq_router* h, const uint32_t* in, uint32_t* out, uint32_t n, wq_route_counters* err) {
    if (!n) return WQ_OK;
    const uint32_t nb = (n + kMScanTile - 1) / kMScanTile;
    uint32_t tag = 0;
    if (int rc = scan_granules(h, nb, &tag)) return rc;
    hipLaunchKernelGGL(scan_u32_multi_kernel, dim3(nb), dim3(kMScanThreads), 0, h->stream, in, out, n,
                       h->rws.sgran.as<uint64_t>(), tag, err);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

constexpr uint32_t kScanOneBlockMax = 8192;  // tiles: up to here the one-block scan is the faster

// The tick's tile scan (n_tiles >= 1): one block for a few thousand tiles (C2: 3,907),
// rocPRIM + tile_finish_kernel beyond. P must fit the u32 offsets either way (error bit 2 if not);
// a tick of > 2^32 pairs wraps the prefix, which the error bit already reports. With sp.async_end,
// *async_done says whether the scan took the asynchronous tick's end (the one-block scan only).
inline int launch_tile_scan(wq_router* h, const TileScanParams& sp, bool* async_done = nullptr,
                            bool* out_done = nullptr) {
    hipStream_t s = h->stream;
    if (async_done) *async_done = false;
    if (out_done) *out_done = false;
    // the one-block scan below 2,048 tiles, and up to kScanOneBlockMax when it takes an asynchronous
    // tick's end; the multi-block scan otherwise (C3 17.8 -> 8.7 us; an 8-GPU rank's 4,883 tiles
    // 206.8-207.5 -> 205.8-206.3 us per tick, alternating). WQ_SCAN_MULTI_MIN moves the threshold
    static const uint32_t multi_min =
        getenv("WQ_SCAN_MULTI_MIN") ? (uint32_t)strtoul(getenv("WQ_SCAN_MULTI_MIN"), nullptr, 10) : 2048u;
    if (sp.n_tiles <= kScanOneBlockMax && (sp.async_end || sp.n_tiles < multi_min)) {
        hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, sp);
        WQ_HIP(h, hipGetLastError());
        if (async_done) *async_done = sp.async_end;
        if (out_done) *out_done = sp.out != nullptr;
        return WQ_OK;
    }
    // WQ_SCAN_MULTI=0: rocPRIM's look-back scan + tile_finish_kernel (the round-5 path, for A/B)
    static const bool multi = !getenv("WQ_SCAN_MULTI") || atoi(getenv("WQ_SCAN_MULTI")) != 0;
    if (multi) {
        RouteWs& rw = h->rws;
        const uint32_t nb = (sp.n_tiles + kMScanTile - 1) / kMScanTile;
        uint32_t tag = 0;
        if (int rc = scan_granules(h, 2ull * nb, &tag)) return rc;
        hipLaunchKernelGGL(tile_scan_multi_kernel, dim3(nb), dim3(kMScanThreads), 0, s, sp, rw.sgran.as<uint64_t>(), tag);
        WQ_HIP(h, hipGetLastError());
        if (out_done) *out_done = sp.out != nullptr;
        return WQ_OK;
    }
    size_t bytes = 0;
    WQ_HIP(h, rocprim::exclusive_scan(nullptr, bytes, sp.tile_total, sp.tile_prefix, 0u, (size_t)sp.n_tiles,
                                      rocprim::plus<uint32_t>(), s));
    WQ_ALLOC(h, h->rws.scan_tmp, bytes);
    WQ_HIP(h, rocprim::exclusive_scan(h->rws.scan_tmp.p, bytes, sp.tile_total, sp.tile_prefix, 0u,
                                      (size_t)sp.n_tiles, rocprim::plus<uint32_t>(), s));
    const unsigned g = std::min<unsigned>(256u, (sp.n_tiles + kBlock * 8 - 1) / (kBlock * 8));
    hipLaunchKernelGGL(tile_finish_kernel, dim3(g), dim3(kBlock), 0, s, sp);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

}  // namespace wq
