// route_gather.hpp — rows of words gathered from anywhere into one contiguous output.
//
// The sharded tick (wq_sharded.hip) describes every message's recipients, and every cube list an
// owner ships to another GPU, as a row descriptor {len, skip, pointer}: output word k of the row
// is src[k + (k >= skip)] — the cube's list or a record's inline peers with the sender's own
// entry skipped (ExceptSelf), a list copied into a received pool, or the sender itself
// (OnlySelf). gather_rows_kernel writes rows i = 0 .. n-1 contiguously with the owner-map windows
// of emit_map_kernel (route_emit.hpp): per block 256 rows; each row marks where its range enters a
// window of W = R * 256 outputs in a u16 map, a block-wide max-scan carries each owner over its
// outputs, and thread t writes outputs t, t + 256, ... (one contiguous 256-word run per store
// instruction), so the stores stream whatever the row lengths. Two ways to place the rows:
//   CSR = false  row i at start[i] (an exclusive prefix with start[n] = total; its length is
//                start[i + 1] - start[i], so rows of length 0 need no descriptor at all);
//   CSR = true   the message-major CSR: row lengths e[i], the block's first output from the tile
//                scan of the per-256-row totals (route_scan.hpp), the in-block prefix by a row
//                scan; the kernel writes offsets[i] as well (offsets[n] comes from the tile scan).
#pragma once
#include "route_common.hpp"

namespace wq {

struct GatherParams {
    const uint32_t* start;  // CSR = false: exclusive prefix of the row lengths, n + 1 entries
    const uint4* desc;      // {len, skip (kNone: none), pointer lo, pointer hi} per row
    uint32_t n;
    uint32_t* out;
    uint32_t* out_row;      // nullable: the row index of every output word (the CSR's msgs[])
    uint64_t capacity;      // outputs at or beyond it are not written
    // CSR = true
    const uint32_t* e = nullptr;            // row lengths
    const uint32_t* tile_prefix = nullptr;  // exclusive prefix of the 256-row totals
    uint32_t* offsets = nullptr;            // out: offsets[0 .. n)
    // CSR = false, optional: block b's rows go to out[blk_base[b] + (start[i] - start[256 b])], and
    // outputs at or beyond blk_lim[b] are not written (the sharded tick's budgeted pool segments)
    const uint64_t* blk_base = nullptr;
    const uint64_t* blk_lim = nullptr;
};

template <int R>
struct GatherSmem {
    alignas(16) uint4 desc[kBlock];
    alignas(16) uint16_t map[R * kBlock];
    uint32_t wave_max[kWaves];
    uint32_t wave_tot[kWaves];
};

// Per-256-row totals of e (the tile scan's input), for gather_rows_kernel<R, true>.
__global__ __launch_bounds__(kBlock) void row_tile_sums_kernel(const uint32_t* __restrict__ e, uint32_t n,
                                                               uint32_t* __restrict__ tile_total) {
    __shared__ uint64_t part[kWaves];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t s = wave_sum_u64(i < n ? e[i] : 0u);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) t += part[w];
        tile_total[blockIdx.x] = t > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t;
    }
}

template <int R, bool CSR = false>
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(GatherParams p) {
    static_assert(R % 8 == 0, "map rows of whole 16-byte words");
    constexpr uint32_t W = R * kBlock;
    __shared__ GatherSmem<R> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t i0 = blockIdx.x * kBlock;
    const uint32_t i = i0 + tid;
    uint32_t g, T, e, st;
    // the descriptor is loaded first, so its latency hides behind the row scan
    const uint4 d0 = i < p.n ? p.desc[i] : make_uint4(0, kNone, 0, 0);
    if (CSR) {
        e = i < p.n ? p.e[i] : 0u;
        const uint32_t incl = wave_incl_scan_add(e, lane);
        if (lane == 63) sm.wave_tot[wave] = incl;
        lds_barrier();
        uint32_t before = 0;
        T = 0;
#pragma unroll
        for (int u = 0; u < kWaves; ++u) {
            const uint32_t t = sm.wave_tot[u];
            if (u < wave) before += t;
            T += t;
        }
        st = before + incl - e;
        g = p.tile_prefix[blockIdx.x];
        if (i < p.n) p.offsets[i] = g + st;
    } else {
        g = p.start[i0];
        T = p.start[i0 + kBlock < p.n ? i0 + kBlock : p.n] - g;
        e = i < p.n ? p.start[i + 1] - p.start[i] : 0u;
        st = i < p.n ? p.start[i] - g : T;
    }
    if (T == 0 || !p.out) return;  // block-uniform
    uint64_t obase = g, olim = p.capacity;
    if (!CSR && p.blk_base) {
        obase = p.blk_base[blockIdx.x];
        olim = p.blk_lim[blockIdx.x];
    }
    sm.desc[tid] = make_uint4(st, d0.y, d0.z, d0.w);  // (rows of length 0 are never read)
    uint4* my_map = reinterpret_cast<uint4*>(sm.map) + tid * (R / 8);
    for (uint32_t w0 = 0; w0 < T; w0 += W) {
#pragma unroll
        for (int q = 0; q < R / 8; ++q) my_map[q] = make_uint4(0, 0, 0, 0);
        lds_barrier();
        if (e && st + e > w0 && st < w0 + W) sm.map[(st > w0 ? st : w0) - w0] = (uint16_t)(tid + 1);
        lds_barrier();
        uint4 v[R / 8];
#pragma unroll
        for (int q = 0; q < R / 8; ++q) v[q] = my_map[q];
        uint32_t run = 0;
#pragma unroll
        for (int q = 0; q < R / 8; ++q) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&v[q]);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                uint32_t lo = w[hh] & 0xFFFFu, hi = w[hh] >> 16;
                run = lo > run ? lo : run;
                lo = run;
                run = hi > run ? hi : run;
                w[hh] = lo | (run << 16);
            }
        }
        const uint32_t incl = wave_incl_scan_max(run, lane);
        uint32_t pre = __shfl_up(incl, 1, 64);
        if (lane == 0) pre = 0;
        if (lane == 63) sm.wave_max[wave] = incl;
        lds_barrier();
#pragma unroll
        for (int u = 0; u < kWaves; ++u)
            if (u < wave) pre = sm.wave_max[u] > pre ? sm.wave_max[u] : pre;
#pragma unroll
        for (int q = 0; q < R / 8; ++q) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&v[q]);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const uint32_t lo = w[hh] & 0xFFFFu, hi = w[hh] >> 16;
                w[hh] = (lo > pre ? lo : pre) | ((hi > pre ? hi : pre) << 16);
            }
            my_map[q] = v[q];
        }
        lds_barrier();
        const uint32_t last = (T - 1 - w0) < W - 1 ? (T - 1 - w0) : W - 1;
        uint32_t val[R], own[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t x = (uint32_t)(u * kBlock + tid) < last ? (uint32_t)(u * kBlock + tid) : last;
            const uint32_t j = (uint32_t)sm.map[x] - 1u;
            const uint4 dj = sm.desc[j];
            const uint32_t k = w0 + x - dj.x;
            const uint32_t* a = reinterpret_cast<const uint32_t*>(((uint64_t)dj.w << 32) | dj.z);
            val[u] = a[k + (k >= dj.y ? 1u : 0u)];
            own[u] = j;
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t r = w0 + u * kBlock + tid;
            const uint64_t o = obase + r;
            if (r < T && o < olim) {
                p.out[o] = val[u];
                if (p.out_row) p.out_row[o] = i0 + own[u];
            }
        }
        lds_barrier();  // the next window rewrites the map
    }
}

}  // namespace wq
