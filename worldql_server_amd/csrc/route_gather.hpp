// route_gather.hpp — rows of words gathered from anywhere into one contiguous output.
//
// The sharded tick (wq_sharded.hip) describes every message's recipients, and every cube list an
// owner ships to another GPU, as a row descriptor {len, skip, pointer}: output word k of the row
// is src[k + (k >= skip)] — the cube's list or a record's inline peers with the sender's own
// entry skipped (ExceptSelf), a list copied into a received pool, or the sender itself
// (OnlySelf). gather_rows_kernel writes rows i = 0 .. n-1 at out[start[i] ..) with the owner-map
// windows of emit_map_kernel (route_emit.hpp): per block 256 rows; each row marks where its range
// enters a window of W = R * 256 outputs in a u16 map, a block-wide max-scan carries each owner
// over its outputs, and thread t writes outputs t, t + 256, ... (one contiguous 256-word run per
// store instruction), so the stores stream whatever the row lengths.
#pragma once
#include "route_common.hpp"

namespace wq {

struct GatherParams {
    const uint32_t* start;  // exclusive prefix of the row lengths, n + 1 entries (start[n] = total)
    const uint4* desc;      // {len, skip (kNone: none), pointer lo, pointer hi} per row
    uint32_t n;
    uint32_t* out;
    uint32_t* out_row;      // nullable: the row index of every output word (the CSR's msgs[])
    uint64_t capacity;      // outputs at or beyond it are not written
};

template <int R>
struct GatherSmem {
    alignas(16) uint4 desc[kBlock];
    alignas(16) uint16_t map[R * kBlock];
    uint32_t wave_max[kWaves];
};

template <int R>
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(GatherParams p) {
    static_assert(R % 8 == 0, "map rows of whole 16-byte words");
    constexpr uint32_t W = R * kBlock;
    __shared__ GatherSmem<R> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t i0 = blockIdx.x * kBlock;
    const uint32_t i = i0 + tid;
    const uint32_t g = p.start[i0];
    const uint32_t T = p.start[i0 + kBlock < p.n ? i0 + kBlock : p.n] - g;
    if (T == 0) return;  // block-uniform
    const uint4 d = i < p.n ? p.desc[i] : make_uint4(0, kNone, 0, 0);
    const uint32_t e = d.x;
    const uint32_t st = i < p.n ? p.start[i] - g : T;
    sm.desc[tid] = make_uint4(st, d.y, d.z, d.w);
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
            const uint64_t o = (uint64_t)g + r;
            if (r < T && o < p.capacity) {
                p.out[o] = val[u];
                if (p.out_row) p.out_row[o] = i0 + own[u];
            }
        }
        lds_barrier();  // the next window rewrites the map
    }
}

}  // namespace wq
