// route_tick.hpp — the whole tick in ONE launch (see wq_route.hip).
//
// Block b owns messages [b*RC, (b+1)*RC). It
//   1. counts them (count_rows: quantise, probe, sender filter), keeping e_m and the locators in
//      LDS — nothing of the count pass goes through HBM;
//   2. publishes its total as one tagged 8-byte granule {tag, total} (a relaxed agent-scope
//      store: the value is the whole hand-off, so it needs no fence);
//   3. sums the totals of blocks 0..b-1, polling each granule until it carries this call's tag
//      (relaxed agent-scope loads, which bypass the non-coherent L1; bounded, see below);
//   4. emits its rows (emit_row) at that global offset.
// A block waits only on LOWER-numbered blocks, which were dispatched before it: they are resident
// or finished, so the chain always drains (the launcher also sizes the grid to the resident
// capacity). Every poll is bounded: a block that gives up sets counters.error bit 2 and emits at a
// wrong offset instead of hanging the GPU.
// Compared with count / tile_scan / emit launches this removes the e / locator round trip through
// HBM (12 B per message), the scan launch and one launch gap; the tick's only inter-block
// traffic is one 8-byte granule per block (C2: 977 blocks).
#pragma once
#include "route_count.hpp"
#include "route_emit.hpp"

namespace wq {

struct TickParams {
    RouteIn in;
    TableView t;
    uint32_t* offsets;  // out: CSR offsets[0 .. M]
    EmitOut out;        // peers == nullptr: offsets only
    uint64_t* agg;      // [2 * gridDim.x] tagged block totals, then tagged block candidate counts
    uint32_t tag;       // this call's tag (non-zero, differs from the previous call's)
    wq_route_counters* cnt;
    wq_route_counters* cnt_next;
    uint64_t* stamps;   // diagnostics (wq_debug_set_timeline) or nullptr
};

constexpr uint32_t kErrSpin = 4u;
constexpr uint32_t kSpinLimit = 1u << 21;  // x s_sleep(2) ~ 0.1 s, far beyond any tick

__device__ __forceinline__ uint32_t wait_granule(const uint64_t* g, uint32_t tag, bool* gave_up) {
    for (uint32_t it = 0;; ++it) {
        const uint64_t v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(v >> 32) == tag) return (uint32_t)v;
        if (it >= kSpinLimit) {
            *gave_up = true;
            return 0u;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

template <int RC>
struct TickSmem {
    uint32_t e[RC];
    uint2 info[RC];
    uint64_t wave_u64[2][kWaves];
    uint32_t wave_tot[kWaves];
};

template <bool RAW_KEYS, int RC, int STAGE>
__global__ __launch_bounds__(kBlock) void tick_kernel(TickParams p) {
    constexpr int ROWS = RC / kBlock;
    constexpr int G = ROWS < 4 ? ROWS : 4;  // rows counted together (messages per lane)
    static_assert(RC % (G * kBlock) == 0, "RC: whole groups of rows");
    __shared__ TickSmem<RC> sm;
    __shared__ EmitRowSmem<STAGE> es;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t base = b * RC;
    const bool stamp = p.stamps && tid == 0;
    if (stamp) p.stamps[4 * b] = __builtin_amdgcn_s_memrealtime();
    if (b == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }

    // ---- 1. count, G rows at a time ----
    uint64_t F_local = 0;
    uint32_t E_local = 0;
#pragma unroll 1
    for (int r0 = 0; r0 < ROWS; r0 += G) {
        uint32_t e_out[G];
        uint2 inf_out[G];
        count_rows<RAW_KEYS, G>(p.in, p.t, base + r0 * kBlock, e_out, inf_out, F_local, E_local);
#pragma unroll
        for (int i = 0; i < G; ++i) {
            sm.e[(r0 + i) * kBlock + tid] = e_out[i];
            sm.info[(r0 + i) * kBlock + tid] = inf_out[i];
        }
    }
    const uint64_t Fw = wave_sum_u64(F_local);
    const uint64_t Ew = wave_sum_u64(E_local);
    if (lane == 0) {
        sm.wave_u64[0][wave] = Fw;
        sm.wave_u64[1][wave] = Ew;
    }
    lds_barrier();
    uint64_t Fb = 0, Eb = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        Fb += sm.wave_u64[0][w];
        Eb += sm.wave_u64[1][w];
    }
    bool gave_up = false;
    if (stamp) p.stamps[4 * b + 1] = __builtin_amdgcn_s_memrealtime();
    // ---- 2. publish ----
    if (tid == 0) {
        if (Eb > 0xFFFFFFFFull) atomicOr(&p.cnt->error, 2u);  // a block total past u32: offsets cannot hold it
        const uint64_t g = ((uint64_t)p.tag << 32) | (Eb & 0xFFFFFFFFull);
        __hip_atomic_store(p.agg + b, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t f = ((uint64_t)p.tag << 32) | (Fb > 0xFFFFFFFFull ? 0xFFFFFFFFull : Fb);
        __hip_atomic_store(p.agg + gridDim.x + b, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- 3. prefix over lower blocks ----
    // (the last block also sums every block's candidate count for the counters)
    const bool last = b == gridDim.x - 1;
    uint64_t pre = 0, Fall = 0;
    for (uint32_t k = tid; k < b; k += kBlock) pre += wait_granule(p.agg + k, p.tag, &gave_up);
    if (last)
        for (uint32_t k = tid; k < gridDim.x; k += kBlock) Fall += wait_granule(p.agg + gridDim.x + k, p.tag, &gave_up);
    pre = wave_sum_u64(pre);
    Fall = wave_sum_u64(Fall);
    lds_barrier();  // wave_u64 reuse
    if (lane == 0) {
        sm.wave_u64[0][wave] = pre;
        sm.wave_u64[1][wave] = Fall;
    }
    const bool any_gave_up = __syncthreads_or(gave_up);
    pre = 0;
    Fall = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        pre += sm.wave_u64[0][w];
        Fall += sm.wave_u64[1][w];
    }
    if (tid == 0) {
        if (any_gave_up) atomicOr(&p.cnt->error, kErrSpin);
        if (last) {  // the last block knows P and F
            const uint64_t P = pre + Eb;
            p.cnt->n_candidates = Fall;
            p.offsets[p.in.M] = (uint32_t)P;
            p.cnt->n_pairs = P;
            if (P > p.out.capacity) atomicOr(&p.cnt->overflow, 1u);
            if (P > 0xFFFFFFFFull) atomicOr(&p.cnt->error, 2u);  // u32 CSR offsets cannot hold it
        }
    }

    if (stamp) p.stamps[4 * b + 2] = __builtin_amdgcn_s_memrealtime();
    // ---- 4. offsets and emit, one row of 256 messages at a time ----
    uint64_t g = pre;
#pragma unroll 1
    for (int r = 0; r < ROWS; ++r) {
        const uint32_t m0 = base + r * kBlock;
        if (m0 >= p.in.M) break;  // block-uniform
        const uint32_t m = m0 + tid;
        const uint32_t e = sm.e[r * kBlock + tid];
        const uint2 inf = sm.info[r * kBlock + tid];
        uint32_t T;
        const uint32_t st = row_scan(e, sm.wave_tot, &T);
        if (m < p.in.M) p.offsets[m] = (uint32_t)(g + st);
        if (p.out.peers) emit_row<STAGE>(es, p.t, p.out, m0, e, inf, st, g, T);
        else lds_barrier();  // wave_tot reuse
        g += T;
    }
    if (stamp) p.stamps[4 * b + 3] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace wq
