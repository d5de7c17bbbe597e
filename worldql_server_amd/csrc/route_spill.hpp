// route_spill.hpp — the tick as count+spill / tile_scan / copy launches (route config 7).
//
// The single-launch tick (route_tick.hpp) holds each block's LDS image and registers while its
// decoupled look-back waits for the slowest lower-numbered block (C2: ~10 us of a ~22 us block
// lifetime, profiles/r01_tick_timeline.txt). Here no block ever waits on another:
//   A. spill_count_kernel — block b counts its 256 messages from the whole record line (the same
//      count_rows / stage_image as the tick), writes e_m and its block total, and copies its
//      image to a per-block scratch slot [b * STAGE, b * STAGE + T) with 16-byte stores;
//   B. tile_scan_kernel (route_scan.hpp) — exclusive prefix of the block totals, P, counters;
//   C. spill_copy_kernel — block b reloads its slot into LDS (aligned 16-byte loads), writes the
//      CSR offsets and copies the image out exactly as the tick does.
// The records are read once; the extra traffic is the image written and re-read (5 B per
// output), which a recent write leaves in the MALL. A block whose outputs exceed STAGE keeps its
// locators instead and C emits it through emit_row (re-reading its records) — exact either way.
#pragma once
#include "route_scan.hpp"
#include "route_tick.hpp"

namespace wq {

struct SpillParams {
    RouteIn in;
    TableView t;
    EmitOut out;             // peers == nullptr: offsets only
    uint32_t* offsets;       // out: CSR offsets[0 .. M) (C; offsets[M] by the scan)
    uint32_t* e;             // u32[M]: filtered counts, A -> C
    uint2* info;             // uint2[M]: locators of blocks that overflow the image, A -> C
    uint32_t* tile_total;    // per block: outputs (A), scanned by B
    uint32_t* tile_F;        // per block: candidates (A)
    const uint32_t* tile_prefix;  // per block: exclusive prefix (B -> C)
    uint32_t* spill_p;       // [blocks * STAGE] peers of each block's image
    uint8_t* spill_m;        // [blocks * STAGE] ... and their row-local message index
    wq_route_counters* cnt_next;
};

template <bool RAW_KEYS, int STAGE>
__global__ __launch_bounds__(kBlock) void spill_count_kernel(SpillParams p) {
    static_assert(STAGE % 4 == 0, "STAGE: whole 16-byte quads");
    __shared__ TickSmem<STAGE> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t m0 = b * kBlock, m = m0 + tid;
    if (b == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    if (tid == 0) sm.es.q.n_gq = 0;

    uint64_t F_local = 0;
    uint32_t E_local = 0;
    uint32_t e1[1];
    uint2 inf1[1];
    uint4 pc[1][6];
    count_rows<RAW_KEYS, 1, 0, true>(p.in, p.t, m0, e1, inf1, F_local, E_local, pc);
    const uint32_t e = e1[0];
    const uint2 inf = inf1[0];

    const uint64_t Fw = wave_sum_u64(F_local);
    if (lane == 0) sm.wave_u64[wave] = Fw;
    uint32_t T;
    const uint32_t st = row_scan(e, sm.wave_tot, &T);  // its barrier also publishes wave_u64
    if (tid == 0) {
        uint64_t Fb = 0;
#pragma unroll
        for (int u = 0; u < kWaves; ++u) Fb += sm.wave_u64[u];
        p.tile_F[b] = Fb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Fb;
        p.tile_total[b] = T;
    }
    if (m < p.in.M) p.e[m] = e;
    if (!p.out.peers) return;
    if (T <= (uint32_t)STAGE) {  // block-uniform
        stage_image<STAGE>(sm.es, p.t, p.out, m, e, inf, st, pc[0]);
        lds_barrier();
        uint32_t* dp = p.spill_p + (uint64_t)b * STAGE;
        uint8_t* dm = p.spill_m + (uint64_t)b * STAGE;
        // the last quad may carry up to three stale image words: they stay inside this block's slot
        for (uint32_t qd = 4u * tid; qd < T; qd += 4u * kBlock) {
            *reinterpret_cast<uint4*>(dp + qd) = *reinterpret_cast<const uint4*>(&sm.es.op[qd]);
            *reinterpret_cast<uint32_t*>(dm + qd) = *reinterpret_cast<const uint32_t*>(&sm.es.om[qd]);
        }
    } else if (m < p.in.M) {
        p.info[m] = inf;
    }
}

template <int STAGE, int U>
__global__ __launch_bounds__(kBlock) void spill_copy_kernel(SpillParams p) {
    __shared__ TickSmem<STAGE> sm;
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint32_t m0 = b * kBlock, m = m0 + tid;
    const uint32_t e = m < p.in.M ? p.e[m] : 0u;
    uint32_t T;
    const uint32_t st = row_scan(e, sm.wave_tot, &T);
    const uint64_t g0 = p.tile_prefix[b];
    if (m < p.in.M) p.offsets[m] = (uint32_t)(g0 + st);
    if (!p.out.peers) return;
    if (T <= (uint32_t)STAGE) {
        const uint32_t* sp = p.spill_p + (uint64_t)b * STAGE;
        const uint8_t* smm = p.spill_m + (uint64_t)b * STAGE;
        for (uint32_t qd = 4u * tid; qd < T; qd += 4u * kBlock) {
            *reinterpret_cast<uint4*>(&sm.es.op[qd]) = *reinterpret_cast<const uint4*>(sp + qd);
            *reinterpret_cast<uint32_t*>(&sm.es.om[qd]) = *reinterpret_cast<const uint32_t*>(smm + qd);
        }
        lds_barrier();
        copy_image_out<STAGE>(sm.es, p.out, m0, g0, T);
    } else {
        const uint2 inf = m < p.in.M ? p.info[m] : make_uint2(0, kNone);
        emit_row<STAGE, U>(sm.es, p.t, p.out, m0, e, inf, st, g0, T);
    }
}

}  // namespace wq
