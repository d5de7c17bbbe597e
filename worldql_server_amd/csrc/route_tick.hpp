// route_tick.hpp — the whole tick in ONE launch and ONE pass over the record lines.
//
// The three-launch tick (count / tile_scan / emit) reads every message's record line twice; at
// ~50 G random lines/s that second pass alone costs ~20 us of a C2 tick. Here block b owns the
// 256 messages [256b, 256b + 256) and
//   1. counts them, one lane per message (count_rows: quantise, probe, sender filter);
//   2. scans e over the block (row-local output positions) and publishes its total as a tagged
//      8-byte granule {tag, A, total} — decoupled look-back, Merrill & Garland;
//   3. stages its outputs in LDS in output order while that granule propagates: the count read
//      each message's whole record line in one round (lane per message), so the lane already
//      holds the peers and writes each quad of them with one 16-byte and one 4-byte LDS store
//      (the four peers and their message index); the sender's skipped entry, long lists (the
//      block copies them from `list`) and OnlySelf take slower paths;
//   4. looks back over the lower blocks' granules, 64 per wave instruction, summing aggregates
//      until the nearest inclusive prefix, and publishes its own inclusive prefix {tag, P, ...};
//   5. writes CSR offsets and copies the image out in 16-byte quads aligned to the global
//      output (the block's first and last quads, shared with its neighbours, word by word).
// A block waits only on LOWER-numbered blocks, dispatched before it and therefore resident or
// finished, so the chain always drains. Every poll is bounded: a block that gives up sets
// counters.error bit 2 and writes at a wrong offset instead of hanging the GPU.
// A block whose outputs exceed the LDS image (skewed fan-out) emits through emit_row, which
// re-reads its records window by window — exact either way.
#pragma once
#include "route_count.hpp"
#include "route_emit.hpp"

namespace wq {

struct TickParams {
    RouteIn in;
    TableView t;
    uint32_t* offsets;  // out: CSR offsets[0 .. M]
    EmitOut out;        // peers == nullptr: offsets only
    uint64_t* look;     // [gridDim.x] look-back granules
    uint64_t* fgran;    // [gridDim.x] tagged per-block candidate counts (summed by the last block)
    uint32_t tag;       // this call's tag, 1 .. 2^30-1, differs from the previous call's
    wq_route_counters* cnt;
    wq_route_counters* cnt_next;
    uint32_t* health;   // sticky {error, overflow} words (flag_route)
    uint64_t* stamps;  // diagnostics (wq_debug_set_timeline) or nullptr
    uint32_t n_tiles;   // 256-message tiles (one block each)
    // the caller's counters (wq_route_tick_device): the last block copies cnt there once it is final,
    // instead of a copy launch after the tick; nullable
    wq_route_counters* out_cnt = nullptr;
};

constexpr uint32_t kErrSpin = 4u;
constexpr uint32_t kSpinLimit = 1u << 21;  // x s_sleep(2) ~ 0.1 s, far beyond any tick
constexpr uint32_t kFlagA = 1u, kFlagP = 2u;

// granule: [tag:30][flag:2][value:32]
__device__ __forceinline__ uint64_t granule(uint32_t tag, uint32_t flag, uint32_t v) {
    return ((uint64_t)((tag << 2) | flag) << 32) | v;
}

__device__ __forceinline__ uint64_t poll_granule(const uint64_t* g, uint32_t tag, bool* gave_up) {
    for (uint32_t it = 0;; ++it) {
        const uint64_t v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(v >> 34) == tag) return v;
        if (it >= kSpinLimit) {
            *gave_up = true;
            return granule(tag, kFlagP, 0);
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Exclusive prefix of block b's total over blocks 0 .. b-1 (called by one whole wave; b > 0).
__device__ __forceinline__ uint64_t look_back(const uint64_t* look, uint32_t b, uint32_t tag, bool* gave_up) {
    const int lane = threadIdx.x & 63;
    uint64_t acc = 0;
    for (int64_t hi = (int64_t)b - 1; hi >= 0; hi -= 64) {
        const int64_t idx = hi - lane;  // lane 0 = the nearest block
        uint64_t v = 0;
        if (idx >= 0) v = poll_granule(look + idx, tag, gave_up);
        const uint32_t flag = (uint32_t)(v >> 32) & 3u;
        const uint64_t pm = __ballot(idx >= 0 && flag == kFlagP);
        const int first = pm ? __builtin_ctzll(pm) : 64;  // nearest inclusive prefix
        const uint64_t x = (lane <= first && idx >= 0) ? (uint32_t)v : 0u;
        acc += wave_sum_u64(x);
        if (pm) break;
    }
    return acc;
}

template <int STAGE>
struct TickSmem {
    EmitRowSmem<STAGE> es;  // image (op / om) + long-list queue; also the fallback's LDS
    uint32_t wave_tot[kWaves];
    uint64_t wave_u64[kWaves];
    uint64_t pre;
};

typedef uint32_t u32x4_lds __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32_a1 __attribute__((aligned(1)));

// Stage the block's outputs in the LDS image in output order (caller: T <= STAGE, every thread
// of the block, sm.q.n_gq zeroed and a barrier passed since). Inline records: the lane holds its
// cube's peers in registers (pc) and writes each quad of them with one 16-byte and one 4-byte LDS
// store; the sender's skipped entry, long lists (copied from `list` by the whole block) and
// OnlySelf take slower paths. Ends with the image complete up to the caller's next barrier.
template <int STAGE>
__device__ __forceinline__ void stage_image(EmitRowSmem<STAGE>& es, const TableView& tv, const EmitOut& out,
                                            uint32_t m, uint32_t e, uint2 inf, uint32_t st, const uint4 (&pc)[6]) {
    const int tid = threadIdx.x;
    const bool self = e && (inf.x & kLocSelf);
    uint32_t slot = kNone, meta = 0;
    if (e && !self) {
        if (inf.x & kLocGlobal) {
            const uint32_t q = atomicAdd(&es.q.n_gq, 1u);
            es.q.gq_j[q] = tid;
            es.q.gq_off[q] = (inf.x & ~kLocGlobal) + 1;
            es.q.gq_skip[q] = inf.y;
            es.q.gq_e[q] = e;
            es.q.gq_st[q] = st;
        } else {
            const uint32_t s24 = inf.y & kSkipNone24;
            slot = inf.x;
            meta = (inf.y >> 24) | ((s24 == kSkipNone24 ? 0xFFu : s24) << 8);
        }
    }
    if (self) {
        es.op[st] = out.sender[m];
        es.om[st] = (uint8_t)tid;
    }
    if (slot != kNone) {  // inline record: the peers are in this lane's registers
        const uint32_t cnt = meta & 0xFF, skip = meta >> 8;
        const uint8_t j = (uint8_t)tid;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t i0 = 4u * k;  // first peer index of chunk 2 + k
            if (i0 >= cnt) continue;
            const uint4 c = pc[k];
            if (i0 + 4 <= cnt && (skip == 0xFFu || skip < i0)) {
                // four peers, none of them the sender: one quad
                const uint32_t pos = st + i0 - (skip != 0xFFu ? 1u : 0u);
                *reinterpret_cast<u32x4_lds*>(&es.op[pos]) = u32x4_lds{c.x, c.y, c.z, c.w};
                *reinterpret_cast<u32_a1*>(&es.om[pos]) = 0x01010101u * j;
            } else {
                const uint32_t vv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t idx = i0 + i;
                    if (idx >= cnt || idx == skip) continue;
                    const uint32_t pos = st + idx - (skip != 0xFFu && idx > skip ? 1u : 0u);
                    es.op[pos] = vv[i];
                    es.om[pos] = j;
                }
            }
        }
    }
    lds_barrier();  // the long-list queue is complete
    const uint32_t n_gq = es.q.n_gq;
    for (uint32_t q = 0; q < n_gq; ++q) {
        const uint32_t j = es.q.gq_j[q], s0 = es.q.gq_st[q], ej = es.q.gq_e[q];
        const uint32_t off = es.q.gq_off[q], sk = es.q.gq_skip[q];
        for (uint32_t k = tid; k < ej; k += kBlock) {
            es.op[s0 + k] = tv.list[off + k + (k >= sk ? 1u : 0u)];
            es.om[s0 + k] = (uint8_t)j;
        }
    }
}

// Copy a complete image of T outputs to the global output at g0 (every thread of the block; the
// image is complete and a barrier passed): 16-byte quads aligned to the global output, the
// block's first and last quads (shared with its neighbours) word by word.
template <int STAGE, bool NT = false>
__device__ __forceinline__ void copy_image_out(const EmitRowSmem<STAGE>& es, const EmitOut& out, uint32_t m0,
                                               uint64_t g0, uint32_t T) {
    const int tid = threadIdx.x;
    const uint64_t gA = g0 & ~3ull;
    const uint32_t lead = (uint32_t)(g0 - gA);
    const uint32_t span = lead + T;
    for (uint32_t qd = 4u * tid; qd < span; qd += 4u * kBlock) {
        // image index of global output gA + qd + i is qd + i - lead
        const uint64_t out0 = gA + qd;
        if (qd >= lead && qd + 4 <= span && out0 + 4 <= out.capacity) {
            const u32x4_lds pv = *reinterpret_cast<const u32x4_lds*>(&es.op[qd - lead]);
            const uint32_t mv = *reinterpret_cast<const u32_a1*>(&es.om[qd - lead]);
            const uint4 pq = make_uint4(pv.x, pv.y, pv.z, pv.w);
            const uint4 mq = make_uint4(m0 + (mv & 0xFF), m0 + ((mv >> 8) & 0xFF), m0 + ((mv >> 16) & 0xFF), m0 + (mv >> 24));
            if (NT) {  // streamed: nothing on the GPU reads the pairs back in this tick
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(v4u{pq.x, pq.y, pq.z, pq.w}, reinterpret_cast<v4u*>(out.peers + out0));
                if (out.msgs)
                    __builtin_nontemporal_store(v4u{mq.x, mq.y, mq.z, mq.w}, reinterpret_cast<v4u*>(out.msgs + out0));
            } else {
                *reinterpret_cast<uint4*>(out.peers + out0) = pq;
                if (out.msgs) *reinterpret_cast<uint4*>(out.msgs + out0) = mq;
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                if (qd + i >= lead && qd + i < span && out0 + i < out.capacity) {
                    out.peers[out0 + i] = es.op[qd + i - lead];
                    if (out.msgs) out.msgs[out0 + i] = m0 + es.om[qd + i - lead];
                }
            }
        }
    }
}

template <bool RAW_KEYS, int STAGE, int U, bool NT = false>
__global__ __launch_bounds__(kBlock) void tick_kernel(TickParams p) {
    // U: record lines in flight per lane in the fallback emit_row
    static_assert(STAGE % 4 == 0, "STAGE: whole 16-byte quads");
    __shared__ TickSmem<STAGE> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TableView& tv = p.t;
    const uint32_t b = blockIdx.x, NB = gridDim.x;
    const uint32_t m0 = b * kBlock, m = m0 + tid;
    const bool stamp = p.stamps && tid == 0;
    if (stamp) p.stamps[4 * b] = __builtin_amdgcn_s_memrealtime();
    if (b == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    if (tid == 0) sm.es.q.n_gq = 0;

    // ---- 1. count ----
    uint64_t F_local = 0;
    uint32_t E_local = 0;
    uint32_t e1[1];
    uint2 inf1[1];
    uint4 pc[1][6];  // the message's peer chunks (inline records): staged from registers below
    count_rows<RAW_KEYS, 1, 0, true>(p.in, tv, m0, e1, inf1, F_local, E_local, pc);
    const uint32_t e = e1[0];
    const uint2 inf = inf1[0];

    // ---- 2. row scan, publish the aggregate ----
    const uint64_t Fw = wave_sum_u64(F_local);
    if (lane == 0) sm.wave_u64[wave] = Fw;
    uint32_t T;
    const uint32_t st = row_scan(e, sm.wave_tot, &T);
    if (tid == 0) {
        uint64_t Fb = 0;
#pragma unroll
        for (int u = 0; u < kWaves; ++u) Fb += sm.wave_u64[u];
        __hip_atomic_store(p.fgran + b, granule(p.tag, kFlagA, Fb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Fb),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p.look + b, granule(p.tag, b == 0 ? kFlagP : kFlagA, T), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (stamp) p.stamps[4 * b + 1] = __builtin_amdgcn_s_memrealtime();

    // ---- 3. stage the block's outputs in LDS (if they fit) ----
    const bool fits = T <= (uint32_t)STAGE && p.out.peers;  // block-uniform
    if (fits) stage_image<STAGE>(sm.es, tv, p.out, m, e, inf, st, pc[0]);
    else if (p.out.peers) direct_meta(sm.es, p.out, m, e, inf, st);

    // ---- 4. look-back (wave 0), publish the inclusive prefix ----
    if (wave == 0) {
        bool gave_up = false;
        uint64_t pre = 0;
        if (b > 0) {
            pre = look_back(p.look, b, p.tag, &gave_up);
            if (lane == 0) {
                __hip_atomic_store(p.look + b, granule(p.tag, kFlagP, (uint32_t)(pre + T)), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (b == NB - 1 && lane == 0) {  // the last block knows P
            const uint64_t P = pre + T;
            p.offsets[p.in.M] = (uint32_t)P;
            p.cnt->n_pairs = P;
            // u32 CSR offsets cannot hold more than 2^32-1 pairs: error bit 2
            flag_route(p.cnt, p.health, P > 0xFFFFFFFFull ? 2u : 0u, P > p.out.capacity ? 1u : 0u);
            check_stale(tv, p.cnt, p.health);
        }
        if (__any(gave_up) && lane == 0) flag_route(p.cnt, p.health, kErrSpin, 0u);
        if (lane == 0) sm.pre = pre;
    }
    if (b == NB - 1) {  // ... and sums every block's candidate count, all four waves polling
        bool gave_up = false;
        uint64_t F = 0;
        for (uint32_t k = tid; k < NB; k += kBlock) F += (uint32_t)poll_granule(p.fgran + k, p.tag, &gave_up);
        F = wave_sum_u64(F);
        const bool any_gave_up = __any(gave_up);  // the whole wave votes, not lane 0 alone
        if (lane == 0) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.cnt->n_candidates), (unsigned long long)F);
            if (any_gave_up) flag_route(p.cnt, p.health, kErrSpin, 0u);
        }
    }
    lds_barrier();
    if (b == NB - 1 && p.out_cnt) {  // block-uniform: every wave's counter atomics drained first
        __syncthreads();
        if (tid == 0) {
            wq_route_counters c;
            c.n_pairs = __hip_atomic_load(&p.cnt->n_pairs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c.n_candidates = __hip_atomic_load(&p.cnt->n_candidates, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c.overflow = __hip_atomic_load(&p.cnt->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c.error = __hip_atomic_load(&p.cnt->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *p.out_cnt = c;
        }
    }
    const uint64_t g0 = sm.pre;
    if (stamp) p.stamps[4 * b + 2] = __builtin_amdgcn_s_memrealtime();

    // ---- 5. offsets, copy-out ----
    if (m < p.in.M) p.offsets[m] = (uint32_t)(g0 + st);
    if (p.out.peers) {
        if (fits) copy_image_out<STAGE, NT>(sm.es, p.out, m0, g0, T);
        else emit_direct<4>(sm.es, tv, p.out, m0, g0, T);
    }
    if (stamp) p.stamps[4 * b + 3] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace wq
