// route_common.hpp — shared constants and wave/LDS helpers of the route kernels (wq_route.hip).
#pragma once
#include <algorithm>

#include "wq_internal.hpp"

namespace wq {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
// locator (info.x)
constexpr uint32_t kLocGlobal = 0x80000000u;  // offset of the full list in `list`
constexpr uint32_t kLocSelf = 0x40000000u;    // the one recipient is the sender
constexpr uint32_t kLocMask = 0x3FFFFFFFu;    // otherwise: record slot (inline list)
// info.y for an inline record: count << 24 | skipped index (kSkipNone24 = none)
constexpr uint32_t kSkipNone24 = 0xFFFFFFu;
// emit base[]
constexpr uint32_t kGlobal = 0x80000000u;        // index into `list`, not the stage
constexpr uint32_t kSelfSentinel = 0xFFFFFFFFu;  // the recipient is the sender (stage overflow)

__device__ __forceinline__ uint32_t wave_incl_scan_add(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan_max(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v = v > t ? v : t;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Workgroup barrier that orders LDS only: global loads stay in flight across it (a plain
// __syncthreads() also waits vmcnt(0)). No kernel here hands global memory between threads of
// one workgroup.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Message q (0 .. 64*IPT-1) of wave w sits at strided tile index (q/64)*256 + w*64 + q%64.
template <int IPT>
__device__ __forceinline__ uint32_t wave_msg(int wave, uint32_t q) {
    return (q >> 6) * kBlock + wave * 64 + (q & 63);
}

// Error / overflow bits of a route call go to its counters and, sticky across calls, to the
// handle's two health words {error OR, overflow OR} (wq_route_health), so a run of asynchronous
// ticks whose counters were never read back can still be checked afterwards. Only ever reached
// when something is wrong: a normal tick never touches the health words.
__device__ __forceinline__ void flag_route(wq_route_counters* c, uint32_t* health, uint32_t err, uint32_t ovf) {
    if (err) {
        atomicOr(&c->error, err);
        if (health) atomicOr(health, err);
    }
    if (ovf) {
        atomicOr(&c->overflow, ovf);
        if (health) atomicOr(health + 1, ovf);
    }
}

// Error bit 8: the table is missing an incremental batch the device could not apply (keys without
// a packed form, list space); the next host call on the handle re-applies it (wq_delta.hip).
constexpr uint32_t kErrStale = 8u;
__device__ __forceinline__ void check_stale(const TableView& t, wq_route_counters* c, uint32_t* health) {
    if (t.stale && *t.stale) flag_route(c, health, kErrStale, 0u);
}

// Compact message slots of the sharded tick (wq_shard.hip shard_scatter20_kernel): five words each,
// the kind in bits 8-15 of word 4 (its low byte is the replication code).
constexpr int kSlotWords = WQ_SLOT_WORDS;  // include/wq_router.h (the owner form exposes slots)
constexpr uint32_t kSlotReg = 0, kSlotHead = 1, kSlotTail = 2;

// Budgeted slot segments of the sharded tick (wq_shard.hip launch_budget_slots): owner d's slots at
// [base[d], base[d] + budget[d]) of the send buffer.
struct SlotLayout {
    uint32_t base[WQ_MAX_SHARDS + 1];
    uint32_t budget[WQ_MAX_SHARDS];
};
constexpr uint32_t kStBudget = 0x80000000u;  // exchange status bit: some budget of the tick was too small

struct RouteIn {
    const double* pos;
    const int64_t* keys;
    const uint32_t* world;
    const uint32_t* sender;
    const uint8_t* repl;
    uint32_t M;
    int64_t si;
    const uint32_t* slots = nullptr;  // count_kernel<..., SLOTS = true>: M compact slots instead of the above
    uint32_t own_G = 1, own_me = 0;   // count_kernel<..., OWN = true>: count only shard own_me's cubes of own_G
    // count_kernel: when set, the number of messages (slots) is min(M, *m_dev) — a count known on the
    // device only (the sharded tick's own slots)
    const uint32_t* m_dev = nullptr;
};

// info.x of a row the sharded tick's owner shipped back: word offset into the received cube-list
// pool (both locator flags set; only ever decoded when EmitParams::pool is set)
constexpr uint32_t kLocPool = 0xC0000000u;
// ... with the radius filter on: info.y of a pool row of <= kInline peers = kPoolShort | length << 24 |
// survivor mask (emit_row_img stages it like an inline record); a longer row's info.y is its length
constexpr uint32_t kPoolShort = 0x80000000u;

}  // namespace wq
