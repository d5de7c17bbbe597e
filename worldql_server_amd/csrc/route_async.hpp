// route_async.hpp — the end of an asynchronous sharded tick (wq_sharded.hip): the small exchange
// vectors' layout, and the snapshot that stands in for the end-of-tick read. The tick's tile scan
// runs it in its own block when it takes the whole scan (tile_scan_kernel, route_scan.hpp), so an
// asynchronous tick ends without a launch of its own; otherwise k_async_result does.
#pragma once
#include "route_common.hpp"

namespace wq {

// The small exchange vectors (ShardCtx::small, allocated at attach). Slot tick: A = {slots, status}
// u32 x 2 per shard (send at kSmallA, receive right after), C = {pool words, status} u32 x 2 per
// shard (send at kSmallC, receive right after), and at kSmallCnt four counter blocks: the
// message-side tile scan (P, error / overflow bits), the own-cube count pass, the owner's count pass
// over received slots, and a scratch block (the count kernels' "next call" slot). Status words:
// bits 0-7 the negated WQ_E_* code of a local failure, 8-23 device error bits (8 stale table, 4
// spin, 2 > 2^32 pairs), 31 (kStBudget) an exchange budget was too small. The expanded-return tick
// uses {count, status} u32 x 2 at kSmallA and {pairs, status} u64 x 2 at kSmallC.
constexpr size_t kSmallA = 0, kSmallC = 1024, kSmallCnt = 5120, kSmallBytes = 8192;
constexpr size_t kCntScan = 0, kCntSelf = 1, kCntOwner = 2, kCntScratch = 3;
static_assert(kSmallA + 4 * WQ_MAX_SHARDS * 4 <= kSmallC && kSmallC + 8 * WQ_MAX_SHARDS * 8 <= kSmallCnt &&
                  kSmallCnt + 4 * sizeof(wq_route_counters) <= kSmallBytes,
              "small exchange vector layout");
constexpr uint32_t kStCodeMask = 0xFFu;
// wq_route_health / counters error bits of an asynchronous sharded tick (include/wq_router.h)
constexpr uint32_t kErrShardStep = 32u, kErrRedo = 64u;

struct AsyncResultParams {
    const uint32_t* a_recv;  // 2G words: {slots, status} from every shard
    const uint32_t* c_recv;  // 2G words: {pool words, status} from every shard
    uint32_t G;
    uint32_t statuses;       // the statuses count (G > 1, or the owner form's budgeted self segment)
    const wq_route_counters* cnt;  // the tick's counter blocks (kCntScan, kCntSelf, kCntOwner)
    uint32_t has_msgs;
    uint64_t capacity;
    wq_route_counters* out;  // the caller's (nullable)
    uint32_t* health;        // the handle's sticky words
    const uint32_t* small;   // the tick's small vectors (words; the ones in use: small_word) ...
    uint32_t* snap;          // ... copied here (mapped pinned memory), then the sequence word
    uint64_t seq;
    uint32_t* zero;          // the small vectors, zeroed last for the next tick
};

// The words of the small vectors a tick uses: A and C (4G words each) and the counter blocks.
__device__ __forceinline__ uint32_t small_word(uint32_t k, uint32_t G) {
    const uint32_t ac = 4 * G;
    return k < ac ? kSmallA / 4 + k : k < 2 * ac ? kSmallC / 4 + (k - ac) : kSmallCnt / 4 + (k - 2 * ac);
}

// (asynchronous tick; one whole block, after every write to the small vectors) what the synchronous
// tick reads back, folded on the device into the caller's counters and the sticky health words: P,
// a shard's failed step (32), the device bits of every shard's statuses and counters, a budget that
// was too small (64: the outputs are not valid; every shard sees it and the next call runs exact).
// The snapshot goes to mapped pinned memory, then its sequence word (system-scope release), and the
// small vectors are zeroed for the next tick.
__device__ inline void async_result_block(const AsyncResultParams& p) {
    // only the words in use cross PCIe (the vectors' 8 KB would be ~20 times as many)
    const uint32_t nw = 8 * p.G + (uint32_t)(4 * sizeof(wq_route_counters) / 4);
    for (uint32_t k = threadIdx.x; k < nw; k += blockDim.x) {
        const uint32_t i = small_word(k, p.G);
        p.snap[i] = p.small[i];
    }
    __threadfence_system();  // every thread's part of the snapshot visible to the host ...
    __syncthreads();
    if (threadIdx.x == 0) {  // ... before the sequence word
        __hip_atomic_store(reinterpret_cast<uint64_t*>(p.snap + kSmallBytes / 4), p.seq, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t err = 0;
        for (uint32_t d = 0; p.statuses && d < p.G; ++d) {
            for (uint32_t st : {p.a_recv[2 * d + 1], p.c_recv[2 * d + 1]}) {
                if (st & kStCodeMask) err |= kErrShardStep;
                err |= (st >> 8) & 0xFFFFu;
                if (st & kStBudget) err |= kErrRedo;
            }
        }
        err |= p.cnt[kCntScan].error | p.cnt[kCntSelf].error | p.cnt[kCntOwner].error;
        const uint64_t P = p.has_msgs ? p.cnt[kCntScan].n_pairs : 0;
        const uint32_t ovf = P > p.capacity ? 1u : 0u;
        if (p.out) {
            p.out->n_pairs = P;
            p.out->n_candidates = p.has_msgs ? p.cnt[kCntScan].n_candidates : 0;
            p.out->overflow = ovf;
            p.out->error = err;
        }
        if (err) atomicOr(p.health, err);
        if (ovf) atomicOr(p.health + 1, 1u);
    }
    __syncthreads();
    // the small vectors zeroed for the next tick (here, rather than a memset launch at its start)
    for (uint32_t k = threadIdx.x; k < nw; k += blockDim.x) p.zero[small_word(k, p.G)] = 0u;
}

}  // namespace wq
