// wq_delta.hip — incremental subscribe / unsubscribe batches (SURVEY.md §8(d) C4 churn) and
// REMOVE_PEER in place (§8(f) F3).
//
// Same semantics as the full rebuild in wq_table.hip — per (world, cube, peer) the last op of the
// batch wins (AreaMap::add_subscription / remove_subscription, area_map.rs:72-119, applied in
// order by thread.rs:122-146) — but the work is proportional to the batch and the cubes it
// touches, not to the whole table. Three steps, no host read-back between them:
//   events   each op -> packed cube key and its record slot (a new cube claims its record here,
//            count 0); the op becomes one u64 sort key  slot << 33 | kind << 32 | peer
//   bucket   a stable LSD radix sort (k_sort_*: two passes of <= 8 bits) over the slot's high
//            bits: a bucket (2^lowbits adjacent slots, ~100-200 ops at C5) is contiguous, in op order
//   apply    one wave per bucket: the bucket's ops (windows of 256) sorted in registers by (slot,
//            peer, op) with a bitonic network, then one LANE per touched cube: it stages the cube's
//            list in LDS, counts adds / removes (the last op of a peer wins), merges straight into
//            the list (in place, or relocated to bump-allocated space when it outgrows its
//            capacity) and rewrites the record's count, signature, capacity and inline peers.
//            Cubes with more than kLaneList peers go to the whole wave (ranks by binary search).
// A cube that empties keeps its record (count 0, key kept), so every probe sequence stays intact.
// The sorted state `st` and the any-keys are left stale and regenerated from the records only
// when something needs them (table_materialize / table_ensure_any). A batch holding an op without
// a packed key is not applied (the caller rebuilds); one whose relocations would overflow `list`
// is applied except for the cubes that did not fit — re-applying the whole batch in the rebuild
// is exact, since a batch fixes the final state of every (cube, peer) it touches.
#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "lane_xchg.hpp"
#include "table_prims.hpp"

namespace wq {

namespace {

// Device-side status of one batch (read back once, after the apply).
struct DeltaStatus {
    uint32_t flags;     // 1: an op without a packed key; 2: an invalid op; 4: relocations overflowed `list`
    uint32_t n_wave;    // cubes the wave path took
    uint64_t new_recs;  // records claimed by this batch's new cubes
    uint64_t bump;      // list words bump-allocated past t.list_used
    uint64_t pad;
};

struct DeltaTable {
    Record* recs;
    uint32_t* rclaim;
    uint64_t rmask;
    int rshift;
    uint64_t hmask;
    uint32_t* list;
};

__device__ __forceinline__ void op_key(const wq_op& o, double sf, int64_t si, int64_t* k) {
    if (o.key_is_raw) {  // impl ToCubeArea for CubeArea: identity (cube_area.rs:65-70)
        k[0] = o.u.key[0];
        k[1] = o.u.key[1];
        k[2] = o.u.key[2];
    } else {  // CubeArea::from_vector3 (cube_area.rs:50-56)
        k[0] = coord_clamp_dev(o.u.pos[0], sf, si);
        k[1] = coord_clamp_dev(o.u.pos[1], sf, si);
        k[2] = coord_clamp_dev(o.u.pos[2], sf, si);
    }
}

// Per op: packed key and the record slot of its cube — a cube the table does not hold yet gets
// its record here, count 0 (the caller guarantees free slots: load <= 1/2).
// Claim words (rclaim, one per record slot): 0 free, kClaiming while an op writes a new cube's key,
// otherwise the slot holds a key — builds write the cube index + 2 (< 2^31), a delta batch writes
// its tag (kBatchTag | batch number). The 96-bit key spans two words of the record: the claimer
// writes both, then publishes its tag (release). A reader takes the record line first (one line
// per op in the common case): its own key -> found; a visible other key -> the next slot, unless
// this very batch is claiming or has claimed the slot (then the claim word decides, after an
// acquire fence); ext == 0 -> the slot looks free, and the claim word is the arbiter.
constexpr uint32_t kClaiming = 1u, kBatchTag = 0x80000000u;
constexpr uint64_t kNoKey = ~0ull;  // an op without a record: sorts after every real slot

__global__ void k_delta_events(const wq_op* __restrict__ ops, uint32_t n, double sf, int64_t si, Record* recs,
                               uint32_t* rclaim, uint32_t tag, uint64_t rmask, int rshift, uint64_t hmask,
                               uint64_t* keys, DeltaStatus* status) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const wq_op o = ops[i];
    int64_t k[3];
    op_key(o, sf, si, k);
    uint64_t p = 0;
    uint32_t x = 0;
    uint64_t key = kNoKey;
    if (o.kind > WQ_OP_UNSUBSCRIBE || o.world == WQ_WORLD_INVALID) {
        atomicOr(&status->flags, 2u);  // bad op
    } else if (!pack_key(o.world, k[0], k[1], k[2], sf, &p, &x)) {
        atomicOr(&status->flags, 1u);
    } else {
        uint64_t j = slot_of(rec_hash(p, x) & hmask, rshift);
        for (;;) {
            const uint32_t* line = reinterpret_cast<const uint32_t*>(recs + j);
            uint64_t rp = *reinterpret_cast<const uint64_t*>(line);
            uint32_t rx = line[7];
            if (rp == p && rx == x) break;
            uint32_t c;
            if (rx == 0) {  // looks free: claim it (or learn who did)
                c = __hip_atomic_load(&rclaim[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (c == 0) c = atomicCAS(&rclaim[j], 0u, kClaiming);
                if (c == 0) {  // won: a new cube (count 0) with this key
                    recs[j].pk = p;
                    recs[j].ext = x;
                    __hip_atomic_store(&rclaim[j], tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    atomicAdd(reinterpret_cast<unsigned long long*>(&status->new_recs), 1ull);
                    break;
                }
            } else {  // another key is visible: final unless this batch is claiming the slot
                c = __hip_atomic_load(&rclaim[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (c == kClaiming) continue;  // being claimed: look again
            if (c == tag) {                // claimed by this batch: order the key loads after the tag
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                rp = __hip_atomic_load(&recs[j].pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                rx = __hip_atomic_load(&recs[j].ext, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (rp == p && rx == x) break;
            }
            j = (j + 1) & rmask;
        }
        key = (j << 33) | ((uint64_t)(o.kind == WQ_OP_SUBSCRIBE ? 1u : 0u) << 32) | o.peer;
    }
    keys[i] = key;
}

// Bucket b = sorted keys whose slot >> lowbits is b: bstart[b] = first such index (b <= NBr;
// bstart[NBr] ends the real slots, kNoKey ops follow). One flat pass over the sorted keys: thread i
// sees the buckets of keys i - 1 and i and writes the starts of the buckets between them (a
// binary search per bucket instead was ~20 dependent loads: 7.6 us for C4's 4,096 buckets).
__global__ void k_bucket_bounds(const uint64_t* __restrict__ keys, uint32_t n, int lowbits, uint32_t NBr,
                                uint32_t* bstart) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i > n) return;
    const int sh = 33 + lowbits;
    const int64_t cur = i < n ? (int64_t)std::min<uint64_t>(keys[i] >> sh, NBr) : (int64_t)NBr + 1;
    const int64_t prev = i > 0 ? (int64_t)std::min<uint64_t>(keys[i - 1] >> sh, NBr) : -1;
    for (int64_t b = prev + 1; b <= cur && b <= (int64_t)NBr; ++b) bstart[b] = i;
}

// End of a batch, one thread: snapshot {status, stat deltas} straight into the host's pinned
// buffer (no copy launch), zero both for the next batch, mark the table stale if the batch was not
// fully applied (the host re-applies it), and switch the peer boxes off (subscribes may widen
// them; per-op box atomics cost more than they save, so the count pass searches every long list
// until the next build). (Folding this into the last bucket block by a done-counter was measured:
// one agent-scope fence and same-address atomic per block made C5's update 0.78 -> 3.1 ms — each
// fence writes the XCD's L2 back.)
__global__ void k_delta_finish(DeltaStatus* status, int64_t* dstat, uint64_t* snap, uint32_t* stale,
                               uint32_t* pbox_valid) {
    const uint64_t* sw = reinterpret_cast<const uint64_t*>(status);
#pragma unroll
    for (int i = 0; i < 4; ++i) snap[i] = sw[i];
    snap[4] = (uint64_t)dstat[0];
    snap[5] = (uint64_t)dstat[1];
    if (status->flags) *stale = 1u;
    if (pbox_valid) *pbox_valid = 0u;
    *status = DeltaStatus{};
    dstat[0] = 0;
    dstat[1] = 0;
}

// ---- shared helpers (bucket apply, REMOVE_PEER) ---------------------------------------------
constexpr int kG = 16;
constexpr int kGroups = kBlock / kG;
constexpr uint32_t kGroupGrid = 2048;

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lds_lower_bound(const uint32_t* a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Adds per-block entry / live-cube deltas (REMOVE_PEER) into the running totals.
__global__ __launch_bounds__(kBlock) void k_delta_stats(const uint64_t* __restrict__ part, uint32_t nb,
                                                        uint64_t* dstat) {
    __shared__ unsigned long long acc[2];
    if (threadIdx.x < 2) acc[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long v0 = 0, v1 = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += kBlock) {
        v0 += part[2ull * b];
        v1 += part[2ull * b + 1];
    }
    if (v0) atomicAdd(&acc[0], v0);
    if (v1) atomicAdd(&acc[1], v1);
    __syncthreads();
    if (threadIdx.x == 0) {
        dstat[0] += acc[0];
        dstat[1] += acc[1];
    }
}


// ---- the bucket apply: one wave per bucket, one lane per touched cube ------------------------
constexpr int kWin = 256;        // ops per window (a bucket's ops are taken in op-order windows)
constexpr uint32_t kInlineOnly = 0xFFFFFFFEu;  // a round cube's new list fits the record: no list write
constexpr int kLaneList = 256;         // old lists longer than this go to the wave path
// RW (the bucket kernel's template argument): a round stages at most RW old-list words (and 64
// cubes), and the wave path stages lists of up to RW words in LDS. 1024 (16 KB of LDS per wave, 155
// VGPRs: 10 waves per CU) or 256 (11.2 KB, 119 VGPRs: 14 waves per CU), chosen per batch from the
// table's mean list length (table_apply_delta below).

__device__ __forceinline__ uint32_t grown(uint32_t n) { return n + n / 2 + 4; }

template <uint32_t RW>
struct BucketLds {
    uint64_t op[kWin];              // the window's ops, sorted: slot_lo << 48 | peer << 16 | pos << 8 | kind
    uint32_t lst[RW];      // a round's staged old lists (flat), or the wave path's one list
    union {
        struct {                    // a round
            uint16_t wf[RW];  // staged word: bit 15 removed, bits 9-14 its cube in the round, 0-8 adds placed right before it
            uint8_t fl[kWin];          // per op: 1 add / 2 remove
            uint16_t at[kWin];         // per op: #old peers below it
            uint16_t pa[kWin + 1];     // exclusive prefix of add flags over the round's ops
            uint16_t pr[kWin + 1];     // exclusive prefix of remove flags
        } r;
        uint32_t ar[2 * kWin];      // wave path: the cube's adds [0, kWin) and removes [kWin, 2 kWin)
    } u;
    uint32_t hoc[kWin];             // window: per cube, old count (prefetched headers)
    uint32_t hoff[kWin];            // window: per cube, list offset
    uint32_t hcap[kWin];            // window: per cube, list capacity
    uint64_t csrc[64];              // round: per cube, where its old peers are (inline words or list)
    uint64_t csig[64];              // round: per cube, OR of peer_sig over its new list
    uint32_t cpre[65];              // round: per cube, first staged word
    uint32_t cdst[64];              // round: per cube, where the new list goes (kNone: unchanged)
    uint32_t cslot[64];             // round: per cube, its record slot
    uint16_t cR[64];                // round: per cube, removed staged words before its first word
    uint16_t cA[64];                // round: per cube, adds placed before its first word
    uint64_t smask[RW / 64];  // round: bit x = staged word x starts a cube's list
    uint16_t mcum[RW / 64];   // round: list starts in the mask words before this one
    uint8_t su[64];                 // round: the cubes with staged words, in order
    uint64_t bigm[kWin / 64];       // window: cubes (cs index) the wave path takes
    uint16_t cs[kWin + 1];          // cube starts in op[]
    uint8_t cid[kWin];              // per op: its cube (window-local index mod 256)
};

// The round cube owning staged word x (the last list start at or before x).
template <uint32_t RW>
__device__ __forceinline__ uint32_t owner_of(const BucketLds<RW>& sm, uint32_t x) {
    const uint32_t j = x >> 6;
    const uint64_t upto = (2ull << (x & 63)) - 1ull;  // bits 0..x & 63 (all ones for bit 63)
    return sm.su[sm.mcum[j] + (uint32_t)__popcll(sm.smask[j] & upto) - 1];
}

// a[r] of lane (lane ^ j), j a power of two below 64 (a constant once the sort is unrolled)
__device__ __forceinline__ uint64_t xchg_dyn_u64(uint64_t v, int j, int lane) {
    switch (j) {
        case 1: return xchg_u64<1>(v, lane);
        case 2: return xchg_u64<2>(v, lane);
        case 4: return xchg_u64<4>(v, lane);
        case 8: return xchg_u64<8>(v, lane);
        case 16: return xchg_u64<16>(v, lane);
        default: return xchg_u64<32>(v, lane);
    }
}

// Bitonic sort of 64 * E u64 held strided (element r * 64 + lane in a[r]) by one wave, ascending.
template <int E>
__device__ __forceinline__ void wave_bitonic(uint64_t (&a)[4], int lane) {
    constexpr int P = 64 * E;
#pragma unroll
    for (int k = 2; k <= P; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {  // partner: same lane, register r ^ (j / 64)
#pragma unroll
                for (int r = 0; r < E; ++r) {
                    const int r2 = r ^ (j >> 6);
                    if (r2 > r) {
                        const bool up = ((r * 64 + lane) & k) == 0;
                        const uint64_t x = a[r], y = a[r2];
                        const bool sw = up ? (x > y) : (x < y);
                        a[r] = sw ? y : x;
                        a[r2] = sw ? x : y;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < E; ++r) {
                    const uint64_t o = xchg_dyn_u64(a[r], j, lane);
                    const bool up = ((r * 64 + lane) & k) == 0;
                    const bool keep_min = ((lane & j) == 0) == up;
                    a[r] = keep_min ? (o < a[r] ? o : a[r]) : (o > a[r] ? o : a[r]);
                }
            }
        }
    }
}

__device__ __forceinline__ uint32_t op_peer(uint64_t x) { return (uint32_t)(x >> 16); }

// lower_bound of v in a[0, n), n <= N, in log2(N) branch-free steps (independent searches of one
// lane can overlap: no loop-carried control flow).
template <int N>
__device__ __forceinline__ uint32_t lds_lower_bound_fixed(const uint32_t* a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, len = n;
#pragma unroll
    for (int s = N; s > 1; s >>= 1) {
        const uint32_t half = len >> 1;
        const bool right = half && a[lo + half - 1] < v;
        lo += right ? half : 0u;
        len = right ? len - half : (half ? half : len);
    }
    return (len && a[lo] < v) ? lo + 1 : lo;
}


// Inclusive wave64 prefix sum by DPP row shifts and row broadcasts (no LDS round trips).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// ---- the bucket sort: stable LSD radix passes over the sort key's bucket field --------------
// Per pass (digit = kSortBits or fewer bits): a per-tile digit histogram (tile = 4096 keys in op
// order), a per-digit exclusive scan over the tiles, and a stable scatter in which each tile's
// block ranks its keys round by round (a wave matches equal digits by ballots, the four waves'
// counts are combined per digit in LDS). Two passes cover the <= 16 bucket bits.
constexpr int kSortTile = 4096;
constexpr int kSortPer = kSortTile / kBlock;  // keys per thread per tile

// Exclusive prefix of v over a 256-thread block (sc: 4 words of LDS); *total = the block's sum.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* sc, uint32_t* total) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t incl = wave_incl_scan_dpp(v);
    if (lane == 63) sc[wave] = incl;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint32_t x = sc[w];
        pre += w < wave ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return pre + incl - v;
}

__global__ __launch_bounds__(kBlock) void k_sort_hist(const uint64_t* __restrict__ keys, uint32_t n, int sh,
                                                      uint32_t dmask, uint32_t ntiles, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[256];
    const int t = threadIdx.x;
    h[t] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    // clamped, unconditional loads: all kSortPer in flight (a load under a per-lane branch gets its
    // own vmcnt(0) wait, and the 16 loads completed one after another)
    uint64_t kk[kSortPer];
#pragma unroll
    for (int r = 0; r < kSortPer; ++r) {
        const uint64_t i = base + (uint64_t)r * kBlock + t;
        kk[r] = keys[i < n ? i : (uint64_t)n - 1];
    }
    uint32_t d[kSortPer];
#pragma unroll
    for (int r = 0; r < kSortPer; ++r) {
        const uint64_t i = base + (uint64_t)r * kBlock + t;
        d[r] = i < n ? (uint32_t)(kk[r] >> sh) & dmask : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int r = 0; r < kSortPer; ++r)
        if (d[r] != 0xFFFFFFFFu) atomicAdd(&h[d[r]], 1u);
    __syncthreads();
    if ((uint32_t)t <= dmask) cnt[(uint64_t)t * ntiles + blockIdx.x] = h[t];
}

// One block per digit: its row of tile counts -> exclusive prefixes (in place), and the total.
__global__ __launch_bounds__(kBlock) void k_sort_rowscan(uint32_t* __restrict__ cnt, uint32_t ntiles,
                                                         uint32_t* __restrict__ tot) {
    __shared__ uint32_t sc[kBlock / 64];
    uint32_t* row = cnt + (uint64_t)blockIdx.x * ntiles;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < ntiles; c0 += kBlock) {
        const uint32_t j = c0 + threadIdx.x;
        const uint32_t v = j < ntiles ? row[j] : 0u;
        uint32_t s;
        const uint32_t ex = block_excl_scan256(v, sc, &s);
        if (j < ntiles) row[j] = carry + ex;
        carry += s;
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

// Each wave ranks a quarter of the tile (1024 consecutive keys, 64 per round) against its own
// digit counters (no block barrier per round); the quarters are then combined per digit, the
// tile's keys staged in LDS in digit order, and written out in runs (a digit's keys of one tile
// are contiguous in the output).
__global__ __launch_bounds__(kBlock) void k_sort_scatter(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                         uint32_t n, int sh, uint32_t dmask, int dbits,
                                                         uint32_t ntiles, const uint32_t* __restrict__ rowpre,
                                                         const uint32_t* __restrict__ tot) {
    constexpr int NW = kBlock / 64, QR = kSortTile / kBlock;  // waves; rounds per wave
    __shared__ uint64_t stage[kSortTile];
    __shared__ uint32_t gbase[256], lstart[256], wcnt[NW][256], sc[NW];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t tile = blockIdx.x;
    {
        const bool dig = (uint32_t)t <= dmask;
        const uint64_t rp = (uint64_t)t * ntiles + tile;
        const uint32_t cur = dig ? rowpre[rp] : 0u;
        const uint32_t nxt = dig ? (tile + 1 < ntiles ? rowpre[rp + 1] : tot[t]) : 0u;
        uint32_t s0, s1;
        const uint32_t gex = block_excl_scan256(dig ? tot[t] : 0u, sc, &s0);
        const uint32_t lex = block_excl_scan256(nxt - cur, sc, &s1);  // this tile's keys of digit t
        gbase[t] = gex + cur;
        lstart[t] = lex;
#pragma unroll
        for (int w = 0; w < NW; ++w) wcnt[w][t] = 0;
    }
    const uint64_t t0 = (uint64_t)tile * kSortTile;
    const uint32_t cnt = (uint32_t)min((uint64_t)kSortTile, (uint64_t)n - t0);
    const uint32_t q0 = (uint32_t)wave * (kSortTile / NW);  // this wave's quarter
    uint64_t k[QR];
#pragma unroll
    for (int r = 0; r < QR; ++r) {
        const uint32_t i = q0 + r * 64 + lane;
        k[r] = i < cnt ? in[t0 + i] : 0ull;
    }
    __syncthreads();
    uint32_t lr[QR];
#pragma unroll
    for (int r = 0; r < QR; ++r) {
        const bool valid = q0 + r * 64 + lane < cnt;
        const uint32_t d = (uint32_t)(k[r] >> sh) & dmask;
        uint64_t eq = __ballot(valid);
        for (int b = 0; b < dbits; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            eq &= bit ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(eq & lt);
        const uint32_t old = valid ? wcnt[wave][d] : 0u;
        lr[r] = old + rank;
        wave_lds_sync();
        if (valid && rank == 0) wcnt[wave][d] = old + (uint32_t)__popcll(eq);
        wave_lds_sync();
    }
    __syncthreads();
    if ((uint32_t)t <= dmask) {  // per digit: the waves' counts -> their exclusive prefixes
        uint32_t acc = lstart[t];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint32_t c = wcnt[w][t];
            wcnt[w][t] = acc;
            acc += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < QR; ++r) {
        const bool valid = q0 + r * 64 + lane < cnt;
        const uint32_t d = (uint32_t)(k[r] >> sh) & dmask;
        if (valid) stage[wcnt[wave][d] + lr[r]] = k[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < QR; ++r) {
        const uint32_t j = r * kBlock + t;
        if (j < cnt) {
            const uint64_t x = stage[j];
            const uint32_t d = (uint32_t)(x >> sh) & dmask;
            out[gbase[d] + (j - lstart[d])] = x;
        }
    }
}

// Record words 2..6 {count, list_off, sig lo, sig hi, cap} of slot.
__device__ __forceinline__ void write_header(Record* rec, uint32_t nc, uint32_t off, uint64_t sig, uint32_t cap) {
    uint32_t* rw = reinterpret_cast<uint32_t*>(rec);
    *reinterpret_cast<uint2*>(rw + 2) = make_uint2(nc, off);
    *reinterpret_cast<uint2*>(rw + 4) = make_uint2((uint32_t)sig, (uint32_t)(sig >> 32));
    rw[6] = cap;
}

struct BucketArgs {
    DeltaTable tb;
    const uint64_t* keys;    // sorted by slot >> lowbits, stable
    const uint32_t* bstart;  // [NBr + 1]
    int lowbits;
    DeltaStatus* status;
    int64_t* dstat;          // running {entries, live cubes} deltas
    uint64_t list_base;      // first free list word (t.list_used)
    uint64_t list_room;      // words available past list_base
    uint64_t* stamps;        // diagnostics (WQ_DELTA_STAMPS): per bucket, cycles per phase
    uint32_t nb;             // buckets
};

// Diagnostic phase stamps of the bucket apply (lane 0 of each wave; WQ_DELTA_STAMPS only).
#define WQ_STAMP(k)                                                            \
    do {                                                                       \
        if (a.stamps && lane == 0) {                                           \
            const uint64_t t_now = __builtin_amdgcn_s_memtime();               \
            a.stamps[(uint64_t)B * 16 + (k)] += t_now - t_last;                \
            t_last = t_now;                                                    \
        }                                                                      \
    } while (0)

// Relocation space for `want` words (overflow: kNone, flag 4 — the cube is left unchanged).
__device__ __forceinline__ uint32_t bump_alloc(const BucketArgs& a, uint32_t want) {
    const uint64_t d = atomicAdd(reinterpret_cast<unsigned long long*>(&a.status->bump), (unsigned long long)want);
    if (d + want > a.list_room) {
        atomicOr(&a.status->flags, 4u);
        return kNone;
    }
    return (uint32_t)(a.list_base + d);
}

template <uint32_t RW>
__global__ __launch_bounds__(64) void k_delta_bucket(BucketArgs a) {
    __shared__ BucketLds<RW> sm;
    constexpr uint32_t kLL = RW < (uint32_t)kLaneList ? RW : (uint32_t)kLaneList;  // lane-path lists: <= kLL peers
    const uint32_t flags = a.status->flags;
    if (flags & 3u) return;  // an op without a record: nothing applied, the rebuild takes the batch
    const int lane = threadIdx.x;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint64_t lowmask = (1ull << a.lowbits) - 1ull;
    uint32_t* L = a.tb.list;
    int64_t de = 0, dl = 0;
    uint32_t nwave = 0;
    // buckets blockIdx.x, + gridDim.x, ... (the launch gives each wave one or more buckets)
    for (uint32_t B = blockIdx.x; B < a.nb; B += gridDim.x) {
    const uint32_t s = a.bstart[B], e = a.bstart[B + 1];
    uint64_t t_last = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    if (B != blockIdx.x) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    for (uint32_t w0 = s; w0 < e; w0 += kWin) {
        if (w0 != s) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // this wave's own earlier writes: same CU, same L2
        const uint32_t cnt = min((uint32_t)kWin, e - w0);
        // the window's keys: clamped, unconditional loads (all four in flight; loads in per-lane
        // branches each got their own vmcnt(0) wait)
        uint64_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t q = r * 64 + lane;
            v[r] = a.keys[w0 + (q < cnt ? q : 0u)];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t q = r * 64 + lane;
            const uint64_t k = v[r];
            v[r] = q < cnt ? ((((k >> 33) & lowmask) << 48) | ((uint64_t)(uint32_t)k << 16) | ((uint64_t)q << 8) |
                              ((k >> 32) & 1u))
                           : ~0ull;
        }
        if (cnt <= 64)
            wave_bitonic<1>(v, lane);
        else if (cnt <= 128)
            wave_bitonic<2>(v, lane);
        else
            wave_bitonic<4>(v, lane);
        WQ_STAMP(0);
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.op[r * 64 + lane] = v[r];
        wave_lds_sync();
        // cube heads -> cs
        uint32_t ncub = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t q = r * 64 + lane;
            const bool hd = q < cnt && (q == 0 || (sm.op[q] >> 48) != (sm.op[q - 1] >> 48));
            const uint64_t m = __ballot(hd);
            if (hd) sm.cs[ncub + __popcll(m & lt)] = (uint16_t)q;
            if (q < cnt) sm.cid[q] = (uint8_t)(ncub + __popcll(m & (lt | (1ull << lane))) - 1);
            ncub += (uint32_t)__popcll(m);
        }
        if (lane == 0) sm.cs[ncub] = (uint16_t)cnt;
        if (lane < kWin / 64) sm.bigm[lane] = 0;
        wave_lds_sync();
        // every cube's header at once (up to four record lines per lane in flight)
        {
            uint2 hw[4];
            uint32_t hc[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // clamped, no per-lane branch: the rows' loads in flight together
                if ((uint32_t)r * 64 >= ncub) break;  // (wave-uniform)
                const uint32_t c = r * 64 + lane, cc = c < ncub ? c : 0u;
                const uint32_t slot = (B << a.lowbits) | (uint32_t)(sm.op[sm.cs[cc]] >> 48);
                const uint32_t* rw = reinterpret_cast<const uint32_t*>(a.tb.recs + slot);
                hw[r] = *reinterpret_cast<const uint2*>(rw + 2);
                hc[r] = rw[6];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t c = r * 64 + lane;
                if (c < ncub) {
                    sm.hoc[c] = hw[r].x;
                    sm.hoff[c] = hw[r].y;
                    sm.hcap[c] = hc[r];
                }
            }
        }
        WQ_STAMP(1);
        wave_lds_sync();
        // ---- rounds of up to 64 cubes, data-parallel ----
        // One lane per cube reads its header; the round's old lists are staged flat into LDS; each
        // op (the last of its peer run decides) finds its peer by binary search in its cube's
        // list; ballot prefixes over the ops give every peer's new index (old index - removes
        // below + adds below); kept and added peers are written straight to their places in the
        // (in-place or relocated) list and the record's inline words; one lane per cube finishes
        // the header. Lists longer than kLaneList go to the wave path below.
        uint32_t nbig = 0;
        for (uint32_t c0 = 0, n_round = 0; c0 < ncub; c0 += n_round) {
            const uint32_t c = c0 + lane;
            bool act = c < ncub;
            uint32_t slot = 0, oc = 0, off = 0, cap = 0;
            if (act) {
                slot = (B << a.lowbits) | (uint32_t)(sm.op[sm.cs[c]] >> 48);
                oc = sm.hoc[c];
                off = sm.hoff[c];
                cap = sm.hcap[c];
            }
            const uint64_t src_base = reinterpret_cast<uint64_t>(
                oc <= (uint32_t)kInline ? reinterpret_cast<const uint32_t*>(a.tb.recs + slot) + kInlineWord0 : L + off + 1);
            bool isbig = act && oc > kLL;
            uint32_t oc_st = isbig ? 0u : oc;
            const uint32_t incl = wave_incl_scan_dpp(oc_st);
            // the round: the cubes whose staged words fit RW (at least one: oc <= kLaneList)
            n_round = (uint32_t)__popcll(__ballot(act && incl <= RW));
            act = act && (uint32_t)lane < n_round;
            isbig = isbig && act;
            oc_st = act ? oc_st : 0u;
            const uint32_t pre = incl - oc_st;
            if (act) sm.cpre[lane] = pre;
            if (lane == (int)n_round - 1) sm.cpre[n_round] = incl;
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)n_round - 1);
            const uint32_t qa0 = sm.cs[c0], qb0 = sm.cs[c0 + n_round];
            if (act) {
                sm.csrc[lane] = src_base;
                sm.cslot[lane] = slot;
            }
            // owner map: a bit at each staged list's first word, the cubes with words in order
            if (lane < (int)(RW / 64)) sm.smask[lane] = 0;
            wave_lds_sync();
            {
                const bool has = oc_st > 0;  // (implies act)
                const uint64_t mh = __ballot(has);
                if (has) {
                    sm.su[__popcll(mh & lt)] = (uint8_t)lane;
                    atomicOr(reinterpret_cast<unsigned long long*>(&sm.smask[pre >> 6]), 1ull << (pre & 63));
                }
            }
            wave_lds_sync();
            {
                const uint32_t pc = lane < (int)(RW / 64) ? (uint32_t)__popcll(sm.smask[lane]) : 0u;
                const uint32_t ic = wave_incl_scan_dpp(pc);
                if (lane < (int)(RW / 64)) sm.mcum[lane] = (uint16_t)(ic - pc);
            }
            wave_lds_sync();
            WQ_STAMP(2);
            // stage the round's old lists flat: all of the round's loads in flight at once
            // (T <= RW: RW / 64 per lane)
            {
                // owners and source addresses first (LDS only), then every global load: the
                // sources are global memory (record inline words or `list`), so they are read as
                // such — a flat load would also count in lgkmcnt, and each LDS wait would then wait
                // for the loads issued before it
                typedef const __attribute__((address_space(1))) uint32_t* gptr;
                uint32_t val[RW / 64];
                uint64_t src[RW / 64];
#pragma unroll
                for (int r = 0; r < (int)(RW / 64); ++r) {
                    const uint32_t x = r * 64 + lane;
                    src[r] = 0;
                    if (x < T) {
                        const uint32_t u = owner_of(sm, x);
                        src[r] = sm.csrc[u] + 4ull * (x - sm.cpre[u]);
                        sm.u.r.wf[x] = (uint16_t)(u << 9);  // the owner rides along (bits 9-14)
                    }
                }
#pragma unroll
                for (int r = 0; r < (int)(RW / 64); ++r) {
                    const uint32_t x = r * 64 + lane;
                    val[r] = x < T ? *reinterpret_cast<gptr>(src[r]) : 0u;
                }
#pragma unroll
                for (int r = 0; r < (int)(RW / 64); ++r) {
                    const uint32_t x = r * 64 + lane;
                    if (x < T) sm.lst[x] = val[r];
                }
            }
            wave_lds_sync();
            WQ_STAMP(3);
            // per op of the round: the deciding op of each peer run (the last), present or not
            for (uint32_t q0 = qa0; q0 < qb0; q0 += 64) {
                const uint32_t q = q0 + lane;
                if (q < qb0) {
                    const uint64_t x = sm.op[q];
                    const uint32_t pp = op_peer(x);
                    const bool last = q + 1 == qb0 || (sm.op[q + 1] >> 16) != (x >> 16);  // cube and peer
                    const uint32_t lo = (uint32_t)sm.cid[q] - c0;  // the op's cube within the round
                    const uint32_t b0 = sm.cpre[lo], n0 = sm.cpre[lo + 1] - b0;
                    uint8_t f = 0;
                    uint32_t l2 = 0;
                    if (last) {  // (a wave-path cube stages nothing: n0 = 0, and its cdst is kNone)
                        l2 = lds_lower_bound_fixed<kLL>(sm.lst + b0, n0, pp);
                        const bool present = l2 < n0 && sm.lst[b0 + l2] == pp;
                        const uint32_t wpos = b0 + l2;
                        uint32_t* wf32 = reinterpret_cast<uint32_t*>(sm.u.r.wf) + (wpos >> 1);
                        if ((x & 1u) && !present) {
                            f = 1;
                            // an add lands right before old word l2 (none after the last one)
                            if (l2 < n0) atomicAdd(wf32, 1u << (16 * (wpos & 1u)));
                        }
                        if (!(x & 1u) && present) {
                            f = 2;
                            atomicOr(wf32, 0x8000u << (16 * (wpos & 1u)));
                        }
                    }
                    sm.u.r.fl[q - qa0] = f;
                    sm.u.r.at[q - qa0] = (uint16_t)l2;
                }
            }
            // exclusive prefixes of the add / remove flags over the round's ops
            {
                uint32_t ra = 0, rr = 0;
                for (uint32_t q0 = 0; q0 < qb0 - qa0; q0 += 64) {
                    const uint32_t q = q0 + lane;
                    const uint8_t f = q < qb0 - qa0 ? sm.u.r.fl[q] : 0;
                    const uint64_t ma = __ballot(f == 1), mr = __ballot(f == 2);
                    if (q < qb0 - qa0) {
                        sm.u.r.pa[q] = (uint16_t)(ra + __popcll(ma & lt));
                        sm.u.r.pr[q] = (uint16_t)(rr + __popcll(mr & lt));
                    }
                    ra += (uint32_t)__popcll(ma);
                    rr += (uint32_t)__popcll(mr);
                }
                if (lane == 0) {
                    sm.u.r.pa[qb0 - qa0] = (uint16_t)ra;
                    sm.u.r.pr[qb0 - qa0] = (uint16_t)rr;
                }
            }
            wave_lds_sync();
            WQ_STAMP(4);
            // one lane per cube: new count, destination
            uint32_t nc = oc, dst = kNone, ncap = cap;
            if (act && isbig) sm.cdst[lane] = kNone;
            if (act && !isbig) {
                const uint32_t s0 = sm.cs[c] - qa0, s1 = sm.cs[c + 1] - qa0;
                const uint32_t nadd = sm.u.r.pa[s1] - sm.u.r.pa[s0], nrm = sm.u.r.pr[s1] - sm.u.r.pr[s0];
                nc = oc + nadd - nrm;
                if (nadd | nrm) {
                    // <= kInline peers: the record's inline words only (the list block, if any,
                    // goes stale); longer: the whole list rewritten, in place or relocated
                    dst = nc <= (uint32_t)kInline ? kInlineOnly : off;
                    if (nc > (uint32_t)kInline && nc > cap) {
                        ncap = grown(nc);
                        dst = bump_alloc(a, 1 + ncap);
                    }
                    if (dst != kNone) {
                        de += (int64_t)nc - (int64_t)oc;
                        dl += (int64_t)(oc == 0 && nc > 0) - (int64_t)(oc > 0 && nc == 0);
                    }
                }
                sm.cdst[lane] = dst;
                sm.csig[lane] = 0;
            }
            wave_lds_sync();
            WQ_STAMP(6);
            // kept old peers: new index = old index - removed words below it + adds placed at or
            // below it, both from flat prefix sums over the round's staged words less their value
            // at the cube's first word. Eight chunks of 64 words at a time (independent chains).
            {
                constexpr int NG = 2;
                uint32_t cr = 0, ca = 0;
#pragma unroll 1
                for (uint32_t g0 = 0; g0 < T; g0 += NG * 64) {
                    uint32_t rex[NG], aex[NG], wv[NG];
                    uint64_t sm_m[NG];
#pragma unroll
                    for (int r = 0; r < NG; ++r) {  // the chunks' mark words and list-start masks at once
                        const uint32_t x = g0 + r * 64 + lane;
                        wv[r] = x < T ? (uint32_t)sm.u.r.wf[x] : 0u;
                        sm_m[r] = sm.smask[(x >> 6) < RW / 64 ? (x >> 6) : 0u];
                    }
#pragma unroll
                    for (int r = 0; r < NG; ++r) {
                        const uint32_t w = wv[r];
                        const uint64_t mr = __ballot(w >> 15);
                        const uint32_t ac = w & 0x1FFu;  // adds placed before it (<= kWin)
                        const uint32_t ainc = wave_incl_scan_dpp(ac);
                        rex[r] = cr + (uint32_t)__popcll(mr & lt);
                        // bit 31 removed, 25-30 owner cube, 16-24 ac, 0-15 adds before the word
                        aex[r] = (ca + ainc - ac) | (w & 0x8000u) << 16 | ((w >> 9) & 0x3Fu) << 25 | ac << 16;
                        cr += (uint32_t)__popcll(mr);
                        ca += (uint32_t)__builtin_amdgcn_readlane((int)ainc, 63);
                    }
#pragma unroll
                    for (int r = 0; r < NG; ++r) {
                        const uint32_t x = g0 + r * 64 + lane;
                        if (x < T && ((sm_m[r] >> lane) & 1ull)) {
                            const uint32_t u = (aex[r] >> 25) & 0x3Fu;
                            sm.cR[u] = (uint16_t)rex[r];
                            sm.cA[u] = (uint16_t)aex[r];
                        }
                    }
                    wave_lds_sync();
                    // every LDS read of the NG chunks first (one round trip), then the stores
                    uint32_t cd[NG], cy[NG], cp[NG], cq[NG], cz[NG], cl[NG];
#pragma unroll
                    for (int r = 0; r < NG; ++r) {
                        const uint32_t x = g0 + r * 64 + lane;
                        const uint32_t u = (aex[r] >> 25) & 0x3Fu;  // (0 past T)
                        cd[r] = sm.cdst[u];
                        cy[r] = sm.lst[x < (uint32_t)RW ? x : 0u];
                        cp[r] = sm.cpre[u];
                        cq[r] = sm.cR[u];
                        cz[r] = sm.cA[u];
                        cl[r] = sm.cslot[u];
                    }
#pragma unroll
                    for (int r = 0; r < NG; ++r) {
                        const uint32_t x = g0 + r * 64 + lane;
                        const uint32_t u = (aex[r] >> 25) & 0x3Fu, d = cd[r], y = cy[r];
                        if (x >= T || (aex[r] >> 31) || d == kNone) continue;
                        const uint32_t ax = aex[r] & 0xFFFFu, ac = (aex[r] >> 16) & 0x1FFu;
                        const uint32_t k = (x - cp[r]) - (rex[r] - cq[r]) + (ax + ac - cz[r]);
                        if (d != kInlineOnly) L[d + 1 + k] = y;
                        if (k < (uint32_t)kInline) reinterpret_cast<uint32_t*>(a.tb.recs + cl[r])[kInlineWord0 + k] = y;
                        atomicOr(reinterpret_cast<unsigned long long*>(&sm.csig[u]), (unsigned long long)peer_sig(y));
                    }
                }
            }
            WQ_STAMP(7);
            // added peers: new index = #old below - removes below + adds below
            for (uint32_t q = lane; q < qb0 - qa0; q += 64) {
                if (sm.u.r.fl[q] != 1) continue;
                const uint32_t u = (uint32_t)sm.cid[qa0 + q] - c0, d = sm.cdst[u];
                if (d == kNone) continue;
                const uint32_t s0 = sm.cs[c0 + u] - qa0;
                const uint32_t y = op_peer(sm.op[qa0 + q]);
                const uint32_t k = sm.u.r.at[q] - (sm.u.r.pr[q] - sm.u.r.pr[s0]) + (sm.u.r.pa[q] - sm.u.r.pa[s0]);
                if (d != kInlineOnly) L[d + 1 + k] = y;
                if (k < (uint32_t)kInline) reinterpret_cast<uint32_t*>(a.tb.recs + sm.cslot[u])[kInlineWord0 + k] = y;
                atomicOr(reinterpret_cast<unsigned long long*>(&sm.csig[u]), (unsigned long long)peer_sig(y));
            }
            wave_lds_sync();
            WQ_STAMP(8);
            // one lane per cube: count word, header, inline padding
            if (act && !isbig && dst != kNone) {
                if (dst != kInlineOnly) L[dst] = nc;
                Record* rec = a.tb.recs + slot;
                write_header(rec, nc, dst != kInlineOnly ? dst : off, sm.csig[lane], ncap);
                uint32_t* inl = reinterpret_cast<uint32_t*>(rec) + kInlineWord0;
                for (uint32_t k = nc; k < min(oc, (uint32_t)kInline); ++k) inl[k] = kNone;  // beyond oc: kNone already
            }
            if (isbig) atomicOr(reinterpret_cast<unsigned long long*>(&sm.bigm[c >> 6]), 1ull << (c & 63));
            nbig += (uint32_t)__popcll(__ballot(isbig));
            wave_lds_sync();  // the next round restages lst
        }
        wave_lds_sync();
        WQ_STAMP(9);
        // ---- wave path: lists longer than kLaneList, one cube at a time ----
        uint32_t bj = 0;
        uint64_t brem = sm.bigm[0];
        for (uint32_t bi = 0; bi < nbig; ++bi) {
            while (!brem) brem = sm.bigm[++bj];
            const uint32_t c = bj * 64 + (uint32_t)__builtin_ctzll(brem);
            brem &= brem - 1ull;
            const uint32_t qa = sm.cs[c], qb = sm.cs[c + 1];
            const uint32_t slot = (B << a.lowbits) | (uint32_t)(sm.op[qa] >> 48);
            Record* rec = a.tb.recs + slot;
            const uint4 h0 = reinterpret_cast<const uint4*>(rec)[0];
            const uint32_t oc = h0.z, off = h0.w, cap = reinterpret_cast<const uint32_t*>(rec)[6];
            const bool staged = oc <= RW;
            const uint32_t* G = L + off + 1;
            if (staged)
                for (uint32_t i = lane; i < oc; i += 64) sm.lst[i] = G[i];
            wave_lds_sync();
            const uint32_t* O = staged ? sm.lst : G;  // the old list (LDS or global)
            uint32_t nadd = 0, nrm = 0;
            for (uint32_t t0 = qa; t0 < qb; t0 += 64) {
                const uint32_t t = t0 + lane;
                bool is_add = false, is_rm = false;
                uint32_t pp = 0;
                if (t < qb) {
                    const uint64_t x = sm.op[t];
                    pp = op_peer(x);
                    if (t + 1 == qb || op_peer(sm.op[t + 1]) != pp) {
                        uint32_t lo = 0, hi = oc;
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (O[mid] < pp) lo = mid + 1; else hi = mid;
                        }
                        const bool present = lo < oc && O[lo] == pp;
                        is_add = (x & 1u) && !present;
                        is_rm = !(x & 1u) && present;
                    }
                }
                const uint64_t ma = __ballot(is_add), mr = __ballot(is_rm);
                if (is_add) sm.u.ar[nadd + __popcll(ma & lt)] = pp;
                if (is_rm) sm.u.ar[kWin + nrm + __popcll(mr & lt)] = pp;
                nadd += (uint32_t)__popcll(ma);
                nrm += (uint32_t)__popcll(mr);
            }
            wave_lds_sync();
            if ((nadd | nrm) && !staged && oc + nadd - nrm <= cap) {
                // a list longer than the LDS in place: compaction of the removals (forward, 64
                // words at a time: a word only moves down), then the adds opened up backwards (a
                // word only moves up), then the adds themselves
                const uint32_t nc = oc + nadd - nrm;
                const uint32_t* A = sm.u.ar;
                const uint32_t* R = sm.u.ar + kWin;
                uint32_t* W = L + off + 1;
                uint32_t* inl = reinterpret_cast<uint32_t*>(rec) + kInlineWord0;
                uint32_t gone = 0;
                for (uint32_t c0 = 0; c0 < oc; c0 += 64) {
                    const uint32_t i = c0 + lane;
                    const uint32_t y = i < oc ? W[i] : 0u;
                    const uint32_t r = lds_lower_bound(R, nrm, y);
                    const bool rm = i < oc && r < nrm && R[r] == y;
                    const uint64_t m = __ballot(rm);
                    if (i < oc && !rm) W[i - gone - (uint32_t)__popcll(m & lt)] = y;
                    gone += (uint32_t)__popcll(m);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // stores drained before the next reads
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // this wave's own writes, read back below
                const uint32_t w = oc - nrm;
                // each add's place among the kept peers (W[0, w) now), kept in the removes' LDS
                uint32_t* KB = sm.u.ar + kWin;
                for (uint32_t q = lane; q < nadd; q += 64) {
                    const uint32_t y = A[q];
                    uint32_t lo = 0, hi = w;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (W[mid] < y) lo = mid + 1; else hi = mid;
                    }
                    KB[q] = lo;
                }
                wave_lds_sync();
                uint64_t sig = 0;
                for (int64_t c0 = (int64_t)((w + 63) / 64) * 64 - 64; c0 >= 0; c0 -= 64) {
                    const uint32_t j = (uint32_t)c0 + lane;
                    if (j < w) {
                        const uint32_t y = W[j];
                        const uint32_t k = j + lds_lower_bound(A, nadd, y);
                        W[k] = y;
                        if (k < (uint32_t)kInline) inl[k] = y;
                        sig |= peer_sig(y);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                }
                for (uint32_t q = lane; q < nadd; q += 64) {
                    const uint32_t y = A[q], k = KB[q] + q;
                    W[k] = y;
                    if (k < (uint32_t)kInline) inl[k] = y;
                    sig |= peer_sig(y);
                }
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) sig |= __shfl_xor(sig, d, 64);
                if ((uint32_t)lane >= nc && lane < kInline) inl[lane] = kNone;
                if (lane == 0) {
                    L[off] = nc;
                    write_header(rec, nc, off, sig, cap);
                    de += (int64_t)nc - (int64_t)oc;
                    dl += (int64_t)(oc == 0 && nc > 0) - (int64_t)(oc > 0 && nc == 0);
                    nwave++;
                }
            }
            if ((nadd | nrm) && (staged || oc + nadd - nrm > cap)) {
                const uint32_t nc = oc + nadd - nrm;
                uint32_t dst = off, ncap = cap;
                if (nc > cap) {
                    ncap = grown(nc);
                    uint32_t d0 = 0;
                    if (lane == 0) d0 = bump_alloc(a, 1 + ncap);
                    dst = __shfl(d0, 0, 64);
                }
                if (dst != kNone) {
                    const uint32_t* A = sm.u.ar;
                    const uint32_t* R = sm.u.ar + kWin;
                    uint32_t* out = L + dst + 1;
                    uint32_t* inl = reinterpret_cast<uint32_t*>(rec) + kInlineWord0;
                    uint64_t sig = 0;
                    for (uint32_t i = lane; i < oc; i += 64) {
                        const uint32_t y = O[i];
                        const uint32_t r = lds_lower_bound(R, nrm, y);
                        if (r < nrm && R[r] == y) continue;
                        const uint32_t k = i - r + lds_lower_bound(A, nadd, y);
                        out[k] = y;
                        if (k < (uint32_t)kInline) inl[k] = y;
                        sig |= peer_sig(y);
                    }
                    for (uint32_t q = lane; q < nadd; q += 64) {
                        const uint32_t y = A[q];
                        uint32_t lo = 0, hi = oc;
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (O[mid] < y) lo = mid + 1; else hi = mid;
                        }
                        const uint32_t k = q + lo - lds_lower_bound(R, nrm, y);
                        out[k] = y;
                        if (k < (uint32_t)kInline) inl[k] = y;
                        sig |= peer_sig(y);
                    }
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) sig |= __shfl_xor(sig, d, 64);
                    if ((uint32_t)lane >= nc && lane < kInline) inl[lane] = kNone;
                    if (lane == 0) {
                        L[dst] = nc;
                        write_header(rec, nc, dst, sig, ncap);
                        de += (int64_t)nc - (int64_t)oc;
                        dl += (int64_t)(oc == 0 && nc > 0) - (int64_t)(oc > 0 && nc == 0);
                        nwave++;
                    }
                }
            }
            wave_lds_sync();  // the next big cube reuses lst / ar
        }
    }
    WQ_STAMP(10);
    wave_lds_sync();
    }  // buckets
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        de += __shfl_xor(de, d, 64);
        dl += __shfl_xor(dl, d, 64);
        nwave += __shfl_xor(nwave, d, 64);
    }
    if (lane == 0) {
        if (de) atomicAdd(reinterpret_cast<unsigned long long*>(&a.dstat[0]), (unsigned long long)de);
        if (dl) atomicAdd(reinterpret_cast<unsigned long long*>(&a.dstat[1]), (unsigned long long)dl);
        if (nwave) atomicAdd(&a.status->n_wave, nwave);
    }
}

// ---- REMOVE_PEER in place (§8(f) F3) -------------------------------------------------------------
// WorldMap::remove_peer / AreaMap::remove_peer (world_map.rs:41-61, area_map.rs:124-135) for a
// batch of peers: one pass over every cube of both tables, 16 lanes per cube, removing the peers
// from each list in place (a chunk's kept peers move only to lower positions, so a forward
// compaction by group ballots is safe) and rewriting the record's count, signature and inline
// peers where something moved. Peers removed from every world are a bitmap test; removals from
// one world a binary search in the sorted (world << 32 | peer) keys. Empty cubes keep their record.
struct RemoveSet {
    const uint32_t* all_bits;  // peers removed from every world (bitmap), nullptr if none
    uint32_t all_n;            // bitmap length in peers
    const uint64_t* keys;      // sorted (world << 32 | peer) removed from one world
    uint32_t n_keys;
};

__device__ __forceinline__ bool removed(const RemoveSet& rs, uint32_t w, uint32_t p) {
    if (rs.all_bits && p < rs.all_n && ((rs.all_bits[p >> 5] >> (p & 31)) & 1u)) return true;
    if (!rs.n_keys) return false;
    const uint64_t v = ((uint64_t)w << 32) | p;
    uint32_t lo = 0, hi = rs.n_keys;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rs.keys[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo < rs.n_keys && rs.keys[lo] == v;
}

__global__ __launch_bounds__(kBlock) void k_remove_peers(DeltaTable tb, const Slot* __restrict__ slots,
                                                         uint64_t scap, RemoveSet rs, uint64_t* part) {
    __shared__ unsigned long long acc[2];
    if (threadIdx.x < 2) acc[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, gl = threadIdx.x & (kG - 1), grp = threadIdx.x / kG;
    const int gshift = lane & ~(kG - 1);
    const uint32_t lt = (1u << gl) - 1u;
    const uint64_t rcap = tb.rmask + 1, D = rcap + scap;
    int64_t de = 0, dl = 0;
    for (uint64_t e = (uint64_t)blockIdx.x * kGroups + grp; e < D; e += (uint64_t)gridDim.x * kGroups) {
        const bool is_rec = e < rcap;
        uint32_t w, off, n;
        if (is_rec) {
            const uint4 h0 = reinterpret_cast<const uint4*>(tb.recs + e)[0];
            const uint32_t ext = reinterpret_cast<const uint32_t*>(tb.recs + e)[7];
            if (!ext || !h0.z) continue;
            w = (ext >> 8) - 1u;
            n = h0.z;
            off = h0.w;
        } else {
            const SlotView v = load_slot(slots, e - rcap);
            if (v.world == kWorldEmpty) continue;
            w = v.world;
            off = v.off;
            n = tb.list[off];
        }
        uint32_t* rw = reinterpret_cast<uint32_t*>(tb.recs + e);
        // a record cube with <= kInline peers keeps them only inline (its list block is stale)
        const bool inl_only = is_rec && n <= (uint32_t)kInline;
        uint32_t* L = inl_only ? rw + kInlineWord0 : tb.list + off + 1;
        uint32_t kept = 0;
        uint64_t sig = 0;
        for (uint32_t c0 = 0; c0 < n; c0 += kG) {
            const uint32_t k = c0 + gl;
            const uint32_t x = k < n ? L[k] : 0u;
            const bool keep = k < n && !removed(rs, w, x);
            const uint32_t mk = (uint32_t)(__ballot(keep) >> gshift) & 0xFFFFu;
            if (keep) {
                const uint32_t pos = kept + (uint32_t)__popc(mk & lt);
                sig |= peer_sig(x);
                if (pos != k) {  // shifted by an earlier removal
                    L[pos] = x;
                    if (is_rec && !inl_only && pos < (uint32_t)kInline) rw[kInlineWord0 + pos] = x;
                }
            }
            kept += (uint32_t)__popc(mk);
        }
        if (kept == n) continue;  // group-uniform: nothing removed here
#pragma unroll
        for (int d = kG / 2; d >= 1; d >>= 1) sig |= __shfl_xor(sig, d, kG);
        if (gl == 0 && !inl_only) L[-1] = kept;
        if (is_rec) {
            for (uint32_t k = kept + gl; k < n && k < (uint32_t)kInline; k += kG) rw[kInlineWord0 + k] = kNone;
            if (gl == 0) {
                rw[2] = kept;
                rw[4] = (uint32_t)sig;
                rw[5] = (uint32_t)(sig >> 32);
            }
        }
        if (gl == 0) {
            de -= (int64_t)(n - kept);
            dl -= kept == 0 ? 1 : 0;
        }
    }
    if (de) atomicAdd(&acc[0], (unsigned long long)de);
    if (dl) atomicAdd(&acc[1], (unsigned long long)dl);
    __syncthreads();
    if (threadIdx.x < 2) part[2ull * blockIdx.x + threadIdx.x] = acc[threadIdx.x];
}

// ---- materialize: the sorted-state arrays from the records and slots ---------------------------

__device__ __forceinline__ void record_key(const Record& r, int64_t s, uint32_t* w, int64_t* k) {
    uint32_t a[3];
    unpack_key(r.pk, r.ext, w, a);
#pragma unroll
    for (int d = 0; d < 3; ++d) k[d] = ((int64_t)a[d] - (int64_t)kAxisBias) * s;
}

__global__ void k_mat_count(const Record* __restrict__ recs, uint64_t rcap, const Slot* __restrict__ slots,
                            uint64_t scap, const uint32_t* __restrict__ list, uint32_t* cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < rcap) {
        cnt[i] = recs[i].ext ? recs[i].count : 0u;
    } else if (i < rcap + scap) {
        const SlotView s = load_slot(slots, i - rcap);
        cnt[i] = s.world == kWorldEmpty ? 0u : list[s.off];
    }
}

__global__ void k_mat_write(const Record* __restrict__ recs, uint64_t rcap, const Slot* __restrict__ slots,
                            uint64_t scap, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                            const uint32_t* __restrict__ pos, int64_t s, uint64_t hmask, uint64_t* st_h,
                            uint32_t* st_w, int64_t* st_kx, int64_t* st_ky, int64_t* st_kz, uint32_t* st_p) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= rcap + scap) return;
    const uint32_t n = cnt[i];
    if (!n) return;
    uint32_t w, off;
    int64_t k[3];
    const uint32_t* src;
    if (i < rcap) {
        const Record& r = recs[i];
        record_key(r, s, &w, k);
        off = r.list_off;
        src = n <= (uint32_t)kInline ? r.peers : list + off + 1;  // short lists live inline only
    } else {
        const SlotView v = load_slot(slots, i - rcap);
        w = v.world;
        k[0] = v.k0;
        k[1] = v.k1;
        k[2] = v.k2;
        off = v.off;
        src = list + off + 1;
    }
    const uint64_t hh = cube_hash(w, k[0], k[1], k[2]) & hmask;
    const uint32_t o = pos[i];
    for (uint32_t j = 0; j < n; ++j) {
        st_h[o + j] = hh;
        st_w[o + j] = w;
        st_kx[o + j] = k[0];
        st_ky[o + j] = k[1];
        st_kz[o + j] = k[2];
        st_p[o + j] = src[j];
    }
}

}  // namespace

int table_sync_delta_stats(wq_router* h) {
    if (int rc = table_resolve(h, true)) return rc;
    if (!h->dstat_pending) {
        WQ_HIP(h, hipStreamSynchronize(h->stream));
        return WQ_OK;
    }
    uint64_t v[2];
    WQ_HIP(h, hipMemcpyAsync(v, h->dws.dstat.p, 16, hipMemcpyDeviceToHost, h->stream));
    WQ_HIP(h, hipMemsetAsync(h->dws.dstat.p, 0, 16, h->stream));
    WQ_HIP(h, hipStreamSynchronize(h->stream));
    h->st.n = (uint64_t)((int64_t)h->st.n + (int64_t)v[0]);
    h->tab.n_cubes = (uint64_t)((int64_t)h->tab.n_cubes + (int64_t)v[1]);
    h->dstat_pending = false;
    return WQ_OK;
}

int table_apply_delta(wq_router* h, size_t n_ops, bool* applied) {
    *applied = false;
    if (n_ops == 0) {
        *applied = true;
        return WQ_OK;
    }
    const uint32_t n = (uint32_t)n_ops;
    DeltaWs& d = h->dws;
    Table& t = h->tab;
    hipStream_t s = h->stream;
    const int rbits = 64 - t.rec_shift;
    // every op may bring a new cube: keep the record table at load <= 1/2 through the claims; the
    // sort key holds a 31-bit slot
    if (2 * (t.n_recs + n) > t.rec_cap || rbits > 30) {
        h->n_delta_fallbacks++;
        return WQ_OK;
    }
    // buckets of ~128 ops (a wave's window is 256): sorted bits = log2(n / 128), at most 16 (two
    // radix passes), and enough that a bucket spans at most 2^16 slots (the in-window key field)
    // (the real buckets are 2^(sbits - 1): the top sorted bit only parts kNoKey ops off)
    static const uint64_t per_bucket = getenv("WQ_DELTA_OPS_PER_BUCKET") ? strtoull(getenv("WQ_DELTA_OPS_PER_BUCKET"), nullptr, 10) : 128;
    int sbits = 1;
    while (sbits < 16 && (per_bucket << sbits) <= n) sbits++;
    if (sbits > rbits + 1) sbits = rbits + 1;
    if (rbits + 1 - sbits > 16) sbits = rbits + 1 - 16;
    const int lowbits = rbits + 1 - sbits;
    const uint32_t NBr = 1u << (rbits - lowbits);
    WQ_ALLOC(h, h->key64_a, (uint64_t)n * 8);
    WQ_ALLOC(h, h->key64_b, (uint64_t)n * 8);
    WQ_ALLOC(h, h->cube_start, ((uint64_t)NBr + 1) * 4);
    WQ_ALLOC(h, d.summ, 128);  // DeltaStatus, then the host snapshot at +64
    if (!d.dstat.p) {
        WQ_ALLOC(h, d.dstat, 16);
        WQ_HIP(h, hipMemsetAsync(d.dstat.p, 0, 16, s));
    }
    DeltaStatus* status = d.summ.as<DeltaStatus>();
    PendingDelta& pd = h->pend;
    if (!pd.pinned) {  // first batch: the status zero, then k_delta_finish re-arms it
        WQ_HIP(h, hipMemsetAsync(d.summ.p, 0, 128, s));
        WQ_HIP(h, hipHostMalloc(&pd.pinned, 64, hipHostMallocCoherent | hipHostMallocMapped));
    }
    uint64_t* keys = h->key64_a.as<uint64_t>();
    uint64_t* skeys = h->key64_b.as<uint64_t>();
    hipLaunchKernelGGL(k_delta_events, dim3(grid_for(n)), dim3(kBlock), 0, s, h->cur_ops, n, (double)h->cube_size,
                       (int64_t)h->cube_size, t.recs.as<Record>(), t.rclaim.as<uint32_t>(),
                       kBatchTag | (uint32_t)(++h->n_delta_batches & 0x7FFFFFFFu), t.rec_cap - 1, t.rec_shift,
                       h->hash_mask, keys, status);
    // stable LSD passes over the bucket field: key bits [33 + lowbits, 33 + lowbits + sbits)
    const uint32_t ntiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
    WQ_ALLOC(h, d.sort_cnt, (uint64_t)256 * ntiles * 4);
    WQ_ALLOC(h, d.sort_tot, 256 * 4);
    const int fbits = rbits + 1 - lowbits;  // == sbits
    const int p1 = std::min(fbits, 8), p2 = fbits - p1;
    auto sort_pass = [&](const uint64_t* in, uint64_t* out, int sh, int bits) {
        const uint32_t dmask = (1u << bits) - 1u;
        hipLaunchKernelGGL(k_sort_hist, dim3(ntiles), dim3(kBlock), 0, s, in, n, sh, dmask, ntiles,
                           d.sort_cnt.as<uint32_t>());
        hipLaunchKernelGGL(k_sort_rowscan, dim3(dmask + 1), dim3(kBlock), 0, s, d.sort_cnt.as<uint32_t>(), ntiles,
                           d.sort_tot.as<uint32_t>());
        hipLaunchKernelGGL(k_sort_scatter, dim3(ntiles), dim3(kBlock), 0, s, in, out, n, sh, dmask, bits, ntiles,
                           d.sort_cnt.as<uint32_t>(), d.sort_tot.as<uint32_t>());
    };
    sort_pass(keys, skeys, 33 + lowbits, p1);
    if (p2 > 0) {
        sort_pass(skeys, keys, 33 + lowbits + p1, p2);
        std::swap(keys, skeys);  // the sorted keys are in key64_a
    }
    uint32_t* bstart = h->cube_start.as<uint32_t>();
    hipLaunchKernelGGL(k_bucket_bounds, dim3(grid_for((uint64_t)n + 1)), dim3(kBlock), 0, s, skeys, n, lowbits, NBr,
                       bstart);
    BucketArgs ba;
    ba.tb = DeltaTable{t.recs.as<Record>(), t.rclaim.as<uint32_t>(), t.rec_cap - 1, t.rec_shift, h->hash_mask,
                       t.list.as<uint32_t>()};
    ba.keys = skeys;
    ba.bstart = bstart;
    ba.lowbits = lowbits;
    ba.status = status;
    ba.dstat = d.dstat.as<int64_t>();
    const uint64_t list_limit = std::min<uint64_t>(t.list_cap, 0xFFFFFFFFull);
    ba.list_base = t.list_used;
    ba.list_room = list_limit > t.list_used ? list_limit - t.list_used : 0;
    static const bool stamps = getenv("WQ_DELTA_STAMPS") != nullptr;  // diagnostics only
    ba.stamps = nullptr;
    if (!t.stale.p) {
        WQ_ALLOC(h, t.stale, 4);
        WQ_HIP(h, hipMemsetAsync(t.stale.p, 0, 4, s));
    }
    if (stamps) {
        WQ_ALLOC(h, h->idx_b, (uint64_t)NBr * 16 * 8);
        WQ_HIP(h, hipMemsetAsync(h->idx_b.p, 0, (uint64_t)NBr * 16 * 8, s));
        ba.stamps = h->idx_b.as<uint64_t>();
    }
    ba.nb = NBr;
    // Buckets per wave (grid stride): two once there are >= 4,096 buckets. Tens of thousands of
    // one-wave workgroups of 16 KB LDS each turn over faster than they work (C5: 32,768 buckets,
    // update 0.81 -> 0.75 ms with two per wave; C4: 4,096, 0.198 -> 0.19); four leave C4 too few
    // waves (0.254). WQ_DELTA_BPW overrides (diagnostics, tools/delta_bpw.sh).
    static const int bpw_env = getenv("WQ_DELTA_BPW") ? std::max(1, atoi(getenv("WQ_DELTA_BPW"))) : 0;
    const uint32_t bpw = bpw_env ? (uint32_t)bpw_env : (NBr >= 4096 ? 2u : 1u);
    // Round words: 256 while the table's lists average <= 20 peers (C5, ~13: update 0.718 -> 0.680 ms
    // on one box — the higher occupancy outweighs the extra rounds), 1024 above (C4, ~34: 0.189 ms
    // against 0.237 at 256 and 0.202 at 512; profiles/r06_churn_round_words_ab.json). 128 (15 waves
    // per CU) was slower at C5: 0.758-0.770 ms. The counts
    // lag one batch (folded in by the next call), which a mean does not notice. WQ_ROUND_WORDS
    // (256 / 1024) overrides.
    static const int rw_env = getenv("WQ_ROUND_WORDS") ? atoi(getenv("WQ_ROUND_WORDS")) : 0;
    const bool short_lists = rw_env ? rw_env <= 256 : h->st.n <= 20ull * std::max<uint64_t>(t.n_cubes, 1);
    if (short_lists)
        hipLaunchKernelGGL(k_delta_bucket<256>, dim3((NBr + bpw - 1) / bpw), dim3(64), 0, s, ba);
    else
        hipLaunchKernelGGL(k_delta_bucket<1024>, dim3((NBr + bpw - 1) / bpw), dim3(64), 0, s, ba);
    WQ_HIP(h, hipGetLastError());
    if (ba.stamps) {  // diagnostics: mean cycles per bucket and phase
        std::vector<uint64_t> st((size_t)NBr * 16);
        WQ_HIP(h, hipMemcpyAsync(st.data(), ba.stamps, st.size() * 8, hipMemcpyDeviceToHost, s));
        WQ_HIP(h, hipStreamSynchronize(s));
        double sum[16] = {0};
        for (uint32_t b = 0; b < NBr; ++b)
            for (int k = 0; k < 16; ++k) sum[k] += (double)st[(size_t)b * 16 + k];
        fprintf(stderr, "delta buckets %u n %u:", NBr, n);
        for (int k = 0; k < 11; ++k) fprintf(stderr, " %d:%.0f", k, sum[k] / NBr);
        fprintf(stderr, "\n");
    }
    hipLaunchKernelGGL(k_delta_finish, dim3(1), dim3(1), 0, s, status, d.dstat.as<int64_t>(),
                       static_cast<uint64_t*>(pd.pinned), t.stale.as<uint32_t>(),
                       t.n_pbox ? t.pbox.as<uint32_t>() + (uint64_t)kBoxWords * t.n_pbox : nullptr);
    WQ_HIP(h, hipGetLastError());
    if (!pd.ev) WQ_HIP(h, hipEventCreateWithFlags(&pd.ev, hipEventDisableTiming));
    WQ_HIP(h, hipEventRecord(pd.ev, s));
    h->dstat_pending = false;
    pd.active = true;
    pd.ops = h->cur_ops;
    pd.n = n_ops;
    pd.list_room = ba.list_room;
    h->st_stale = true;
    h->any_stale = true;
    h->n_delta_applies++;
    *applied = true;
    return WQ_OK;
}

int table_rebuild_batch(wq_router* h, size_t n_ops);  // wq_table.hip: the full rebuild of h->cur_ops

int table_resolve(wq_router* h, bool blocking) {
    PendingDelta& pd = h->pend;
    if (!pd.active) return WQ_OK;
    if (!blocking) {
        const hipError_t q = hipEventQuery(pd.ev);
        if (q == hipErrorNotReady) return WQ_OK;
        if (q != hipSuccess) return set_error(h, WQ_E_HIP, "hipEventQuery", q);
    }
    WQ_HIP(h, hipEventSynchronize(pd.ev));
    pd.active = false;
    Table& t = h->tab;
    DeltaStatus hs;
    int64_t v[2];
    std::memcpy(&hs, pd.pinned, sizeof(hs));
    std::memcpy(v, static_cast<const char*>(pd.pinned) + 32, sizeof(v));
    // the claims of a batch that is not applied stay as empty records (count 0): invisible to
    // every query, dropped by the rebuild
    t.n_recs += hs.new_recs;
    h->st.n = (uint64_t)((int64_t)h->st.n + v[0]);
    t.n_cubes = (uint64_t)((int64_t)t.n_cubes + v[1]);
    t.list_used += std::min<uint64_t>(hs.bump, pd.list_room);
    if (hs.n_wave) h->n_delta_wave_batches++;
    if (!hs.flags) return WQ_OK;
    // not applied (1: an op without a packed key; 2: an invalid op) or applied except the cubes
    // whose relocation did not fit (4): the rebuild takes the table as it stands plus the whole
    // batch again — exact, since the batch fixes the final state of every pair it touches
    h->n_delta_applies--;
    WQ_HIP(h, hipMemsetAsync(t.stale.p, 0, 4, h->stream));
    if (hs.flags & 2u) {
        // the batch held an invalid op and was not applied (the table is as before it). The call
        // folding it in goes on with its own work; the rejection stays visible in wq_last_error and
        // as error bit 16 of wq_route_health (no silently dropped call)
        WQ_HIP(h, hipStreamSynchronize(h->stream));
        RouteWs& rw = h->rws;
        if (!rw.buf.p) {  // as route_counters lays it out: health words first
            WQ_ALLOC(h, rw.buf, 128);
            WQ_HIP(h, hipMemsetAsync(rw.buf.p, 0, 128, h->stream));
            rw.calls = 0;
        }
        uint32_t w = 0;
        WQ_HIP(h, hipMemcpyAsync(&w, rw.buf.p, 4, hipMemcpyDeviceToHost, h->stream));
        WQ_HIP(h, hipStreamSynchronize(h->stream));
        w |= kErrBadBatch;
        WQ_HIP(h, hipMemcpyAsync(rw.buf.p, &w, 4, hipMemcpyHostToDevice, h->stream));
        WQ_HIP(h, hipStreamSynchronize(h->stream));
        h->err = "bad op (kind or reserved world id) in an earlier device batch: that batch was not applied";
        return WQ_OK;
    }
    h->n_delta_fallbacks++;
    h->table_gen++;
    h->tab.hdr_ok = false;
    h->cur_ops = pd.ops;
    return table_rebuild_batch(h, pd.n);
}

int table_remove_peers_inplace(wq_router* h, const uint64_t* keys, size_t n_rm) {
    DeltaWs& d = h->dws;
    Table& t = h->tab;
    hipStream_t s = h->stream;
    // split: (WQ_WORLD_INVALID, peer) = every world -> bitmap; the rest stay sorted keys
    size_t n_all = 0;
    uint32_t max_all = 0;
    while (n_all < n_rm && (keys[n_rm - 1 - n_all] >> 32) == WQ_WORLD_INVALID) {
        max_all = std::max<uint32_t>(max_all, (uint32_t)keys[n_rm - 1 - n_all]);
        ++n_all;
    }
    const size_t n_one = n_rm - n_all;  // keys sort by world first: the every-world ones are last
    RemoveSet rs{nullptr, 0, nullptr, (uint32_t)n_one};
    std::vector<uint32_t> bits;  // read by an asynchronous copy: lives until the synchronize below
    if (n_all) {
        const uint32_t words = max_all / 32 + 1;
        bits.assign(words, 0u);
        for (size_t i = n_one; i < n_rm; ++i) {
            const uint32_t p = (uint32_t)keys[i];
            bits[p >> 5] |= 1u << (p & 31);
        }
        WQ_ALLOC(h, d.rm_bits, (uint64_t)words * 4);
        WQ_HIP(h, hipMemcpyAsync(d.rm_bits.p, bits.data(), (size_t)words * 4, hipMemcpyHostToDevice, s));
        rs.all_bits = d.rm_bits.as<uint32_t>();
        rs.all_n = words * 32;
    }
    if (n_one) {
        WQ_ALLOC(h, h->key32_b, n_one * 8);
        WQ_HIP(h, hipMemcpyAsync(h->key32_b.p, keys, n_one * 8, hipMemcpyHostToDevice, s));
        rs.keys = h->key32_b.as<uint64_t>();
    }
    WQ_ALLOC(h, d.part, (uint64_t)kGroupGrid * 32);
    if (!d.dstat.p) {
        WQ_ALLOC(h, d.dstat, 16);
        WQ_HIP(h, hipMemsetAsync(d.dstat.p, 0, 16, s));
    }
    DeltaTable tb{t.recs.as<Record>(), t.rclaim.as<uint32_t>(), t.rec_cap - 1, t.rec_shift, h->hash_mask,
                  t.list.as<uint32_t>()};
    const uint64_t D = t.rec_cap + t.cap;
    const uint32_t ng = (uint32_t)std::min<uint64_t>((D + kGroups - 1) / kGroups, kGroupGrid);
    hipLaunchKernelGGL(k_remove_peers, dim3(ng), dim3(kBlock), 0, s, tb, t.slots.as<Slot>(), t.cap, rs,
                       d.part.as<uint64_t>());
    hipLaunchKernelGGL(k_delta_stats, dim3(1), dim3(kBlock), 0, s, d.part.as<uint64_t>(), ng, d.dstat.as<uint64_t>());
    WQ_HIP(h, hipGetLastError());
    h->dstat_pending = true;
    h->st_stale = true;
    h->any_stale = true;
    // the host arrays above are read by copies still in flight
    WQ_HIP(h, hipStreamSynchronize(s));
    return WQ_OK;
}

int table_materialize(wq_router* h) {
    if (!h->st_stale) return WQ_OK;
    int rc0 = table_sync_delta_stats(h);
    if (rc0) return rc0;
    Table& t = h->tab;
    hipStream_t s = h->stream;
    const uint64_t D = t.rec_cap + t.cap;
    if (D >= 0xFFFFFFFFull) return set_error(h, WQ_E_INVALID, "table too large to materialize");
    WQ_ALLOC(h, h->flags, D * 4);
    WQ_ALLOC(h, h->scan, D * 4);
    uint32_t* cnt = h->flags.as<uint32_t>();
    uint32_t* pos = h->scan.as<uint32_t>();
    hipLaunchKernelGGL(k_mat_count, dim3(grid_for(D)), dim3(kBlock), 0, s, t.recs.as<Record>(), t.rec_cap,
                       t.slots.as<Slot>(), t.cap, t.list.as<uint32_t>(), cnt);
    int rc = scan_u32(h, cnt, pos, D, false);
    if (rc) return rc;
    uint32_t lp = 0, lc = 0;
    if ((rc = read_u32(h, pos, D - 1, &lp))) return rc;
    if ((rc = read_u32(h, cnt, D - 1, &lc))) return rc;
    const uint64_t S = (uint64_t)lp + lc;
    if (S != h->st.n) return set_error(h, WQ_E_HIP, "materialize: entry count disagrees with the table");
    if ((rc = ensure_state(h, h->st, S))) return rc;
    hipLaunchKernelGGL(k_mat_write, dim3(grid_for(D)), dim3(kBlock), 0, s, t.recs.as<Record>(), t.rec_cap,
                       t.slots.as<Slot>(), t.cap, t.list.as<uint32_t>(), cnt, pos, (int64_t)h->cube_size,
                       h->hash_mask, h->st.h.as<uint64_t>(), h->st.w.as<uint32_t>(), h->st.kx.as<int64_t>(),
                       h->st.ky.as<int64_t>(), h->st.kz.as<int64_t>(), h->st.p.as<uint32_t>());
    WQ_HIP(h, hipGetLastError());
    h->st_stale = false;
    return WQ_OK;
}

}  // namespace wq
