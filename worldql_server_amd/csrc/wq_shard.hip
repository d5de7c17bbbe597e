// wq_shard.hip — cube-hash ownership for the multi-GPU path.
//
// Every (world, cube) bucket is independent, so the table is partitioned by a hash of the
// quantised key: owner(world, key) = shard_of(...) in [0, G). A tick on G GPUs is
//   (1) shard_messages: quantise each ingested message (kernel 1), compute its owner, and group
//       the messages by owner into 40-byte records, stable in message order (three launches:
//       per-block owner histograms -> one flat scan -> ballot-ranked scatter);
//   (2) an all-to-all of the records (wq_sharded.hip's exchange: RCCL, the hub, or the caller's
//       transport through wq_shard_attach_exchange);
//   (3) route_records: the single-GPU route (count / scan / emit) on the received records —
//       keys are already quantised, so the count pass takes its raw-key branch;
//   (4) the pairs return to the ingesting GPU with a second all-to-all.
// Subscription ops go to the owner of their cube (op_owner_kernel); REMOVE_PEER goes to all.
// The per-message body that runs on the owner is still local_message.rs:52-86.
#include "route_common.hpp"
#include "route_tick.hpp"  // granule / poll_granule: the tagged look-back words

namespace wq {

constexpr int kShardIPT = 4;                  // messages per thread
constexpr uint32_t kShardTile = kBlock * kShardIPT;
constexpr int kScanThreads1 = 1024;

static_assert(sizeof(wq_msg_rec) == 40, "wq_msg_rec is 40 bytes");

struct ShardIn {
    const double* pos;
    const int64_t* keys;
    const uint32_t* world;
    const uint32_t* sender;
    const uint8_t* repl;
    uint32_t M;
    uint32_t G;
    uint32_t nblk;
    double sf;
    int64_t si;
    bool pos_rec;  // records carry the positions (radius filter on)
    uint32_t me = kNone;  // budgeted slots (slot_*_kernel): this shard's own messages take no slot
    // ... unless own_slots is set: then they are slots too, in own_slots (never exchanged; its slot
    // -> message map in own_perm), and the histogram's column `me` counts them
    uint32_t* own_slots = nullptr;
    uint32_t* own_perm = nullptr;
    bool own_too = false;
    // own_slots with a budget: the owner form writes its self segment straight into its receive
    // buffer (no self copy in the exchange), budgeted like every other segment
    uint32_t own_budget = 0xFFFFFFFFu;
    uint32_t* zero_e = nullptr;  // slot_count_kernel: e[m] = 0 for every message (rows no step writes)
    // slot_scatter_kernel (the owner form's budgeted tick): the budget bit of ANY of this shard's
    // segments goes to every segment's status word, so each owner learns of every short budget
    // from X1 alone
    uint32_t* a_or = nullptr;
};

template <bool RAW>
__device__ __forceinline__ void msg_key(const ShardIn& in, uint32_t m, int64_t& x, int64_t& y, int64_t& z) {
    if (RAW) {
        x = in.keys[3ull * m];
        y = in.keys[3ull * m + 1];
        z = in.keys[3ull * m + 2];
    } else {
        x = coord_clamp_dev(in.pos[3ull * m], in.sf, in.si);
        y = coord_clamp_dev(in.pos[3ull * m + 1], in.sf, in.si);
        z = coord_clamp_dev(in.pos[3ull * m + 2], in.sf, in.si);
    }
}

// Compact records (COMPACT = true; the sharded tick of wq_sharded.hip with the radius filter off):
// 20-byte slots of five words. A message whose cube has a packed key (pack_key: the regular case)
// takes one slot
//   {pk lo, pk hi, ext, sender, repl | kSlotReg << 8}
// and any other (raw off-grid keys, NaN / huge coordinates, world ids >= 2^24 - 1) takes two:
//   {x lo, x hi, world, sender, repl | kSlotHead << 8}, {y lo, y hi, z lo, z hi, kSlotTail << 8}.
// The owner needs no message index (the answers return in slot order), so the ingesting GPU keeps
// slot -> message in perm[] (kNone for a tail). Half the bytes of a 40-byte wq_msg_rec on xGMI.
// (the shared definitions — kSlot*, kSlotWords — are in route_common.hpp)

template <bool RAW, bool COMPACT>
__device__ __forceinline__ uint32_t msg_weight(const ShardIn& in, uint32_t w, int64_t x, int64_t y, int64_t z) {
    if (!COMPACT) return 1u;
    uint64_t pk;
    uint32_t ext;
    return pack_key(w, x, y, z, in.sf, &pk, &ext) ? 1u : 2u;
}

// (1a) per-block owner histogram (records, or compact slots), stored owner-major:
// counts[d * nblk + b]. A flat exclusive scan of that array is then directly each (owner, block)
// pair's first output slot.
template <bool RAW, bool COMPACT = false>
__global__ void __launch_bounds__(kBlock) shard_count_kernel(ShardIn in, uint32_t* __restrict__ counts) {
    __shared__ uint32_t cnt[WQ_MAX_SHARDS];
    for (uint32_t d = threadIdx.x; d < in.G; d += kBlock) cnt[d] = 0;
    __syncthreads();
    const uint32_t m0 = blockIdx.x * kShardTile + threadIdx.x;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        const bool valid = m < in.M;
        uint32_t own = 0xFFFFFFFFu, wt = 0;
        if (valid) {
            int64_t x, y, z;
            msg_key<RAW>(in, m, x, y, z);
            const uint32_t w = in.world[m];
            own = shard_of(w, x, y, z, in.G);
            wt = msg_weight<RAW, COMPACT>(in, w, x, y, z);
        }
        // one LDS add per distinct owner in the wave (G = 1: one per wave, not 64 on one word)
        const uint64_t wide = __ballot(wt == 2);
        uint64_t todo = __ballot(valid);
        while (todo) {
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const uint32_t d = __shfl(own, leader, 64);
            const uint64_t mask = __ballot(own == d);
            if (lane == leader) atomicAdd(&cnt[d], (uint32_t)(__popcll(mask) + __popcll(mask & wide)));
            todo &= ~mask;
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < in.G; d += kBlock) counts[(uint64_t)d * in.nblk + blockIdx.x] = cnt[d];
}

// (1b) one block: exclusive scan of the n = G * nblk histogram entries in place; per-owner totals
// at dest_counts[d * stride].
__global__ void __launch_bounds__(kScanThreads1)
    shard_scan_kernel(uint32_t* __restrict__ v, uint32_t nblk, uint32_t G, uint32_t* __restrict__ dest_counts,
                      uint32_t stride) {
    __shared__ uint32_t wsum[kScanThreads1 / 64];
    __shared__ uint32_t carry_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t n = nblk * G;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += kScanThreads1) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t x = i < n ? v[i] : 0;
        const uint32_t inc = wave_incl_scan_add(x, lane);
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        if (wave == 0) {
            const uint32_t s = lane < kScanThreads1 / 64 ? wsum[lane] : 0;
            const uint32_t si = wave_incl_scan_add(s, lane);
            if (lane < kScanThreads1 / 64) wsum[lane] = si - s;
        }
        __syncthreads();
        const uint32_t carry = carry_s;
        if (i < n) v[i] = carry + wsum[wave] + inc - x;
        __syncthreads();
        if (threadIdx.x == kScanThreads1 - 1) carry_s = carry + wsum[wave] + inc;
        __syncthreads();
    }
    // v is visible to this block after the last barrier (same workgroup, global memory, fenced).
    __threadfence_block();
    const uint32_t total = carry_s;
    for (uint32_t d = threadIdx.x; d < G; d += kScanThreads1) {
        const uint32_t lo = v[(uint64_t)d * nblk];
        const uint32_t hi = d + 1 < G ? v[(uint64_t)(d + 1) * nblk] : total;
        dest_counts[(uint64_t)d * stride] = hi - lo;
    }
}

// (1c') the compact form of (1c): the same stable, ballot-ranked scatter, where a message weighs
// its slot count (1 regular, 2 head + tail) in the ranks; writes the slots and perm[slot].
template <bool RAW>
__global__ void __launch_bounds__(kBlock)
    shard_scatter20_kernel(ShardIn in, const uint32_t* __restrict__ base, uint32_t* __restrict__ out,
                           uint32_t* __restrict__ perm) {
    __shared__ uint32_t wc[kShardIPT * kWaves][WQ_MAX_SHARDS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t k = threadIdx.x; k < kShardIPT * kWaves * WQ_MAX_SHARDS; k += kBlock) (&wc[0][0])[k] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
    const uint32_t m0 = blockIdx.x * kShardTile + threadIdx.x;
    int64_t kx[kShardIPT], ky[kShardIPT], kz[kShardIPT];
    uint64_t pk[kShardIPT];
    uint32_t ext[kShardIPT], own[kShardIPT], rank[kShardIPT];
    bool reg[kShardIPT];
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        const bool valid = m < in.M;
        own[i] = 0xFFFFFFFFu;
        rank[i] = 0;
        reg[i] = true;
        if (valid) {
            msg_key<RAW>(in, m, kx[i], ky[i], kz[i]);
            const uint32_t w = in.world[m];
            own[i] = shard_of(w, kx[i], ky[i], kz[i], in.G);
            reg[i] = pack_key(w, kx[i], ky[i], kz[i], in.sf, &pk[i], &ext[i]);
        }
        const uint64_t wide = __ballot(valid && !reg[i]);
        uint64_t todo = __ballot(valid);
        while (todo) {
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const uint32_t d = __shfl(own[i], leader, 64);
            const uint64_t mask = __ballot(own[i] == d);
            if (own[i] == d) rank[i] = __popcll(mask & lt) + __popcll(mask & wide & lt);
            if (lane == leader) wc[i * kWaves + wave][d] = __popcll(mask) + __popcll(mask & wide);
            todo &= ~mask;
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < in.G; d += kBlock) {
        uint32_t run = base[(uint64_t)d * in.nblk + blockIdx.x];
#pragma unroll
        for (int k = 0; k < kShardIPT * kWaves; ++k) {
            const uint32_t t = wc[k][d];
            wc[k][d] = run;
            run += t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        if (m >= in.M) continue;
        const uint32_t slot = wc[i * kWaves + wave][own[i]] + rank[i];
        uint32_t* o = out + (uint64_t)kSlotWords * slot;
        const uint32_t rp = in.repl[m];
        if (reg[i]) {
            o[0] = (uint32_t)pk[i];
            o[1] = (uint32_t)(pk[i] >> 32);
            o[2] = ext[i];
            o[3] = in.sender[m];
            o[4] = rp | (kSlotReg << 8);
            perm[slot] = m;
        } else {
            o[0] = (uint32_t)(uint64_t)kx[i];
            o[1] = (uint32_t)((uint64_t)kx[i] >> 32);
            o[2] = in.world[m];
            o[3] = in.sender[m];
            o[4] = rp | (kSlotHead << 8);
            o[5] = (uint32_t)(uint64_t)ky[i];
            o[6] = (uint32_t)((uint64_t)ky[i] >> 32);
            o[7] = (uint32_t)(uint64_t)kz[i];
            o[8] = (uint32_t)((uint64_t)kz[i] >> 32);
            o[9] = kSlotTail << 8;
            perm[slot] = m;
            perm[slot + 1] = kNone;
        }
    }
}

// (1c) stable scatter. Message order inside a block is (iteration, wave, lane); each wave ranks
// its messages per owner with ballots (one round per distinct owner in the wave), the 4*IPT
// (iteration, wave) groups are scanned per owner in LDS, and the scanned histogram gives the
// block's first slot per owner.
template <bool RAW>
__global__ void __launch_bounds__(kBlock)
    shard_scatter_kernel(ShardIn in, const uint32_t* __restrict__ base, wq_msg_rec* __restrict__ out) {
    __shared__ uint32_t wc[kShardIPT * kWaves][WQ_MAX_SHARDS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t k = threadIdx.x; k < kShardIPT * kWaves * WQ_MAX_SHARDS; k += kBlock) (&wc[0][0])[k] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
    const uint32_t m0 = blockIdx.x * kShardTile + threadIdx.x;
    int64_t kx[kShardIPT], ky[kShardIPT], kz[kShardIPT];
    uint32_t own[kShardIPT], rank[kShardIPT];
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        const bool valid = m < in.M;
        own[i] = 0xFFFFFFFFu;
        rank[i] = 0;
        if (valid) {
            msg_key<RAW>(in, m, kx[i], ky[i], kz[i]);
            own[i] = shard_of(in.world[m], kx[i], ky[i], kz[i], in.G);
        }
        uint64_t todo = __ballot(valid);
        while (todo) {
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const uint32_t d = __shfl(own[i], leader, 64);
            const uint64_t mask = __ballot(own[i] == d);
            if (own[i] == d) rank[i] = __popcll(mask & lt);
            if (lane == leader) wc[i * kWaves + wave][d] = __popcll(mask);
            todo &= ~mask;
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < in.G; d += kBlock) {
        uint32_t run = base[(uint64_t)d * in.nblk + blockIdx.x];
#pragma unroll
        for (int k = 0; k < kShardIPT * kWaves; ++k) {
            const uint32_t t = wc[k][d];
            wc[k][d] = run;
            run += t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        if (m < in.M) {
            wq_msg_rec r;
            if (!RAW && in.pos_rec) {  // the owner's radius filter needs the position itself
                r.key[0] = __double_as_longlong(in.pos[3ull * m]);
                r.key[1] = __double_as_longlong(in.pos[3ull * m + 1]);
                r.key[2] = __double_as_longlong(in.pos[3ull * m + 2]);
                r.flags = WQ_REC_POS;
            } else {
                r.key[0] = kx[i];
                r.key[1] = ky[i];
                r.key[2] = kz[i];
                r.flags = 0;
            }
            r.world = in.world[m];
            r.sender = in.sender[m];
            r.msg = m;
            r.repl = in.repl[m];
            r.pad_[0] = r.pad_[1] = 0;
            out[wc[i * kWaves + wave][own[i]] + rank[i]] = r;
        }
    }
}

// ---- budgeted slots (the sharded tick of wq_sharded.hip) ----------------------------------------
// Only messages owned by ANOTHER shard become slots: the ingesting shard counts the messages of its
// own cubes in place (count_kernel<..., OWN>). Owner d's slots go to the segment
// [L.base[d], L.base[d] + L.budget[d]) of the send buffer — sizes fixed on the host before the tick
// (the previous tick's counts with headroom, or this tick's exact counts), so the exchanges can be
// enqueued without reading anything back. The true count per owner and a budget-overflow bit go to
// the small exchange vector (a[2d], a[2d + 1]); slots past a budget are not written.
// (SlotLayout, kStBudget: route_common.hpp)

// (b1) per-block owner histogram as shard_count_kernel, own messages weighing 0.
template <bool RAW>
__global__ void __launch_bounds__(kBlock) slot_count_kernel(ShardIn in, uint32_t* __restrict__ counts) {
    __shared__ uint32_t cnt[WQ_MAX_SHARDS];
    for (uint32_t d = threadIdx.x; d < in.G; d += kBlock) cnt[d] = 0;
    __syncthreads();
    const uint32_t m0 = blockIdx.x * kShardTile + threadIdx.x;
    const int lane = threadIdx.x & 63;
    // every message's owner first (all loads of the lane in flight together), then the histogram:
    // interleaved with the ballot loops, each message's loads waited for the previous message's
    bool valid[kShardIPT];
    uint32_t own[kShardIPT], wt[kShardIPT];
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        valid[i] = m < in.M;
        own[i] = 0xFFFFFFFFu;
        wt[i] = 0;
        if (valid[i]) {
            int64_t x, y, z;
            msg_key<RAW>(in, m, x, y, z);
            const uint32_t w = in.world[m];
            own[i] = shard_of(w, x, y, z, in.G);
            wt[i] = msg_weight<RAW, true>(in, w, x, y, z);
            valid[i] = in.own_too || own[i] != in.me;
            if (in.zero_e) in.zero_e[m] = 0u;
        }
    }
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint64_t wide = __ballot(valid[i] && wt[i] == 2);
        uint64_t todo = __ballot(valid[i]);
        while (todo) {
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const uint32_t d = __shfl(own[i], leader, 64);
            const uint64_t mask = __ballot(valid[i] && own[i] == d);
            if (lane == leader) atomicAdd(&cnt[d], (uint32_t)(__popcll(mask) + __popcll(mask & wide)));
            todo &= ~mask;
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < in.G; d += kBlock) counts[(uint64_t)d * in.nblk + blockIdx.x] = cnt[d];
}

// (b2) one block per owner d (the columns are independent): the exclusive scan of its column of
// block counts (in place); the owner's total and the budget bit to a[2d], a[2d + 1].
__global__ void __launch_bounds__(kScanThreads1)
    slot_scan_kernel(uint32_t* __restrict__ v, uint32_t nblk, uint32_t G, SlotLayout L, uint32_t* __restrict__ a,
                     uint32_t me, uint32_t* __restrict__ out, uint32_t* __restrict__ perm, uint32_t own_budget) {
    __shared__ uint32_t wsum[kScanThreads1 / 64];
    __shared__ uint32_t carry_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t d = blockIdx.x; d < G; d += gridDim.x) {
        uint32_t* col = v + (uint64_t)d * nblk;
        if (threadIdx.x == 0) carry_s = 0;
        __syncthreads();
        for (uint32_t base = 0; base < nblk; base += kScanThreads1) {
            const uint32_t i = base + threadIdx.x;
            const uint32_t x = i < nblk ? col[i] : 0;
            const uint32_t inc = wave_incl_scan_add(x, lane);
            if (lane == 63) wsum[wave] = inc;
            __syncthreads();
            if (wave == 0) {
                const uint32_t s = lane < kScanThreads1 / 64 ? wsum[lane] : 0;
                const uint32_t si = wave_incl_scan_add(s, lane);
                if (lane < kScanThreads1 / 64) wsum[lane] = si - s;
            }
            __syncthreads();
            const uint32_t carry = carry_s;
            if (i < nblk) col[i] = carry + wsum[wave] + inc - x;
            __syncthreads();
            if (threadIdx.x == kScanThreads1 - 1) carry_s = carry + wsum[wave] + inc;
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            a[2 * d] = carry_s;
            // the own column (own slots on): no budget unless own_budget says so
            a[2 * d + 1] = carry_s > (d != me ? L.budget[d] : own_budget) ? kStBudget : 0u;
        }
        // out set (a budgeted tick): the rest of the segment padded here, as slot_pad_kernel does
        // after the scatter — the scatter writes slots [0, n) only, and past a budget it writes no
        // head whose tail does not fit, so padding first gives the same segment
        if (out && d != me) {
            const uint32_t B = L.budget[d], n = carry_s;
            const uint32_t from = n <= B ? n : (B ? B - 1 : 0);
            for (uint32_t j = from + threadIdx.x; j < B; j += blockDim.x) {
                const uint32_t slot = L.base[d] + j;
                uint32_t* o = out + (uint64_t)kSlotWords * slot;
                o[0] = 0;
                o[1] = 0;
                o[2] = 0;
                o[3] = 0;
                o[4] = kSlotTail << 8;
                perm[slot] = kNone;
            }
        }
        __syncthreads();
    }
}

// A thread's kShardIPT messages (m0 + i * kBlock) once quantised and ranked: what the scatter
// writes for a regular key (a wide key's coordinates are quantised again there, so few registers
// stay live across the base computation and every block of a tick can be resident at once).
// inf: bits 0-7 the owner (kNoOwner: no slot), 8-15 replication, 16 regular.
constexpr uint32_t kNoOwner = 0xFFu;
struct SlotRows {
    uint32_t pkl[kShardIPT], pkh[kShardIPT], ext[kShardIPT], snd[kShardIPT], inf[kShardIPT], rank[kShardIPT];
};

// (slot_scatter_kernel, slot_group_kernel) load, quantise and rank a block's messages: every load
// in flight before any is used (no branch between them: a lane past M reads message M - 1 and
// drops it), the key, owner and slot words by quantize_pack, then the ranks within the wave — the
// lanes of one owner found by log2(G') ballots of the owner's bits — and each wave-row's per-owner
// counts in wc (zeroed by the caller; a wide key counts two slots). zero: e[m] = 0 for the slot
// tick's rows (in.zero_e).
template <bool RAW>
__device__ __forceinline__ void slot_rows(const ShardIn& in, uint32_t m0, bool zero,
                                          uint32_t (*wc)[WQ_MAX_SHARDS], SlotRows& r) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1;
    const uint32_t G = in.G;
    uint64_t raw[kShardIPT][3];
    uint32_t wrd[kShardIPT], rpl[kShardIPT];
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = min(m0 + i * kBlock, in.M - 1);
        const uint64_t* src = RAW ? reinterpret_cast<const uint64_t*>(in.keys) + 3ull * m
                                  : reinterpret_cast<const uint64_t*>(in.pos) + 3ull * m;
        raw[i][0] = src[0];
        raw[i][1] = src[1];
        raw[i][2] = src[2];
        wrd[i] = in.world[m];
        r.snd[i] = in.sender[m];
        rpl[i] = in.repl[m];
    }
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        r.inf[i] = kNoOwner;
        r.rank[i] = 0;
        r.pkl[i] = r.pkh[i] = r.ext[i] = 0;
        if (m < in.M) {
            int64_t k[3];
            uint64_t pk = 0;
            bool reg;
            if (RAW) {
                k[0] = (int64_t)raw[i][0];
                k[1] = (int64_t)raw[i][1];
                k[2] = (int64_t)raw[i][2];
                reg = pack_key(wrd[i], k[0], k[1], k[2], in.sf, &pk, &r.ext[i]);
            } else {
                const double c[3] = {__longlong_as_double((long long)raw[i][0]),
                                     __longlong_as_double((long long)raw[i][1]),
                                     __longlong_as_double((long long)raw[i][2])};
                reg = quantize_pack(wrd[i], c, in.sf, in.si, k, &pk, &r.ext[i]);
            }
            const uint32_t own = shard_of(wrd[i], k[0], k[1], k[2], G);
            r.pkl[i] = (uint32_t)pk;
            r.pkh[i] = (uint32_t)(pk >> 32);
            if (own != in.me || in.own_too) r.inf[i] = own | (rpl[i] << 8) | (reg ? 1u << 16 : 0u);
        }
    }
    if (zero && in.zero_e) {
#pragma unroll
        for (int i = 0; i < kShardIPT; ++i)
            if (m0 + i * kBlock < in.M) in.zero_e[m0 + i * kBlock] = 0u;
    }
    uint32_t nbits = 0;
    while ((1u << nbits) < G) ++nbits;
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const bool go = (r.inf[i] & 0xFFu) != kNoOwner, reg = (r.inf[i] >> 16) & 1u;
        const uint32_t own = r.inf[i] & 0xFFu;
        const uint64_t wide = __ballot(go && !reg);
        uint64_t same = __ballot(go);
        for (uint32_t bit = 0; bit < nbits; ++bit) {
            const bool on = (own >> bit) & 1u;
            const uint64_t bm = __ballot(on);
            same &= on ? bm : ~bm;
        }
        if (go) {
            r.rank[i] = __popcll(same & lt) + __popcll(same & wide & lt);
            if ((same & lt) == 0) wc[i * kWaves + wave][own] = __popcll(same) + __popcll(same & wide);
        }
    }
}

// The slots of slot_rows' messages into the budgeted segments: message i of the thread at
// base[d] (nullable: 0) + wc[row][d] (the row's start within the owner's segment) + its rank. A
// message that does not fit its owner's budget whole is not written (the tick is redone exactly).
template <bool RAW>
__device__ __forceinline__ void scatter_rows(const ShardIn& in, const SlotLayout& L, uint32_t m0,
                                             const uint32_t (*wc)[WQ_MAX_SHARDS],
                                             const uint32_t* base, const SlotRows& r, uint32_t* __restrict__ out,
                                             uint32_t* __restrict__ perm) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < kShardIPT; ++i) {
        const uint32_t m = m0 + i * kBlock;
        const uint32_t d = r.inf[i] & 0xFFu;
        if (d == kNoOwner) continue;
        const bool reg = (r.inf[i] >> 16) & 1u;
        const uint32_t j = (base ? base[d] : 0u) + wc[i * kWaves + wave][d] + r.rank[i];  // within the owner's segment
        uint32_t slot;
        uint32_t* pm;
        uint32_t* o;
        if (d == in.me) {  // own slots on: this shard's own message, into its own buffer
            if (j + (reg ? 1u : 2u) > in.own_budget) continue;  // (the owner form's self segment)
            slot = j;
            pm = in.own_perm;
            o = in.own_slots + (uint64_t)kSlotWords * slot;
        } else {
            if (j + (reg ? 1u : 2u) > L.budget[d]) continue;  // over budget: the tick is redone exactly
            slot = L.base[d] + j;
            pm = perm;
            o = out + (uint64_t)kSlotWords * slot;
        }
        const uint32_t rp = (r.inf[i] >> 8) & 0xFFu;
        if (reg) {
            o[0] = r.pkl[i];
            o[1] = r.pkh[i];
            o[2] = r.ext[i];
            o[3] = r.snd[i];
            o[4] = rp | (kSlotReg << 8);
            pm[slot] = m;
        } else {  // a wide key (rare): head and tail slot with the coordinates, quantised again
            int64_t kx, ky, kz;
            msg_key<RAW>(in, m, kx, ky, kz);
            o[0] = (uint32_t)(uint64_t)kx;
            o[1] = (uint32_t)((uint64_t)kx >> 32);
            o[2] = in.world[m];
            o[3] = r.snd[i];
            o[4] = rp | (kSlotHead << 8);
            o[5] = (uint32_t)(uint64_t)ky;
            o[6] = (uint32_t)((uint64_t)ky >> 32);
            o[7] = (uint32_t)(uint64_t)kz;
            o[8] = (uint32_t)((uint64_t)kz >> 32);
            o[9] = kSlotTail << 8;
            pm[slot] = m;
            pm[slot + 1] = kNone;
        }
    }
}

// (b3) the stable ballot-ranked scatter of shard_scatter20_kernel into the budgeted segments; a
// message that does not fit its owner's budget whole is not written (nor is any after it).
template <bool RAW>
__global__ void __launch_bounds__(kBlock)
    slot_scatter_kernel(ShardIn in, const uint32_t* __restrict__ colbase, SlotLayout L, uint32_t* __restrict__ out,
                        uint32_t* __restrict__ perm) {
    __shared__ uint32_t wc[kShardIPT * kWaves][WQ_MAX_SHARDS];
    for (uint32_t k = threadIdx.x; k < kShardIPT * kWaves * WQ_MAX_SHARDS; k += kBlock) (&wc[0][0])[k] = 0;
    lds_barrier();
    if (in.a_or && blockIdx.x == 0 && threadIdx.x == 0) {  // the scan (previous launch) wrote them
        uint32_t any = 0;
        for (uint32_t d = 0; d < in.G; ++d) any |= in.a_or[2 * d + 1] & kStBudget;
        if (any)
            for (uint32_t d = 0; d < in.G; ++d) in.a_or[2 * d + 1] |= any;
    }
    const uint32_t m0 = blockIdx.x * kShardTile + threadIdx.x;
    SlotRows r;
    slot_rows<RAW>(in, m0, false, wc, r);
    lds_barrier();
    for (uint32_t d = threadIdx.x; d < in.G; d += kBlock) {
        uint32_t run = colbase[(uint64_t)d * in.nblk + blockIdx.x];
#pragma unroll
        for (int k = 0; k < kShardIPT * kWaves; ++k) {
            const uint32_t t = wc[k][d];
            wc[k][d] = run;
            run += t;
        }
    }
    lds_barrier();
    scatter_rows<RAW>(in, L, m0, wc, nullptr, r, out, perm);
}

// (b1 + b2 + b3 in one pass: a budgeted tick) block b quantises its kShardTile messages and ranks
// them per owner as slot_scatter_kernel does, publishes its per-owner counts as tagged granules
// (look[d * nblk + b]) and finds each owner's running base over the lower blocks by decoupled
// look-back (route_tick.hpp; wave 0, one group of 64 / G' lanes per owner, each lane one lower
// block per round), then scatters into the budgeted segments. A block waits only on lower-numbered
// blocks, dispatched before it, and every poll is bounded: one that gives up reports
// WQ_E_TIMEOUT in every status word instead of hanging. The last block writes the A vector (every
// owner's true count, its budget bit; with a_or the bit of any segment in all of them);
// slot_pad_kernel pads the segments after it. Against the three passes it saves the histogram
// pass's second quantisation of every message and the scan's launch.
// message tiles per grouping block: 2 halves the look-back's blocks (owner slots at G = 8: 0.1954 ->
// 0.1930 ms, alternating); 4 (159 VGPRs, occupancy 3) was slower, 0.209 ms
constexpr int kGroupTiles = 2;

struct GroupArgs {
    uint64_t* look;  // [G * nblk] granules
    uint32_t tag;    // this launch's tag, 1 .. 2^30 - 1
    uint32_t* a;     // the A vector: {count, status} per owner
    // the owner form's in-place self segment: its {count, status} straight into the received A
    // vector as well (the exchange then skips the self copy), nullable
    uint32_t* a_self = nullptr;
    uint32_t self = 0;
};

template <bool RAW>
__global__ void __launch_bounds__(kBlock)
    slot_group_kernel(ShardIn in, SlotLayout L, uint32_t* __restrict__ out, uint32_t* __restrict__ perm, GroupArgs g) {
    __shared__ uint32_t wc[kGroupTiles * kShardIPT * kWaves][WQ_MAX_SHARDS];
    __shared__ uint32_t bcnt[WQ_MAX_SHARDS], base[WQ_MAX_SHARDS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t b = blockIdx.x, NB = in.nblk, G = in.G;
    for (uint32_t k = threadIdx.x; k < kGroupTiles * kShardIPT * kWaves * WQ_MAX_SHARDS; k += kBlock) (&wc[0][0])[k] = 0;
    lds_barrier();
    const uint32_t m0 = b * (kGroupTiles * kShardTile) + threadIdx.x;
    SlotRows r[kGroupTiles];
#pragma unroll
    for (int t = 0; t < kGroupTiles; ++t) slot_rows<RAW>(in, m0 + t * kShardTile, true, wc + t * kShardIPT * kWaves, r[t]);
    lds_barrier();
    // the block's per-owner totals (published at once) and its rows' offsets within the block
    for (uint32_t d = threadIdx.x; d < G; d += kBlock) {
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < kGroupTiles * kShardIPT * kWaves; ++k) {
            const uint32_t t = wc[k][d];
            wc[k][d] = run;
            run += t;
        }
        bcnt[d] = run;
        __hip_atomic_store(g.look + (uint64_t)d * NB + b, granule(g.tag, b == 0 ? kFlagP : kFlagA, run),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lds_barrier();
    if (wave == 0) {
        // lanes [d * W, d * W + W) look back for owner d, lane k of the group at block b - 1 - (r W + k)
        uint32_t Gp = 1;
        while (Gp < G) Gp <<= 1;
        const uint32_t W = 64u / Gp, d = (uint32_t)lane / W, k = (uint32_t)lane % W;
        const uint64_t gmask = (W == 64 ? ~0ull : ((1ull << W) - 1ull)) << (d * W);
        uint64_t acc = 0;
        bool gave_up = false, done = d >= G || b == 0;
        for (int64_t hi = (int64_t)b - 1; __ballot(!done); hi -= W) {
            const int64_t idx = hi - (int64_t)k;
            uint64_t v = 0;
            if (!done && idx >= 0) v = poll_granule(g.look + (uint64_t)d * NB + idx, g.tag, &gave_up);
            const bool isP = !done && idx >= 0 && ((uint32_t)(v >> 32) & 3u) == kFlagP;
            const uint64_t pm = __ballot(isP) & gmask;
            const uint32_t first = pm ? (uint32_t)__builtin_ctzll(pm) - d * W : W;  // nearest inclusive prefix
            uint64_t x = (!done && idx >= 0 && k <= first) ? (uint32_t)v : 0u;
            for (uint32_t o = W >> 1; o >= 1; o >>= 1) x += __shfl_xor(x, (int)o, 64);  // the group's sum
            if (!done) acc += x;
            // the group is done at an inclusive prefix or past block 0
            if (pm || hi - (int64_t)W < 0) done = true;
        }
        if (d < G && k == 0) {
            base[d] = (uint32_t)acc;
            if (b > 0)
                __hip_atomic_store(g.look + (uint64_t)d * NB + b, granule(g.tag, kFlagP, (uint32_t)acc + bcnt[d]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (__any(gave_up) && lane == 0) {  // WQ_E_TIMEOUT (status code 7) in every status word
            for (uint32_t q = 0; q < G; ++q) atomicOr(&g.a[2 * q + 1], 7u);
            if (g.a_self) atomicOr(&g.a_self[1], 7u);
        }
    }
    lds_barrier();
    if (b == NB - 1) {  // the last block knows every owner's true count
        for (uint32_t d = threadIdx.x; d < G; d += kBlock) {
            const uint32_t n = base[d] + bcnt[d];
            g.a[2 * d] = n;
            // the own column (own slots on): no budget unless own_budget says so
            if (n > (d != in.me ? L.budget[d] : in.own_budget)) atomicOr(&g.a[2 * d + 1], kStBudget);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            if (in.a_or) {
                uint32_t any = 0;
                for (uint32_t d = 0; d < G; ++d) any |= in.a_or[2 * d + 1] & kStBudget;
                if (any)
                    for (uint32_t d = 0; d < G; ++d) atomicOr(&in.a_or[2 * d + 1], any);
            }
            if (g.a_self) {
                g.a_self[0] = g.a[2 * g.self];
                atomicOr(&g.a_self[1], g.a[2 * g.self + 1]);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < kGroupTiles; ++t)
        scatter_rows<RAW>(in, L, m0 + t * kShardTile, wc + t * kShardIPT * kWaves, base, r[t], out, perm);
}

// (b4) the unused rest of every segment becomes tail slots (route to nobody; perm kNone), so the
// owner can count its whole receive budget without knowing the true counts. Over budget, the last
// slot of the segment is overwritten as well (a head whose tail did not fit); that tick is redone.
__global__ void __launch_bounds__(kBlock)
    slot_pad_kernel(SlotLayout L, uint32_t G, const uint32_t* __restrict__ a, uint32_t* __restrict__ out,
                    uint32_t* __restrict__ perm, uint32_t own_d, uint32_t* __restrict__ own_out,
                    uint32_t* __restrict__ own_perm, uint32_t own_budget) {
    const uint32_t d = blockIdx.y;
    if (d >= G) return;
    // own_d: the owner form's self segment, written in place into the receive buffer
    const bool ownd = d == own_d;
    if (ownd) {
        out = own_out;
        perm = own_perm;
    }
    const uint32_t B = ownd ? own_budget : L.budget[d], n = a[2 * d];
    // n == B: every slot fit, nothing of the segment is overwritten; n > B: the last slot may be a
    // head whose tail did not fit, so it becomes a tail too (the tick is redone)
    const uint32_t from = n <= B ? n : (B ? B - 1 : 0);
    for (uint32_t j = from + blockIdx.x * kBlock + threadIdx.x; j < B; j += gridDim.x * kBlock) {
        const uint32_t slot = (ownd ? 0u : L.base[d]) + j;
        uint32_t* o = out + (uint64_t)kSlotWords * slot;
        o[0] = 0;
        o[1] = 0;
        o[2] = 0;
        o[3] = 0;
        o[4] = kSlotTail << 8;
        perm[slot] = kNone;
    }
}

__global__ void op_owner_kernel(const wq_op* __restrict__ ops, uint32_t n, double sf, int64_t si, uint32_t G,
                                uint32_t* __restrict__ owner) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const wq_op op = ops[i];
    if (op.kind == WQ_OP_REMOVE_PEER) {
        owner[i] = WQ_SHARD_ALL;
        return;
    }
    int64_t x, y, z;
    if (op.key_is_raw) {
        x = op.u.key[0];
        y = op.u.key[1];
        z = op.u.key[2];
    } else {
        x = coord_clamp_dev(op.u.pos[0], sf, si);
        y = coord_clamp_dev(op.u.pos[1], sf, si);
        z = coord_clamp_dev(op.u.pos[2], sf, si);
    }
    owner[i] = shard_of(op.world, x, y, z, G);
}

// Records -> the SoA inputs of the route passes: quantised keys, or (pos != nullptr, radius
// filter on) positions — a record without one gets NaN, which no radius test passes.
__global__ void unpack_records_kernel(const wq_msg_rec* __restrict__ r, uint32_t M, int64_t* __restrict__ keys,
                                      double* __restrict__ pos, uint32_t* __restrict__ world,
                                      uint32_t* __restrict__ sender, uint8_t* __restrict__ repl) {
    const uint32_t m = blockIdx.x * kBlock + threadIdx.x;
    if (m >= M) return;
    const wq_msg_rec x = r[m];
    if (pos) {
        const bool has = (x.flags & WQ_REC_POS) != 0;
#pragma unroll
        for (int d = 0; d < 3; ++d) pos[3ull * m + d] = has ? __longlong_as_double(x.key[d]) : __builtin_nan("");
    } else {
        keys[3ull * m] = x.key[0];
        keys[3ull * m + 1] = x.key[1];
        keys[3ull * m + 2] = x.key[2];
    }
    world[m] = x.world;
    sender[m] = x.sender;
    repl[m] = x.repl;
}

int launch_route(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                 const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                 uint32_t* d_peers, uint32_t* d_msgs, size_t capacity);

int launch_shard_messages(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                          const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, wq_msg_rec* d_out,
                          uint32_t* d_counts) {
    hipStream_t s = h->stream;
    if (M == 0) {
        WQ_HIP(h, hipMemsetAsync(d_counts, 0, G * 4, s));
        return WQ_OK;
    }
    ShardIn in;
    in.pos = d_pos;
    in.keys = d_keys;
    in.world = d_world;
    in.sender = d_sender;
    in.repl = d_repl;
    in.M = (uint32_t)M;
    in.G = G;
    in.nblk = (uint32_t)((M + kShardTile - 1) / kShardTile);
    in.sf = (double)h->cube_size;
    in.si = (int64_t)h->cube_size;
    in.pos_rec = h->radius > 0.0 && d_pos != nullptr;
    WQ_ALLOC(h, h->shard_hist, (uint64_t)in.nblk * G * 4);
    uint32_t* hist = h->shard_hist.as<uint32_t>();
    if (d_keys)
        hipLaunchKernelGGL((shard_count_kernel<true>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist);
    else
        hipLaunchKernelGGL((shard_count_kernel<false>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist);
    WQ_HIP(h, hipGetLastError());
    hipLaunchKernelGGL(shard_scan_kernel, dim3(1), dim3(kScanThreads1), 0, s, hist, in.nblk, G, d_counts, 1u);
    WQ_HIP(h, hipGetLastError());
    if (d_keys)
        hipLaunchKernelGGL((shard_scatter_kernel<true>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist, d_out);
    else
        hipLaunchKernelGGL((shard_scatter_kernel<false>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist, d_out);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

// Compact slots (see shard_scatter20_kernel): d_slots holds up to 2M slots of kSlotWords words,
// d_perm 2M words; the slot count for owner d lands at d_counts[d * stride].
int launch_shard_slots(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                       const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, uint32_t* d_slots,
                       uint32_t* d_perm, uint32_t* d_counts, uint32_t stride) {
    hipStream_t s = h->stream;
    if (M == 0) return WQ_OK;  // the caller zeroed the counts
    ShardIn in;
    in.pos = d_pos;
    in.keys = d_keys;
    in.world = d_world;
    in.sender = d_sender;
    in.repl = d_repl;
    in.M = (uint32_t)M;
    in.G = G;
    in.nblk = (uint32_t)((M + kShardTile - 1) / kShardTile);
    in.sf = (double)h->cube_size;
    in.si = (int64_t)h->cube_size;
    in.pos_rec = false;
    WQ_ALLOC(h, h->shard_hist, (uint64_t)in.nblk * G * 4);
    uint32_t* hist = h->shard_hist.as<uint32_t>();
    if (d_keys)
        hipLaunchKernelGGL((shard_count_kernel<true, true>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist);
    else
        hipLaunchKernelGGL((shard_count_kernel<false, true>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist);
    WQ_HIP(h, hipGetLastError());
    hipLaunchKernelGGL(shard_scan_kernel, dim3(1), dim3(kScanThreads1), 0, s, hist, in.nblk, G, d_counts, stride);
    WQ_HIP(h, hipGetLastError());
    if (d_keys)
        hipLaunchKernelGGL((shard_scatter20_kernel<true>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist, d_slots, d_perm);
    else
        hipLaunchKernelGGL((shard_scatter20_kernel<false>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist, d_slots,
                           d_perm);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

// Budgeted slots of this shard's messages owned by other shards (the slot_* kernels above): the
// slots in L's segments of d_slots, perm[slot] = message (kNone for tails and padding), the true
// count and budget bit per owner at d_a[2d], d_a[2d + 1] (zeroed for this shard itself).
// phases: 1 = the counts only (histogram + scan), 2 = the scatter and padding after them, 3 = both.
// me = G (no shard) with own_too: every message is a slot of its owner's budgeted segment, this
// shard's own ones included (the owner form); row_any: see ShardIn::a_or.
int launch_budget_slots(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                        const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, uint32_t me,
                        const SlotLayout& L, uint32_t* d_slots, uint32_t* d_perm, uint32_t* d_a, int phases,
                        bool hist_ready, bool own_too, uint32_t* own_slots, uint32_t* own_perm, uint32_t* zero_e,
                        bool row_any, uint32_t own_budget, uint32_t* a_self) {
    hipStream_t s = h->stream;
    ShardIn in;
    in.pos = d_pos;
    in.keys = d_keys;
    in.world = d_world;
    in.sender = d_sender;
    in.repl = d_repl;
    in.M = (uint32_t)M;
    in.G = G;
    in.nblk = (uint32_t)((M + kShardTile - 1) / kShardTile);
    in.sf = (double)h->cube_size;
    in.si = (int64_t)h->cube_size;
    in.pos_rec = false;
    in.me = me;
    in.own_too = own_too;
    in.own_slots = own_slots;
    in.own_perm = own_perm;
    in.zero_e = zero_e;
    in.own_budget = own_budget;
    in.a_or = row_any && (phases & 3) == 3 ? d_a : nullptr;
    // the owner form's self segment in place: slot_pad_kernel pads it (the scan pads only the others)
    const bool own_in_place = own_slots && own_budget != 0xFFFFFFFFu;
    const uint32_t own_d = own_in_place ? me : G;
    // a budgeted tick (count, scan and scatter in one call): the one-pass grouping, then the padding
    // (WQ_DEBUG_SLOT_3PASS: the three passes, diagnostics)
    static const bool three_pass = getenv("WQ_DEBUG_SLOT_3PASS") != nullptr;
    if (M && (phases & 3) == 3 && d_slots && !hist_ready && !three_pass) {
        in.nblk = (uint32_t)((M + kGroupTiles * kShardTile - 1) / (kGroupTiles * kShardTile));
        const uint64_t ng = (uint64_t)G * in.nblk;
        WQ_ALLOC(h, h->shard_look, ng * 8);
        if (h->shard_look_zeroed < ng) {  // fresh granules: tag 0 never matches a launch's tag
            WQ_HIP(h, hipMemsetAsync(h->shard_look.p, 0, h->shard_look.bytes, s));
            h->shard_look_zeroed = h->shard_look.bytes / 8;
        }
        GroupArgs ga{h->shard_look.as<uint64_t>(), (uint32_t)(h->shard_look_calls++ % ((1ull << 30) - 1)) + 1u, d_a,
                     a_self, me};
        if (d_keys)
            hipLaunchKernelGGL((slot_group_kernel<true>), dim3(in.nblk), dim3(kBlock), 0, s, in, L, d_slots, d_perm, ga);
        else
            hipLaunchKernelGGL((slot_group_kernel<false>), dim3(in.nblk), dim3(kBlock), 0, s, in, L, d_slots, d_perm, ga);
        WQ_HIP(h, hipGetLastError());
        uint32_t bmax = own_in_place ? own_budget : 0u;
        for (uint32_t d = 0; d < G; ++d) bmax = std::max(bmax, L.budget[d]);
        if (bmax) {
            const unsigned gx = std::min<unsigned>(64u, (bmax + kBlock - 1) / kBlock);
            hipLaunchKernelGGL(slot_pad_kernel, dim3(gx, G), dim3(kBlock), 0, s, L, G, d_a, d_slots, d_perm, own_d,
                               own_slots, own_perm, own_budget);
            WQ_HIP(h, hipGetLastError());
        }
        return WQ_OK;
    }
    if (M && (phases & 1)) {
        WQ_ALLOC(h, h->shard_hist, (uint64_t)in.nblk * G * 4);
        uint32_t* hist = h->shard_hist.as<uint32_t>();
        if (hist_ready) {
            // the caller's own-cube count wrote it (wq_sharded.hip own_count_hist_kernel)
        } else if (d_keys)
            hipLaunchKernelGGL((slot_count_kernel<true>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist);
        else
            hipLaunchKernelGGL((slot_count_kernel<false>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist);
        WQ_HIP(h, hipGetLastError());
        // a budgeted tick (count, scan and scatter in one call) pads its segments in the scan
        const bool pad_in_scan = (phases & 3) == 3 && d_slots;
        hipLaunchKernelGGL(slot_scan_kernel, dim3(G), dim3(kScanThreads1), 0, s, hist, in.nblk, G, L, d_a, me,
                           pad_in_scan ? d_slots : nullptr, pad_in_scan ? d_perm : nullptr, own_budget);
        WQ_HIP(h, hipGetLastError());
    } else if (phases & 1) {
        WQ_HIP(h, hipMemsetAsync(d_a, 0, 8 * G, s));
    }
    if (!(phases & 2)) return WQ_OK;
    if (M) {
        uint32_t* hist = h->shard_hist.as<uint32_t>();
        if (d_keys)
            hipLaunchKernelGGL((slot_scatter_kernel<true>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist, L, d_slots,
                               d_perm);
        else
            hipLaunchKernelGGL((slot_scatter_kernel<false>), dim3(in.nblk), dim3(kBlock), 0, s, in, hist, L, d_slots,
                               d_perm);
        WQ_HIP(h, hipGetLastError());
    }
    uint32_t bmax = 0;
    for (uint32_t d = 0; d < G; ++d) bmax = std::max(bmax, L.budget[d]);
    if (own_in_place) bmax = std::max(bmax, own_budget);
    // (phases 3 with messages: padded by the scan, all but an in-place self segment)
    if (bmax && (!(M && (phases & 3) == 3) || own_in_place)) {
        const unsigned gx = std::min<unsigned>(64u, (bmax + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(slot_pad_kernel, dim3(gx, G), dim3(kBlock), 0, s, L, G, d_a, d_slots, d_perm, own_d,
                           own_slots, own_perm, own_budget);
        WQ_HIP(h, hipGetLastError());
    }
    return WQ_OK;
}

uint32_t budget_slot_tile() { return kShardTile; }

int launch_op_owner(wq_router* h, const wq_op* d_ops, size_t n, uint32_t G, uint32_t* d_owner) {
    if (n == 0) return WQ_OK;
    hipLaunchKernelGGL(op_owner_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, h->stream,
                       d_ops, (uint32_t)n, (double)h->cube_size, (int64_t)h->cube_size, G, d_owner);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

int launch_route_records(wq_router* h, const wq_msg_rec* d_recs, size_t M, uint32_t* d_offsets, uint32_t* d_peers,
                         uint32_t* d_msgs, size_t capacity) {
    WQ_ALLOC(h, h->rec_keys, M * 24 + 256);  // keys, or positions with the radius filter on
    WQ_ALLOC(h, h->rec_w, M * 4 + 256);
    WQ_ALLOC(h, h->rec_s, M * 4 + 256);
    WQ_ALLOC(h, h->rec_r, M + 256);
    const bool radius = h->radius > 0.0;
    if (M) {
        hipLaunchKernelGGL(unpack_records_kernel, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           h->stream, d_recs, (uint32_t)M, h->rec_keys.as<int64_t>(),
                           radius ? h->rec_keys.as<double>() : nullptr, h->rec_w.as<uint32_t>(),
                           h->rec_s.as<uint32_t>(), h->rec_r.as<uint8_t>());
        WQ_HIP(h, hipGetLastError());
    }
    return launch_route(h, radius ? h->rec_keys.as<double>() : nullptr, radius ? nullptr : h->rec_keys.as<int64_t>(),
                        h->rec_w.as<uint32_t>(), h->rec_s.as<uint32_t>(), h->rec_r.as<uint8_t>(), M, d_offsets, d_peers,
                        d_msgs, capacity);
}

}  // namespace wq
