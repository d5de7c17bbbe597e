// wq_route.hip — the LocalMessage hot path on gfx950: one tick of messages in three launches.
//
// Replaces, per message, worldql_server/src/processing/local_message.rs:52-86:
//   world_map.get(world) -> Vector3::to_cube_area (cube_area.rs:72-77 -> coord_clamp :23-44)
//   -> AreaMap::get_subscribed_peers (area_map.rs:52-60) -> replication filter (:60-86).
//
// 1. count_kernel   quantise (kernel 1) + exact packed key per message (one lane per message,
//                   coalesced inputs), then the table probe (kernel 2) with EIGHT lanes per
//                   message: one coalesced 128-byte load of the bucket record line (key, count,
//                   28 inline peers) per 8 lanes, the sender compared against the inline peers
//                   in parallel and reduced with lane shuffles. Writes the filtered count e_m
//                   into offsets[m] and an 8-byte locator (record slot + count / list offset /
//                   "the sender itself", skipped index). No LDS round trips, no inter-block waits.
// 2. scan_kernel    in-place exclusive scan of offsets[] (single pass, decoupled look-back over
//                   4096-message tiles; uniform tiny tiles, so no convoy) -> CSR offsets, P.
// 3. emit_kernel    load-balanced expand + compaction (kernel 3): a tile stages its messages'
//                   inline peer lists in LDS (8 lanes per record line again; the table is
//                   Infinity-Cache resident since pass 1), marks each message's first output in
//                   an LDS owner array, max-scans it, and writes output j with thread j % 256 —
//                   one coalesced stream per tile whatever the fan-out skew.
// A single fused launch was measured first: its decoupled look-back made
// every tile wait for the slowest earlier tile's probes (p50 13 us, max 47 us per tile), capping
// it at 115-135 us per C2 tick. The split re-reads the record lines once and removes every wait.
// Output: CSR offsets[M+1] (message-major), peers[P], optional msgs[P].
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

// scan status word: [epoch:24][flag:2][value:38]
constexpr int kValBits = 38;
constexpr uint64_t kValMask = (1ull << kValBits) - 1;
constexpr uint64_t kFlagAgg = 1ull;
constexpr uint64_t kFlagPre = 2ull;
constexpr uint32_t kSpinLimit = 1u << 22;

__device__ __forceinline__ uint64_t make_status(uint32_t epoch, uint64_t flag, uint64_t v) {
    return ((uint64_t)epoch << (kValBits + 2)) | (flag << kValBits) | (v & kValMask);
}
__device__ __forceinline__ uint64_t ld_status(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

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

struct RouteIn {
    const double* pos;
    const int64_t* keys;
    const uint32_t* world;
    const uint32_t* sender;
    const uint8_t* repl;
    uint32_t M;
    int64_t si;
};

// ------------------------------------------------------------------------------------------
// 1. count
// ------------------------------------------------------------------------------------------
struct CountParams {
    RouteIn in;
    TableView t;
    uint32_t* offsets;  // out: e_m (scanned in place by scan_kernel)
    uint2* info;        // out: locator
    wq_route_counters* cnt;
    wq_route_counters* cnt_next;
};

constexpr uint32_t kMetaValid = 1u, kMetaDone = 2u;  // meta: flags | repl << 8

template <int IPT>
struct CountSmem {
    uint64_t pk[kBlock * IPT];
    uint32_t slot[kBlock * IPT];
    uint32_t me[kBlock * IPT];
    uint32_t meta[kBlock * IPT];
    uint64_t wave_F[kWaves];
};

// e / locator once count, membership and list position are known (local_message.rs:60-86)
__device__ __forceinline__ void finish_message(uint32_t cnt, uint8_t rp, bool inl, uint32_t rslot, uint32_t loff,
                                               uint32_t at, bool has, uint32_t* e, uint2* info) {
    if (cnt == 0) {
        *e = 0;
        *info = make_uint2(0, kNone);
    } else if (rp == WQ_REPL_INCLUDING_SELF) {  // :70-75
        *e = cnt;
        *info = inl ? make_uint2(rslot, (cnt << 24) | kSkipNone24) : make_uint2(kLocGlobal | loff, kNone);
    } else if (rp == WQ_REPL_ONLY_SELF) {  // :77-85, the sender only if subscribed
        *e = has ? 1u : 0u;
        *info = make_uint2(kLocSelf, kNone);
    } else {  // ExceptSelf and unknown codes (replication.rs:40), :61-68
        *e = cnt - (has ? 1u : 0u);
        *info = inl ? make_uint2(rslot, (cnt << 24) | (has ? at : kSkipNone24))
                    : make_uint2(kLocGlobal | loff, has ? at : kNone);
    }
}

template <bool RAW_KEYS, int IPT, int U>
__global__ __launch_bounds__(kBlock) void count_kernel(CountParams p) {
    constexpr int TILE = kBlock * IPT;
    __shared__ CountSmem<IPT> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TableView& tv = p.t;
    if (blockIdx.x == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    const uint32_t m0 = blockIdx.x * TILE;
    uint64_t F_local = 0;

    // ---- A: one lane per message — inputs, quantise, packed key, home slot ----
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t j = i * kBlock + tid;
        const uint32_t m = m0 + j;
        const bool valid = m < p.in.M;
        const uint32_t mm = valid ? m : 0;
        const uint32_t w = p.in.world[mm];
        const uint32_t me = p.in.sender[mm];
        const uint8_t rp = p.in.repl[mm];
        int64_t x, y, z;
        if (RAW_KEYS) {
            x = p.in.keys[3ull * mm];
            y = p.in.keys[3ull * mm + 1];
            z = p.in.keys[3ull * mm + 2];
        } else {
            x = coord_clamp_dev(p.in.pos[3ull * mm], tv.sf, p.in.si);
            y = coord_clamp_dev(p.in.pos[3ull * mm + 1], tv.sf, p.in.si);
            z = coord_clamp_dev(p.in.pos[3ull * mm + 2], tv.sf, p.in.si);
        }
        uint64_t pk = 0;
        const bool reg = pack_key(w, x, y, z, tv.sf, &pk);
        uint32_t meta = (valid ? kMetaValid : 0u) | ((uint32_t)rp << 8);
        if (valid && !reg) {  // full-key slot table: rare, finished here one lane per message
            const uint32_t loff = probe(tv.slots, tv.slot_mask, tv.slot_shift, cube_hash(w, x, y, z) & tv.hash_mask,
                                        w, x, y, z);
            const uint32_t cnt = loff != kNone ? tv.list[loff] : 0u;
            uint32_t at = 0;
            bool has = false;
            if (cnt && rp != WQ_REPL_INCLUDING_SELF) {
                const uint32_t* lp = tv.list + loff + 1;
                at = lower_bound_dev(lp, cnt, me);
                has = at < cnt && lp[at] == me;
            }
            uint32_t e;
            uint2 inf;
            finish_message(cnt, rp, false, 0, loff, at, has, &e, &inf);
            p.offsets[m] = e;
            p.info[m] = inf;
            F_local += cnt;
            meta |= kMetaDone;
        }
        sm.pk[j] = pk;
        sm.slot[j] = reg ? (uint32_t)slot_of(rec_hash(pk) & tv.hash_mask, tv.rec_shift) : 0u;
        sm.me[j] = me;
        sm.meta[j] = meta;
    }
    lds_barrier();

    // ---- B: eight lanes per message — one coalesced record-line load, parallel compare ----
    const int grp = lane >> 3, part = lane & 7;
    const uint4* recs4 = reinterpret_cast<const uint4*>(tv.recs);
    for (int r0 = 0; r0 < 8 * IPT; r0 += U) {
        uint4 v[U];
        uint32_t jj[U], sl[U], meta[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            jj[u] = wave_msg<IPT>(wave, 8 * (r0 + u) + grp);
            meta[u] = sm.meta[jj[u]];
            sl[u] = sm.slot[jj[u]];
            const bool act = (meta[u] & (kMetaValid | kMetaDone)) == kMetaValid;
            v[u] = act ? recs4[(uint64_t)sl[u] * 8 + part] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if ((meta[u] & (kMetaValid | kMetaDone)) != kMetaValid) continue;  // uniform per group
            const uint64_t pk = sm.pk[jj[u]];
            const uint32_t me = sm.me[jj[u]];
            const uint8_t rp = (uint8_t)(meta[u] >> 8);
            const int lead = lane & ~7;
            uint32_t hx = __shfl(v[u].x, lead, 64), hy = __shfl(v[u].y, lead, 64);
            uint32_t hz = __shfl(v[u].z, lead, 64), hw = __shfl(v[u].w, lead, 64);
            uint64_t key = ((uint64_t)hy << 32) | hx;
            while (key != 0 && key != pk) {  // collision walk, whole group in step
                sl[u] = (sl[u] + 1) & (uint32_t)tv.rec_mask;
                v[u] = recs4[(uint64_t)sl[u] * 8 + part];
                hx = __shfl(v[u].x, lead, 64);
                hy = __shfl(v[u].y, lead, 64);
                hz = __shfl(v[u].z, lead, 64);
                hw = __shfl(v[u].w, lead, 64);
                key = ((uint64_t)hy << 32) | hx;
            }
            const uint32_t cnt = key != 0 ? hz : 0u;
            const bool inl = cnt <= (uint32_t)kInline;
            uint32_t lt = 0, eq = 0;
            if (cnt && inl && rp != WQ_REPL_INCLUDING_SELF && part > 0) {
                const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                    const uint32_t idx = 4 * (part - 1) + e4;
                    if (idx < cnt) {
                        lt += vv[e4] < me ? 1u : 0u;
                        eq |= vv[e4] == me ? 1u : 0u;
                    }
                }
            }
#pragma unroll
            for (int d = 1; d < 8; d <<= 1) {
                lt += __shfl_xor(lt, d, 64);
                eq |= __shfl_xor(eq, d, 64);
            }
            if (part == 0) {
                uint32_t at = lt;
                bool has = eq != 0;
                if (cnt && !inl && rp != WQ_REPL_INCLUDING_SELF) {  // > 28 peers: search the full list
                    const uint32_t* lp = tv.list + hw + 1;
                    at = lower_bound_dev(lp, cnt, me);
                    has = at < cnt && lp[at] == me;
                }
                uint32_t e;
                uint2 inf;
                finish_message(cnt, rp, inl, sl[u], hw, at, has, &e, &inf);
                const uint32_t m = m0 + jj[u];
                p.offsets[m] = e;
                p.info[m] = inf;
                F_local += cnt;
            }
        }
    }

    const uint64_t Fw = wave_sum_u64(F_local);
    if (lane == 0) sm.wave_F[wave] = Fw;
    lds_barrier();
    if (tid == 0) {
        uint64_t Fb = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) Fb += sm.wave_F[w];
        if (Fb) atomicAdd(reinterpret_cast<unsigned long long*>(&p.cnt->n_candidates), (unsigned long long)Fb);
    }
}

// ------------------------------------------------------------------------------------------
// 2. scan: offsets[0..M) in place, exclusive; offsets[M] = P
// ------------------------------------------------------------------------------------------
constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;

struct ScanParams {
    uint32_t* offsets;
    uint32_t M;
    uint32_t n_tiles;
    uint64_t* status;
    unsigned long long* ticket;
    uint64_t ticket_base;
    uint32_t epoch;
    uint64_t capacity;
    wq_route_counters* cnt;
};

__global__ __launch_bounds__(kBlock) void scan_kernel(ScanParams p) {
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_prefix;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // tile order from a ticket: a tile only waits on tiles dequeued before it by running blocks
    if (tid == 0) s_tile = (uint32_t)(atomicAdd(p.ticket, 1ull) - p.ticket_base);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t b0 = tile * kScanTile + tid * kScanItems;
    uint32_t v[kScanItems];
    uint32_t tsum = 0;
    if (b0 + kScanItems <= p.M) {
        const uint4* src = reinterpret_cast<const uint4*>(p.offsets + b0);
#pragma unroll
        for (int q = 0; q < kScanItems / 4; ++q) {
            const uint4 x = src[q];
            v[4 * q] = x.x;
            v[4 * q + 1] = x.y;
            v[4 * q + 2] = x.z;
            v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k) v[k] = (b0 + k < p.M) ? p.offsets[b0 + k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) tsum += v[k];
    const uint32_t incl = wave_incl_scan_add(tsum, lane);
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t wbase = 0, T = 0;
#pragma unroll
    for (int u = 0; u < kWaves; ++u) {
        const uint32_t t = s_wave[u];
        if (u < wave) wbase += t;
        T += t;
    }
    if (wave == 0) {
        uint64_t excl = 0;
        if (tile == 0) {
            if (lane == 0) st_status(&p.status[0], make_status(p.epoch, kFlagPre, T));
        } else {
            if (lane == 0) st_status(&p.status[tile], make_status(p.epoch, kFlagAgg, T));
            int64_t q0 = (int64_t)tile - 1;
            uint32_t spins = 0;
            for (;;) {
                const int64_t q = q0 - lane;
                uint64_t fl = kFlagPre, val = 0;
                if (q >= 0) {
                    const uint64_t s = ld_status(&p.status[q]);
                    const bool mine = (uint32_t)(s >> (kValBits + 2)) == p.epoch;
                    fl = mine ? ((s >> kValBits) & 3ull) : 0ull;
                    val = s & kValMask;
                }
                const uint64_t pre = __ballot(fl == kFlagPre);
                const uint64_t zero = __ballot(fl == 0);
                const int first_pre = pre ? __builtin_ctzll(pre) : 64;
                const uint64_t need = (first_pre >= 63) ? ~0ull : ((2ull << first_pre) - 1);
                if ((zero & need) && spins < kSpinLimit) {
                    ++spins;
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                if ((zero & need) && lane == 0) atomicOr(&p.cnt->error, 1u);  // gave up
                excl += wave_sum_u64((lane <= first_pre && fl != 0) ? val : 0);
                if (first_pre < 64) break;
                q0 -= 64;
            }
            if (lane == 0) st_status(&p.status[tile], make_status(p.epoch, kFlagPre, excl + T));
        }
        if (lane == 0) s_prefix = excl;
    }
    __syncthreads();
    const uint64_t prefix = s_prefix;
    uint32_t run = (uint32_t)prefix + wbase + incl - tsum;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint32_t x = v[k];
        v[k] = run;
        run += x;
    }
    if (b0 + kScanItems <= p.M) {
        uint4* dst = reinterpret_cast<uint4*>(p.offsets + b0);
#pragma unroll
        for (int q = 0; q < kScanItems / 4; ++q) dst[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k)
            if (b0 + k < p.M) p.offsets[b0 + k] = v[k];
    }
    if (tile == p.n_tiles - 1 && tid == 0) {
        const uint64_t P = prefix + T;
        p.offsets[p.M] = (uint32_t)P;
        p.cnt->n_pairs = P;
        if (P > p.capacity) atomicOr(&p.cnt->overflow, 1u);
        if (P > 0xFFFFFFFFull) atomicOr(&p.cnt->error, 2u);
    }
}

// ------------------------------------------------------------------------------------------
// 3. emit
// ------------------------------------------------------------------------------------------
struct EmitParams {
    const uint32_t* sender;
    uint32_t M;
    TableView t;
    const uint32_t* offsets;
    const uint2* info;
    uint32_t* peers;
    uint32_t* msgs;
    uint64_t capacity;
};

// owner marks: [generation:20][1 + message index:12] — one generation per expansion chunk, so
// stale marks of earlier chunks lose every max and the array never needs clearing.
constexpr int kOwnerIdxBits = 12;
constexpr uint32_t kOwnerIdxMask = (1u << kOwnerIdxBits) - 1;
constexpr uint32_t kMaxGen = (1u << (32 - kOwnerIdxBits)) - 1;

template <int IPT, int CHUNK, int STAGE>
struct EmitSmem {
    uint32_t stage[STAGE];          // staged inline peer lists (tile-local, compacted)
    uint32_t base[kBlock * IPT];    // stage index (or kGlobal | list index) of the message's output 0
    uint32_t skip[kBlock * IPT];    // output index at which the sender is skipped, or kNone
    uint32_t start[kBlock * IPT];   // tile-local first output of the message
    uint32_t slot[kBlock * IPT];    // record slot to stage from, or kNone
    uint32_t spos[kBlock * IPT];    // stage position / count for the staging pass
    uint32_t owner[2][CHUNK];       // double-buffered tagged owner of each chunk output
    uint32_t wave_tot[kWaves];
};

template <int IPT, int CHUNK, int STAGE, int U>
__global__ __launch_bounds__(kBlock) void emit_kernel(EmitParams p) {
    constexpr int TILE = kBlock * IPT;
    constexpr int PER = CHUNK / kBlock;
    static_assert(CHUNK % kBlock == 0 && TILE < (1 << kOwnerIdxBits), "bad emit shape");
    __shared__ EmitSmem<IPT, CHUNK, STAGE> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TableView& tv = p.t;
    const uint32_t m0 = blockIdx.x * TILE;
    const uint32_t m_end = min(p.M, m0 + TILE);
    const uint32_t g0 = p.offsets[m0];
    const uint32_t T = p.offsets[m_end] - g0;

    // ---- A: one lane per message — counts, locators, stage positions ----
    uint32_t e[IPT], st[IPT], sc[IPT];
    uint2 inf[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * kBlock + tid;
        const bool valid = m < p.M;
        const uint32_t mm = valid ? m : p.M - 1;
        const uint32_t a = p.offsets[mm], b = p.offsets[mm + 1];
        e[i] = valid ? b - a : 0u;
        st[i] = a - g0;
        inf[i] = p.info[mm];
        const bool rec = !(inf[i].x & (kLocGlobal | kLocSelf));
        sc[i] = !e[i] ? 0u : rec ? (inf[i].y >> 24) : (inf[i].x & kLocSelf) ? 1u : 0u;
    }
    uint32_t run;
    {
        uint32_t tsum = 0;
#pragma unroll
        for (int i = 0; i < IPT; ++i) tsum += sc[i];
        const uint32_t incl = wave_incl_scan_add(tsum, lane);
        if (lane == 63) sm.wave_tot[wave] = incl;
        lds_barrier();
        run = incl - tsum;
#pragma unroll
        for (int u = 0; u < kWaves; ++u)
            if (u < wave) run += sm.wave_tot[u];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t j = i * kBlock + tid;
        const uint32_t pos = run;
        run += sc[i];
        const bool fits = pos + sc[i] <= (uint32_t)STAGE;
        const bool rec = !(inf[i].x & (kLocGlobal | kLocSelf));
        uint32_t base = 0, skip = kNone, slot = kNone;
        if (e[i]) {
            if (inf[i].x & kLocGlobal) {
                base = kGlobal | ((inf[i].x & ~kLocGlobal) + 1);
                skip = inf[i].y;
            } else if (inf[i].x & kLocSelf) {
                base = fits ? pos : kSelfSentinel;
                if (fits) sm.stage[pos] = p.sender[m0 + j];
            } else {
                const uint32_t s24 = inf[i].y & kSkipNone24;
                skip = s24 == kSkipNone24 ? kNone : s24;
                if (fits) {
                    base = pos;
                    slot = inf[i].x;
                } else {  // stage full: read the full list from HBM (offset in the record header)
                    base = kGlobal | (tv.recs[inf[i].x].list_off + 1);
                }
            }
        }
        (void)rec;
        sm.base[j] = base;
        sm.skip[j] = skip;
        sm.start[j] = st[i];
        sm.slot[j] = slot;
        sm.spos[j] = (pos << 8) | sc[i];
    }
    lds_barrier();

    // ---- B: eight lanes per record line — stage the inline peers ----
    {
        const int grp = lane >> 3, part = lane & 7;
        const uint4* recs4 = reinterpret_cast<const uint4*>(tv.recs);
        for (int r0 = 0; r0 < 8 * IPT; r0 += U) {
            uint4 v[U];
            uint32_t sp[U];
            bool act[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = wave_msg<IPT>(wave, 8 * (r0 + u) + grp);
                const uint32_t sl = sm.slot[j];
                sp[u] = sm.spos[j];
                act[u] = sl != kNone && part > 0;
                v[u] = act[u] ? recs4[(uint64_t)sl * 8 + part] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!act[u]) continue;
                const uint32_t pos = sp[u] >> 8, cnt = sp[u] & 0xFF;
                const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                    const uint32_t idx = 4 * (part - 1) + e4;
                    if (idx < cnt) sm.stage[pos + idx] = vv[e4];
                }
            }
        }
    }
    lds_barrier();

    // ---- C: expand + compact, CHUNK outputs at a time ----
    uint32_t gen = 0;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < T; c0 += CHUNK) {
        if (gen == 0 || gen == kMaxGen) {  // first chunk of the block / tag space exhausted
#pragma unroll
            for (int x = 0; x < 2 * PER; ++x) (&sm.owner[0][0])[x * kBlock + tid] = 0;
            gen = 0;
            lds_barrier();
        }
        ++gen;
        uint32_t* own = sm.owner[gen & 1];
        const uint32_t tag = gen << kOwnerIdxBits;
#pragma unroll
        for (int i = 0; i < IPT; ++i)
            if (e[i] && st[i] >= c0 && st[i] < c0 + CHUNK) own[st[i] - c0] = tag | (uint32_t)(i * kBlock + tid + 1);
        lds_barrier();
        uint32_t v[PER];
        uint32_t tm = 0;
#pragma unroll
        for (int x = 0; x < PER; ++x) {
            const uint32_t y = own[tid * PER + x];
            tm = y > tm ? y : tm;
            v[x] = tm;
        }
        const uint32_t wi = wave_incl_scan_max(tm, lane);
        if (lane == 63) sm.wave_tot[wave] = wi;
        lds_barrier();
        uint32_t before = carry ? (tag | carry) : 0u;
#pragma unroll
        for (int u = 0; u < kWaves; ++u)
            if (u < wave) before = before > sm.wave_tot[u] ? before : sm.wave_tot[u];
        const uint32_t lane_before = __shfl_up(wi, 1, 64);
        if (lane > 0) before = before > lane_before ? before : lane_before;
#pragma unroll
        for (int x = 0; x < PER; ++x) own[tid * PER + x] = v[x] > before ? v[x] : before;
        lds_barrier();
        carry = own[CHUNK - 1] & kOwnerIdxMask;
#pragma unroll
        for (int x = 0; x < PER; ++x) {
            const uint32_t jl = x * kBlock + tid;
            const uint32_t j = c0 + jl;
            if (j < T) {
                const uint32_t k = (own[jl] & kOwnerIdxMask) - 1;
                const uint32_t r = j - sm.start[k];
                const uint32_t b = sm.base[k];
                uint32_t peer;
                if (b == kSelfSentinel) {
                    peer = p.sender[m0 + k];
                } else {
                    const uint32_t idx = (b & ~kGlobal) + r + (r >= sm.skip[k] ? 1u : 0u);
                    peer = (b & kGlobal) ? tv.list[idx] : sm.stage[idx];
                }
                const uint64_t out = (uint64_t)g0 + j;
                if (out < p.capacity) {
                    p.peers[out] = peer;
                    if (p.msgs) p.msgs[out] = m0 + k;
                }
            }
        }
        // no barrier: the next chunk marks the other owner buffer
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
namespace {
struct Cfg {
    int count_ipt;
    int emit_ipt;
    void (*count)(const CountParams&, hipStream_t, unsigned);
    void (*emit)(const EmitParams&, hipStream_t, unsigned);
};

template <int IPT, int U>
void launch_count(const CountParams& p, hipStream_t s, unsigned grid) {
    if (p.in.keys)
        hipLaunchKernelGGL((count_kernel<true, IPT, U>), dim3(grid), dim3(kBlock), 0, s, p);
    else
        hipLaunchKernelGGL((count_kernel<false, IPT, U>), dim3(grid), dim3(kBlock), 0, s, p);
}

template <int IPT, int CHUNK, int STAGE, int U>
void launch_emit(const EmitParams& p, hipStream_t s, unsigned grid) {
    hipLaunchKernelGGL((emit_kernel<IPT, CHUNK, STAGE, U>), dim3(grid), dim3(kBlock), 0, s, p);
}

#define WQ_CFG(cipt, cu, eipt, chunk, stage, eu) \
    {cipt, eipt, &launch_count<cipt, cu>, &launch_emit<eipt, chunk, stage, eu>}
const Cfg kCfgs[] = {
    WQ_CFG(2, 8, 1, 1024, 3072, 8),   // 0: default
    WQ_CFG(2, 8, 2, 1024, 6144, 8),   // 1
    WQ_CFG(1, 8, 1, 1024, 3072, 8),   // 2
    WQ_CFG(4, 8, 1, 1024, 3072, 8),   // 3
    WQ_CFG(2, 4, 1, 512, 3072, 4),    // 4
    WQ_CFG(2, 16, 2, 2048, 6144, 16), // 5
};
#undef WQ_CFG
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);
}  // namespace

int route_config_count() { return kNumCfgs; }

int launch_route(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                 const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                 uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    hipStream_t s = h->stream;
    RouteWs& rw = h->rws;
    const Cfg& cfg = kCfgs[h->route_cfg];
    const uint32_t n_scan = (uint32_t)((M + kScanTile - 1) / kScanTile);
    // workspace: [ticket u64][pad][counters x2 (32 B each) at 64][status u64 x cap at 128]
    if (!rw.buf.p || n_scan > rw.status_cap || rw.epoch >= (1u << 24) - 1) {
        const uint64_t cap = n_scan > rw.status_cap ? (uint64_t)n_scan + n_scan / 2 + 64 : rw.status_cap;
        WQ_ALLOC(h, rw.buf, 128 + cap * 8);
        WQ_HIP(h, hipMemsetAsync(rw.buf.p, 0, 128 + cap * 8, s));
        rw.status_cap = cap;
        rw.epoch = 0;
        rw.calls = 0;
        rw.ticket_base = 0;
    }
    char* base = rw.buf.as<char>();
    wq_route_counters* ring = reinterpret_cast<wq_route_counters*>(base + 64);
    wq_route_counters* cur = ring + (rw.calls & 1);
    wq_route_counters* nxt = ring + ((rw.calls + 1) & 1);
    rw.last = cur;
    if (M == 0) {
        WQ_HIP(h, hipMemsetAsync(d_offsets, 0, 4, s));
        WQ_HIP(h, hipMemsetAsync(cur, 0, sizeof(wq_route_counters), s));
        WQ_HIP(h, hipMemsetAsync(nxt, 0, sizeof(wq_route_counters), s));
        rw.calls++;
        return WQ_OK;
    }
    WQ_ALLOC(h, rw.info, M * sizeof(uint2));

    const TableView tv = table_view(h);
    ProfileEvents& pr = h->prof;
    if (pr.enabled) {
        if (pr.used == pr.start.size()) {
            hipEvent_t a, b;
            WQ_HIP(h, hipEventCreate(&a));
            WQ_HIP(h, hipEventCreate(&b));
            pr.start.push_back(a);
            pr.stop.push_back(b);
        }
        WQ_HIP(h, hipEventRecord(pr.start[pr.used], s));
    }

    CountParams cp;
    cp.in = RouteIn{d_pos, d_keys, d_world, d_sender, d_repl, (uint32_t)M, (int64_t)h->cube_size};
    cp.t = tv;
    cp.offsets = d_offsets;
    cp.info = rw.info.as<uint2>();
    cp.cnt = cur;
    cp.cnt_next = nxt;
    const uint32_t count_tile = kBlock * cfg.count_ipt;
    cfg.count(cp, s, (unsigned)((M + count_tile - 1) / count_tile));
    WQ_HIP(h, hipGetLastError());

    ScanParams sp;
    sp.offsets = d_offsets;
    sp.M = (uint32_t)M;
    sp.n_tiles = n_scan;
    sp.status = reinterpret_cast<uint64_t*>(base + 128);
    sp.ticket = reinterpret_cast<unsigned long long*>(base);
    sp.ticket_base = rw.ticket_base;
    sp.epoch = ++rw.epoch;
    sp.capacity = capacity;
    sp.cnt = cur;
    hipLaunchKernelGGL(scan_kernel, dim3(n_scan), dim3(kBlock), 0, s, sp);
    WQ_HIP(h, hipGetLastError());
    rw.ticket_base += n_scan;

    if (capacity && d_peers) {
        EmitParams ep;
        ep.sender = d_sender;
        ep.M = (uint32_t)M;
        ep.t = tv;
        ep.offsets = d_offsets;
        ep.info = rw.info.as<uint2>();
        ep.peers = d_peers;
        ep.msgs = d_msgs;
        ep.capacity = capacity;
        const uint32_t emit_tile = kBlock * cfg.emit_ipt;
        cfg.emit(ep, s, (unsigned)((M + emit_tile - 1) / emit_tile));
        WQ_HIP(h, hipGetLastError());
    }
    if (pr.enabled) {
        WQ_HIP(h, hipEventRecord(pr.stop[pr.used], s));
        pr.used++;
    }
    rw.calls++;
    return WQ_OK;
}

}  // namespace wq
