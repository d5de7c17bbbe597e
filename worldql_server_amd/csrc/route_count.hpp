// route_count.hpp — pass 1 of the tick: count_kernel (see wq_route.hip).
#pragma once
#include "route_common.hpp"

namespace wq {

// ------------------------------------------------------------------------------------------
// 1. count
// ------------------------------------------------------------------------------------------
struct CountParams {
    RouteIn in;
    TableView t;
    uint32_t* e;           // out: filtered recipient count e_m
    uint2* info;           // out: locator
    uint32_t* tile_total;  // out: sum of e over each block's messages
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
    uint64_t wave_E[kWaves];
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
    uint32_t E_local = 0;

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
            p.e[m] = e;
            p.info[m] = inf;
            F_local += cnt;
            E_local += e;
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
                p.e[m] = e;
                p.info[m] = inf;
                F_local += cnt;
                E_local += e;
            }
        }
    }

    const uint64_t Fw = wave_sum_u64(F_local);
    const uint64_t Ew = wave_sum_u64(E_local);
    if (lane == 0) {
        sm.wave_F[wave] = Fw;
        sm.wave_E[wave] = Ew;
    }
    lds_barrier();
    if (tid == 0) {
        uint64_t Fb = 0, Eb = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            Fb += sm.wave_F[w];
            Eb += sm.wave_E[w];
        }
        if (Fb) atomicAdd(reinterpret_cast<unsigned long long*>(&p.cnt->n_candidates), (unsigned long long)Fb);
        p.tile_total[blockIdx.x] = Eb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Eb;
    }
}

}  // namespace wq
