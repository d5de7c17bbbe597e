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
    uint32_t e[kBlock * IPT];   // results, written to HBM in one coalesced pass at the end: on
    uint2 info[kBlock * IPT];   // gfx9 stores count in vmcnt, so a store inside the probe loop
                                // would make every later load-wait also wait for it
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
    // Every input of the IPT messages is loaded before any of them is used, so a wave waits for
    // memory once here instead of once per coordinate.
    uint32_t in_w[IPT], in_me[IPT];
    uint8_t in_rp[IPT];
    uint64_t in_c[IPT][3];  // f64 bits, or raw keys
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * kBlock + tid;
        const uint32_t mm = m < p.in.M ? m : 0;
        in_w[i] = p.in.world[mm];
        in_me[i] = p.in.sender[mm];
        in_rp[i] = p.in.repl[mm];
        const uint64_t* src = RAW_KEYS ? reinterpret_cast<const uint64_t*>(p.in.keys)
                                       : reinterpret_cast<const uint64_t*>(p.in.pos);
        in_c[i][0] = src[3ull * mm];
        in_c[i][1] = src[3ull * mm + 1];
        in_c[i][2] = src[3ull * mm + 2];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t j = i * kBlock + tid;
        const uint32_t m = m0 + j;
        const bool valid = m < p.in.M;
        const uint32_t w = in_w[i];
        const uint32_t me = in_me[i];
        const uint8_t rp = in_rp[i];
        int64_t x, y, z;
        if (RAW_KEYS) {
            x = (int64_t)in_c[i][0];
            y = (int64_t)in_c[i][1];
            z = (int64_t)in_c[i][2];
        } else {
            x = coord_clamp_dev(__longlong_as_double((long long)in_c[i][0]), tv.sf, p.in.si);
            y = coord_clamp_dev(__longlong_as_double((long long)in_c[i][1]), tv.sf, p.in.si);
            z = coord_clamp_dev(__longlong_as_double((long long)in_c[i][2]), tv.sf, p.in.si);
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
            sm.e[j] = e;
            sm.info[j] = inf;
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
    const int lead = lane & ~7;
    for (int r0 = 0; r0 < 8 * IPT; r0 += U) {
        uint4 v[U];
        uint32_t jj[U], sl[U], meta[U];
        uint64_t pkv[U];
        bool pend[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            jj[u] = wave_msg<IPT>(wave, 8 * (r0 + u) + grp);
            meta[u] = sm.meta[jj[u]];
            sl[u] = sm.slot[jj[u]];
            pkv[u] = sm.pk[jj[u]];
            pend[u] = (meta[u] & (kMetaValid | kMetaDone)) == kMetaValid;  // uniform per group
            if (!pend[u]) sl[u] = (m0 + jj[u]) & (uint32_t)tv.rec_mask;  // spread dummy line
            v[u] = recs4[(uint64_t)sl[u] * 8 + part];  // unconditional: see route_count_lpm.hpp
        }
        // Linear-probe collisions: check every line's key, then re-issue the loads of all groups
        // that hit another cube together, so a round costs one extra round trip per probe
        // DEPTH rather than one per collided message.
        for (;;) {
            bool again = false;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!pend[u]) continue;
                const uint32_t hx = __shfl(v[u].x, lead, 64), hy = __shfl(v[u].y, lead, 64);
                const uint64_t key = ((uint64_t)hy << 32) | hx;
                if (key != 0 && key != pkv[u]) {
                    sl[u] = (sl[u] + 1) & (uint32_t)tv.rec_mask;
                    again = true;
                } else {
                    pend[u] = false;
                }
            }
            if (!__any(again)) break;
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (pend[u]) v[u] = recs4[(uint64_t)sl[u] * 8 + part];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if ((meta[u] & (kMetaValid | kMetaDone)) != kMetaValid) continue;  // uniform per group
            const uint32_t me = sm.me[jj[u]];
            const uint8_t rp = (uint8_t)(meta[u] >> 8);
            const uint32_t hx = __shfl(v[u].x, lead, 64), hy = __shfl(v[u].y, lead, 64);
            const uint32_t hz = __shfl(v[u].z, lead, 64), hw = __shfl(v[u].w, lead, 64);
            const uint64_t key = ((uint64_t)hy << 32) | hx;
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
                sm.e[jj[u]] = e;
                sm.info[jj[u]] = inf;
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
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t j = i * kBlock + tid;
        if (m0 + j < p.in.M) {
            p.e[m0 + j] = sm.e[j];
            p.info[m0 + j] = sm.info[j];
        }
    }
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
