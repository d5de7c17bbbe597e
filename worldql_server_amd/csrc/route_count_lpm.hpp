// route_count_lpm.hpp — pass 1 of the tick, lane-per-message form (see wq_route.hip).
//
// Same contract as count_kernel (route_count.hpp): e_m, the 8-byte locator, the block total and
// F. Each lane owns its messages end to end: it loads its record's whole 128-byte line as eight
// 16-byte loads issued back to back (one line request; the other seven hit it in flight), and
// compares the sender with the <= 28 inline peers in registers. No LDS, no shuffles: the 8-lane
// form spends ~8x the VALU instructions per message on broadcasts and reductions (PMC:
// VALU ~60% busy, profiles/r01_pmc_v6_cfg4.txt).
#pragma once
#include "route_count.hpp"

namespace wq {

template <bool RAW_KEYS, int IPT, int MINW = 1>
__global__ __launch_bounds__(kBlock, MINW) void count_lpm_kernel(CountParams p) {
    __shared__ uint64_t wave_F[kWaves];
    __shared__ uint64_t wave_E[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TableView& tv = p.t;
    if (blockIdx.x == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    const uint32_t m0 = blockIdx.x * (kBlock * IPT);
    uint64_t F_local = 0;
    uint32_t E_local = 0;

    // ---- A: inputs (all loads first), quantise, packed key, home slot ----
    uint32_t in_w[IPT], in_me[IPT];
    uint8_t in_rp[IPT];
    uint64_t in_c[IPT][3];
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
    uint64_t pk[IPT];
    uint32_t sl[IPT], e_out[IPT];
    uint2 inf_out[IPT];
    bool act[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * kBlock + tid;
        const bool valid = m < p.in.M;
        const uint32_t w = in_w[i];
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
        pk[i] = 0;
        const bool reg = pack_key(w, x, y, z, tv.sf, &pk[i]);
        sl[i] = reg ? (uint32_t)slot_of(rec_hash(pk[i]) & tv.hash_mask, tv.rec_shift) : 0u;
        act[i] = valid && reg;
        e_out[i] = 0;
        inf_out[i] = make_uint2(0, kNone);
        if (valid && !reg) {  // full-key slot table: rare
            const uint32_t me = in_me[i];
            const uint8_t rp = in_rp[i];
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
            finish_message(cnt, rp, false, 0, loff, at, has, &e_out[i], &inf_out[i]);
            F_local += cnt;
            E_local += e_out[i];
        }
    }

    // ---- B: the whole record line per lane; collided lanes re-probe together ----
    // Loads are unconditional (no exec-mask branch around them, so the waitcnt pass cannot put a
    // full drain between two messages' lines). Lanes with nothing to probe read a dummy line
    // chosen by message index — never one shared line: a chip-wide hot line serialises on its
    // L2 channel (measured 5x slower). Re-probes re-read the lane's own, L2-hot line.
    const uint4* recs4 = reinterpret_cast<const uint4*>(tv.recs);
    uint4 line[IPT][8];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        if (!act[i]) sl[i] = (m0 + i * kBlock + tid) & (uint32_t)tv.rec_mask;
        const uint64_t base = (uint64_t)sl[i] * 8;
#pragma unroll
        for (int q = 0; q < 8; ++q) line[i][q] = recs4[base + q];
    }
    bool pend[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) pend[i] = act[i];
    for (;;) {
        bool again = false;
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            const uint64_t key = ((uint64_t)line[i][0].y << 32) | line[i][0].x;
            const bool coll = pend[i] && key != 0 && key != pk[i];
            sl[i] = coll ? ((sl[i] + 1) & (uint32_t)tv.rec_mask) : sl[i];
            pend[i] = coll;
            again |= coll;
        }
        if (!__any(again)) break;
        // re-probe only the collided lanes (rare per lane, so the masked branch costs little)
#pragma unroll
        for (int i = 0; i < IPT; ++i)
            if (pend[i])
#pragma unroll
                for (int q = 0; q < 8; ++q) line[i][q] = recs4[(uint64_t)sl[i] * 8 + q];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        if (!act[i]) continue;
        const uint32_t me = in_me[i];
        const uint8_t rp = in_rp[i];
        const uint64_t key = ((uint64_t)line[i][0].y << 32) | line[i][0].x;
        const uint32_t cnt = key != 0 ? line[i][0].z : 0u;
        const uint32_t loff = line[i][0].w;
        const bool inl = cnt <= (uint32_t)kInline;
        uint32_t lt = 0;
        bool has = false;
        if (cnt && rp != WQ_REPL_INCLUDING_SELF) {
            if (inl) {
#pragma unroll
                for (int q = 1; q < 8; ++q) {
                    const uint32_t vv[4] = {line[i][q].x, line[i][q].y, line[i][q].z, line[i][q].w};
#pragma unroll
                    for (int e4 = 0; e4 < 4; ++e4) {
                        const uint32_t idx = 4 * (q - 1) + e4;
                        const bool in = idx < cnt;
                        lt += (in & (vv[e4] < me)) ? 1u : 0u;
                        has |= in & (vv[e4] == me);
                    }
                }
            } else {  // > 28 peers: binary search of the full list
                const uint32_t* lp = tv.list + loff + 1;
                lt = lower_bound_dev(lp, cnt, me);
                has = lt < cnt && lp[lt] == me;
            }
        }
        finish_message(cnt, rp, inl, sl[i], loff, lt, has, &e_out[i], &inf_out[i]);
        F_local += cnt;
        E_local += e_out[i];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * kBlock + tid;
        if (m < p.in.M) {
            p.e[m] = e_out[i];
            p.info[m] = inf_out[i];
        }
    }

    const uint64_t Fw = wave_sum_u64(F_local);
    const uint64_t Ew = wave_sum_u64(E_local);
    if (lane == 0) {
        wave_F[wave] = Fw;
        wave_E[wave] = Ew;
    }
    lds_barrier();
    if (tid == 0) {
        uint64_t Fb = 0, Eb = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            Fb += wave_F[w];
            Eb += wave_E[w];
        }
        if (Fb) atomicAdd(reinterpret_cast<unsigned long long*>(&p.cnt->n_candidates), (unsigned long long)Fb);
        p.tile_total[blockIdx.x] = Eb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Eb;
    }
}

}  // namespace wq
