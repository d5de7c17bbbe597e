// route_radius.hpp — C5: the tick with the exact radius filter.
//
// An extension the reference does not have: after the cube broadphase (local_message.rs:52-86 as
// everywhere else) a pair survives only if the peer's position lies within the radius of the
// message position (within_radius, wq_device.hpp). The count pass therefore needs every candidate's
// id AND position: one lane per message reads the whole record line (chunks 0-7) in one round,
// gathers the positions of the <= 24 inline peers four at a time, and keeps the survivors as a
// 24-bit mask in the locator (info.y = count << 24 | mask), which emit_row<..., RADIUS> expands
// without touching a position again. Longer lists (and full-key slot-table cubes) are walked from
// `list` by the lane, and emit_row re-evaluates them chunk by chunk with a block-wide compaction.
// Replication (local_message.rs:60-86) is folded into the mask: ExceptSelf drops the sender,
// OnlySelf keeps only the sender, IncludingSelf keeps everyone in range.
#pragma once
#include "route_count.hpp"
#include "route_emit.hpp"

namespace wq {

// Survivors of a list in `list` (first peer at lp[0], cnt peers) for one message.
__device__ __forceinline__ uint32_t count_list_radius(const TableView& tv, const uint32_t* lp, uint32_t cnt,
                                                      double mx, double my, double mz, uint8_t rp, uint32_t me) {
    uint32_t e = 0;
    for (uint32_t i = 0; i < cnt; ++i) {
        const uint32_t q = lp[i];
        e += (repl_keeps(rp, q, me) && within_radius(tv, mx, my, mz, q)) ? 1u : 0u;
    }
    return e;
}

// Lane per message; one block = one 256-message tile (tile_total per block, count_tile = 256).
// OWN (the sharded tick's ingesting GPU): only the messages whose cube this shard owns are counted;
// the others get e = 0 and an empty locator here (their rows come back from their owners).
template <bool OWN = false>
__global__ __launch_bounds__(kBlock) void count_radius_kernel(CountParams p) {
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
    const uint32_t m = blockIdx.x * kBlock + tid;
    bool valid = m < p.in.M;
    const uint32_t mm = valid ? m : 0;
    const double mx = p.in.pos[3ull * mm], my = p.in.pos[3ull * mm + 1], mz = p.in.pos[3ull * mm + 2];
    const uint32_t w = p.in.world[mm], me = p.in.sender[mm];
    const uint8_t rp = p.in.repl[mm];
    const int64_t kx = coord_clamp_dev(mx, tv.sf, p.in.si);
    const int64_t ky = coord_clamp_dev(my, tv.sf, p.in.si);
    const int64_t kz = coord_clamp_dev(mz, tv.sf, p.in.si);
    uint64_t pk = 0;
    uint32_t ext = 0;
    const bool reg = pack_key(w, kx, ky, kz, tv.sf, &pk, &ext);
    if (OWN) valid = valid && shard_of(w, kx, ky, kz, p.in.own_G) == p.in.own_me;
    uint32_t e = 0, cnt = 0;
    uint2 info = make_uint2(0, kNone);
    if (valid && !reg) {  // full-key slot table: the list is walked from `list`
        const uint32_t loff = probe(tv.slots, tv.slot_mask, tv.slot_shift, cube_hash(w, kx, ky, kz) & tv.hash_mask, w,
                                    kx, ky, kz);
        if (loff != kNone) {
            cnt = tv.list[loff];
            e = count_list_radius(tv, tv.list + loff + 1, cnt, mx, my, mz, rp, me);
            info = make_uint2(kLocGlobal | loff, cnt);
        }
    }
    // the whole record line: header, signature, 24 inline peers
    const uint4* recs4 = reinterpret_cast<const uint4*>(tv.recs);
    uint32_t sl = reg ? (uint32_t)slot_of(rec_hash(pk, ext) & tv.hash_mask, tv.rec_shift) : (m & (uint32_t)tv.rec_mask);
    uint4 c0, c1, pc[6];
    c0 = recs4[(uint64_t)sl * 8];
    c1 = recs4[(uint64_t)sl * 8 + 1];
#pragma unroll
    for (int k = 0; k < 6; ++k) pc[k] = recs4[(uint64_t)sl * 8 + 2 + k];
    bool pend = valid && reg;
    for (;;) {
        const uint64_t key = ((uint64_t)c0.y << 32) | c0.x;
        const bool coll = pend && c1.w != 0 && (key != pk || c1.w != ext);  // another cube's record
        if (!__any(coll)) break;
        if (coll) {
            sl = (sl + 1) & (uint32_t)tv.rec_mask;
            c0 = recs4[(uint64_t)sl * 8];
            c1 = recs4[(uint64_t)sl * 8 + 1];
#pragma unroll
            for (int k = 0; k < 6; ++k) pc[k] = recs4[(uint64_t)sl * 8 + 2 + k];
        }
    }
    if (pend) {
        cnt = c1.w ? c0.z : 0u;  // ext == 0: empty, no peers
        const uint32_t loff = c0.w;
        if (cnt > (uint32_t)kInline) {
            e = count_list_radius(tv, tv.list + loff + 1, cnt, mx, my, mz, rp, me);
            info = make_uint2(kLocGlobal | loff, cnt);
        } else if (cnt) {
            uint32_t mask = 0;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                if (4u * k >= cnt) break;
                const uint32_t v[4] = {pc[k].x, pc[k].y, pc[k].z, pc[k].w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t idx = 4u * k + i;
                    const bool ok = idx < cnt && repl_keeps(rp, v[i], me) && within_radius(tv, mx, my, mz, v[i]);
                    mask |= ok ? (1u << idx) : 0u;
                }
            }
            e = (uint32_t)__popc(mask);
            info = make_uint2(sl, (cnt << 24) | mask);
        }
    }
    if (m < p.in.M) {
        p.e[m] = e;
        p.info[m] = info;
    }
    const uint64_t Fw = wave_sum_u64(valid ? cnt : 0u);
    const uint64_t Ew = wave_sum_u64(e);
    if (lane == 0) {
        wave_F[wave] = Fw;
        wave_E[wave] = Ew;
    }
    lds_barrier();
    if (tid == 0) {
        uint64_t Fb = 0, Eb = 0;
#pragma unroll
        for (int u = 0; u < kWaves; ++u) {
            Fb += wave_F[u];
            Eb += wave_E[u];
        }
        p.tile_F[blockIdx.x] = Fb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Fb;
        p.tile_total[blockIdx.x] = Eb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Eb;
    }
}

}  // namespace wq
