// route_count.hpp — pass 1 of the tick: count_kernel (see wq_route.hip).
//
// One lane per message, IPT messages per lane. Per message the pass needs the cube's peer count
// and whether the sender is one of its peers (local_message.rs:60-86). Both come from the first
// 32 bytes of the cube's 128-byte record line (wq_device.hpp): chunk 0 = {pk, count, list_off},
// chunk 1 = {sig, -}, where sig is a 64-bit Bloom signature of the cube's peers. A sender whose
// signature bits are not all set is certainly not subscribed; only the rest (C2: ~7% false
// positives plus the true positives) read the inline peers, two chunks per round. So a lookup is two
// 16-byte loads and 8 VGPRs per message, not eight loads and 32 VGPRs for the whole line.
//
// Work that needs another memory round trip — a linear-probe step past a foreign key, or the
// next two chunks of a list being verified — runs as a per-lane state machine: every round each
// pending message issues its two loads, all IPT messages of the lane together, so a wave pays one
// round trip per round whatever mix of probes and verifications it holds.
#pragma once
#include "route_common.hpp"

namespace wq {

struct CountParams {
    RouteIn in;
    TableView t;
    uint32_t* e;           // out: filtered recipient count e_m
    uint2* info;           // out: locator
    uint32_t* tile_total;  // out: sum of e over each block's messages
    uint32_t* tile_F;      // out: candidates (unfiltered peers) over each block's messages
                           // (per-block words, summed by tile_scan: one shared atomic counter
                           // would serialise ~1k blocks at ~90 adds/us)
    wq_route_counters* cnt;
    wq_route_counters* cnt_next;
    uint32_t* health;  // sticky {error, overflow} words (flag_route)
    uint32_t n_tiles = 0;  // count_kernel: tiles of kBlock * IPT messages (grid stride when > gridDim.x)
    // count_kernel: when set, message (slot) m's e and locator go to index perm[m] (kNone: nowhere)
    const uint32_t* perm = nullptr;
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

// per-message probe state
constexpr uint32_t kStDone = 0, kStProbe = 1, kStVerify = 2;

// Messages m0 + i*kBlock + threadIdx.x, i < IPT: filtered count and locator of each (zero for
// m >= in.M), with F (candidates) and E (recipients) accumulated into the caller's sums.
// FULL: the whole record line is read in the first round (the sender filter then needs no extra
// round) and its peer chunks 2-7 are handed back in peers_out (FULL only; valid for inline records).
// OWN (the sharded tick's ingesting GPU, route_common.hpp RouteIn::own_*): only the messages whose
// cube this shard owns are counted; every other message gets e = 0 here (its row comes back from
// its owner, wq_sharded.hip).
template <bool RAW_KEYS, int IPT, int DBG = 0, bool FULL = false, bool SLOTS = false, bool OWN = false>
__device__ __forceinline__ void count_rows(const RouteIn& in, const TableView& tv, uint32_t m0,
                                           uint32_t (&e_out)[IPT], uint2 (&inf_out)[IPT], uint64_t& F_local,
                                           uint32_t& E_local, uint4 (*peers_out)[6] = nullptr,
                                           uint32_t* owner_out = nullptr) {
    const int tid = threadIdx.x;
    // the probe reads the compact header table (TableView::hdr_mask; not FULL, which reads whole lines)
    const bool chdr = !FULL && tv.hdr && tv.hdr_mask;

    // ---- A: inputs (all loads first), quantise (kernel 1), packed key, home slot ----
    // SLOTS: compact slots of the sharded tick (route_common.hpp) — the key arrives packed (a
    // regular slot), or as full coordinates in a head + tail pair; a tail slot routes to nobody.
    uint32_t in_w[IPT], in_me[IPT], in_kind[IPT];
    uint8_t in_rp[IPT];
    uint64_t in_c[IPT][3];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * kBlock + tid;
        const uint32_t mm = m < in.M ? m : 0;
        if (SLOTS) {
            const uint32_t* r = in.slots + (uint64_t)kSlotWords * mm;
            const uint32_t r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
            in_c[i][0] = ((uint64_t)r1 << 32) | r0;  // packed key, or x of a head
            in_c[i][1] = r2;                         // ext, or the world of a head
            in_c[i][2] = 0;
            in_w[i] = r2;
            in_me[i] = r3;
            in_rp[i] = (uint8_t)(r4 & 0xFFu);
            in_kind[i] = (r4 >> 8) & 0xFFu;
            if (in_kind[i] == kSlotHead && m < in.M) {  // rare: y, z in the tail slot
                in_c[i][1] = ((uint64_t)r[6] << 32) | r[5];
                in_c[i][2] = ((uint64_t)r[8] << 32) | r[7];
            }
        } else {
            in_w[i] = in.world[mm];
            in_me[i] = in.sender[mm];
            in_rp[i] = in.repl[mm];
            in_kind[i] = kSlotReg;
            const uint64_t* src = RAW_KEYS ? reinterpret_cast<const uint64_t*>(in.keys)
                                           : reinterpret_cast<const uint64_t*>(in.pos);
            in_c[i][0] = src[3ull * mm];
            in_c[i][1] = src[3ull * mm + 1];
            in_c[i][2] = src[3ull * mm + 2];
        }
    }
    uint64_t pk[IPT];
    uint32_t ext[IPT], sl[IPT], st[IPT];
    bool via_rec[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * kBlock + tid;
        bool valid = m < in.M && in_kind[i] != kSlotTail;
        const uint32_t w = in_w[i];
        int64_t x = 0, y = 0, z = 0;
        pk[i] = 0;
        ext[i] = 0;
        bool reg;
        if (SLOTS) {
            reg = in_kind[i] == kSlotReg;
            if (reg) {
                pk[i] = in_c[i][0];
                ext[i] = (uint32_t)in_c[i][1];
            } else {
                x = (int64_t)in_c[i][0];
                y = (int64_t)in_c[i][1];
                z = (int64_t)in_c[i][2];
            }
        } else {
            if (RAW_KEYS) {
                x = (int64_t)in_c[i][0];
                y = (int64_t)in_c[i][1];
                z = (int64_t)in_c[i][2];
            } else {
                x = coord_clamp_dev(__longlong_as_double((long long)in_c[i][0]), tv.sf, in.si);
                y = coord_clamp_dev(__longlong_as_double((long long)in_c[i][1]), tv.sf, in.si);
                z = coord_clamp_dev(__longlong_as_double((long long)in_c[i][2]), tv.sf, in.si);
            }
            reg = pack_key(w, x, y, z, tv.sf, &pk[i], &ext[i]);
            if (OWN) {
                const uint32_t ow = shard_of(w, x, y, z, in.own_G);
                valid = valid && ow == in.own_me;
                // OWN callers that also group the other shards' messages (wq_sharded.hip
                // own_count_hist_kernel): the owner, bit 31 = a two-slot (unpacked) key
                if (owner_out) owner_out[i] = ow | (reg ? 0u : 0x80000000u);
            }
        }
        // lanes with nothing to probe read a dummy line spread by message index (never one shared
        // line: a chip-wide hot line serialises on its L2 channel). With compact headers the probe
        // walks the header table; the match then hands over the record slot (below)
        sl[i] = reg ? (uint32_t)(chdr ? hdr_home(pk[i], ext[i], tv.hash_mask, tv.hdr_shift, tv.hdr_blk)
                                      : slot_of(rec_hash(pk[i], ext[i]) & tv.hash_mask, tv.rec_shift))
                    : (m & (uint32_t)(chdr ? tv.hdr_mask : tv.rec_mask));
        via_rec[i] = valid && reg;
        st[i] = via_rec[i] ? kStProbe : kStDone;
        e_out[i] = 0;
        inf_out[i] = make_uint2(0, kNone);
        if (valid && !reg) {  // full-key slot table: rare, finished here
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

    // per-peer boxes (PeerBox) on and still valid: skip long-list searches they rule out
    const bool boxes = !(DBG & 4) && tv.pbox && *tv.pbox_valid;

    // ---- B: rounds of two 16-byte loads per pending message ----
    const uint4* recs4 = reinterpret_cast<const uint4*>(tv.recs);
    // probe rounds read the dense headers when the table has them (not FULL: that reads whole lines)
    const uint4* hdr4 = FULL ? nullptr : tv.hdr;
    uint4 c0[IPT], c1[IPT];
    uint4 pc[IPT][FULL ? 6 : 1];  // FULL: the inline peers (chunks 2-7) ride along in the first round
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint4* hp = hdr4 ? hdr4 + (uint64_t)sl[i] * 2 : recs4 + (uint64_t)sl[i] * 8;
        c0[i] = hp[0];
        c1[i] = (DBG & 1) ? c0[i] : hp[1];
        if (FULL)
#pragma unroll
            for (int q = 0; q < 6; ++q) pc[i][q] = recs4[(uint64_t)sl[i] * 8 + 2 + q];
    }
    uint32_t cnt[IPT], loff[IPT], lt[IPT], vc[IPT];
    bool has[IPT], srch[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        cnt[i] = 0;
        loff[i] = 0;
        lt[i] = 0;
        vc[i] = 0;
        has[i] = false;
        srch[i] = false;
    }
    for (;;) {
        bool pending = false;
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            const uint32_t me = in_me[i];
            if (st[i] == kStProbe) {
                const uint64_t key = ((uint64_t)c0[i].y << 32) | c0[i].x;
                const bool empty = c1[i].w == 0;  // ext == 0: an empty slot, the cube has no peers
                if (empty || (key == pk[i] && c1[i].w == ext[i])) {
                    cnt[i] = empty ? 0u : c0[i].z;
                    loff[i] = c0[i].w;
                    st[i] = kStDone;
                    if (chdr && !empty) sl[i] = c1[i].z;  // from here on: the cube's record slot
                    if (cnt[i] && in_rp[i] != WQ_REPL_INCLUDING_SELF) {
                        const uint64_t sig = ((uint64_t)c1[i].y << 32) | c1[i].x;
                        const uint64_t bits = peer_sig(me);
                        if (!(DBG & 3) && (sig & bits) == bits) {  // maybe subscribed: verify
                            if (FULL && cnt[i] <= (uint32_t)kInline) {  // peers already in registers
                                uint32_t l = 0;
                                bool h = false;
#pragma unroll
                                for (int q = 0; q < kInline; ++q) {
                                    const uint4 c = pc[i][q / 4];
                                    const uint32_t w = (q & 3) == 0 ? c.x : (q & 3) == 1 ? c.y : (q & 3) == 2 ? c.z : c.w;
                                    const bool in = (uint32_t)q < cnt[i];
                                    l += (in & (w < me)) ? 1u : 0u;
                                    h |= in & (w == me);
                                }
                                lt[i] = l;
                                has[i] = h;
                            } else if (cnt[i] <= (uint32_t)kInline) {  // inline peers from chunk 2 on
                                st[i] = kStVerify;
                                vc[i] = 2;
                            } else {
                                srch[i] = true;  // > kInline peers: after the probe loop
                            }
                        }
                    }
                } else {
                    sl[i] = (sl[i] + 1) & (uint32_t)(chdr ? tv.hdr_mask : tv.rec_mask);
                }
            } else if (st[i] == kStVerify) {
                // chunks vc, vc+1 hold peers 4*vc-8 .. 4*vc-1; the list is ascending, so the first
                // peer >= me ends the search
                const uint32_t v[8] = {c0[i].x, c0[i].y, c0[i].z, c0[i].w, c1[i].x, c1[i].y, c1[i].z, c1[i].w};
                const uint32_t b = 4 * vc[i] - kInlineWord0;
                bool stop = false;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const bool in = b + q < cnt[i];
                    lt[i] += (in & (v[q] < me)) ? 1u : 0u;
                    has[i] |= in & (v[q] == me);
                    stop |= in & (v[q] >= me);
                }
                vc[i] += 2;
                if (stop || 4 * vc[i] - kInlineWord0 >= cnt[i]) st[i] = kStDone;
            }
            pending |= st[i] != kStDone;
        }
        if (!__any(pending)) break;
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            if (st[i] == kStDone) continue;
            const uint32_t q = st[i] == kStProbe ? 0u : vc[i];  // vc <= 6: chunks q, q+1 <= 7
            const uint4* hp = (hdr4 && q == 0) ? hdr4 + (uint64_t)sl[i] * 2 : recs4 + (uint64_t)sl[i] * 8 + q;
            c0[i] = hp[0];
            c1[i] = hp[1];
            if (FULL && st[i] == kStProbe)
#pragma unroll
                for (int c = 0; c < 6; ++c) pc[i][c] = recs4[(uint64_t)sl[i] * 8 + 2 + c];
        }
    }
    // long lists (> kInline peers) whose signature admits the sender: unless the sender's box
    // rules the cube out, a binary search — outside the probe loop, whose record lines are dead
    // by now (fewer live registers there)
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        if (srch[i] && (!boxes || box_may_hold(tv, in_me[i], pk[i], ext[i]))) {
            const uint32_t* lp = tv.list + loff[i] + 1;
            lt[i] = lower_bound_dev(lp, cnt[i], in_me[i]);
            has[i] = lt[i] < cnt[i] && lp[lt[i]] == in_me[i];
        }
    }

#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        if (via_rec[i]) {
            finish_message(cnt[i], in_rp[i], cnt[i] <= (uint32_t)kInline, sl[i], loff[i], lt[i], has[i], &e_out[i],
                           &inf_out[i]);
            F_local += cnt[i];
            E_local += e_out[i];
        }
        if (FULL && peers_out)
#pragma unroll
            for (int c = 0; c < 6; ++c) peers_out[i][c] = pc[i][c];
    }
}

template <bool RAW_KEYS, int IPT, int MINW, int DBG = 0, bool FULL = false, bool SLOTS = false, bool OWN = false>
__global__ __launch_bounds__(kBlock, MINW) void count_kernel(CountParams p) {
    if (p.in.m_dev) {
        const uint32_t mv = *p.in.m_dev;
        if (mv < p.in.M) p.in.M = mv;
    }
    __shared__ uint64_t wave_F[kWaves];
    __shared__ uint64_t wave_E[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (blockIdx.x == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    const uint32_t nt = p.n_tiles ? p.n_tiles : gridDim.x;
    for (uint32_t blk = blockIdx.x; blk < nt; blk += gridDim.x) {
        const uint32_t m0 = blk * (kBlock * IPT);
        if (m0 >= p.in.M && blk > 0) break;  // past a device-side count (m_dev): nothing left here
        uint64_t F_local = 0;
        uint32_t E_local = 0;
        uint32_t e_out[IPT];
        uint2 inf_out[IPT];
        count_rows<RAW_KEYS, IPT, DBG, FULL, SLOTS, OWN>(p.in, p.t, m0, e_out, inf_out, F_local, E_local);
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            const uint32_t m = m0 + i * kBlock + tid;
            if (m < p.in.M) {
                const uint32_t dst = p.perm ? p.perm[m] : m;
                if (dst != kNone) {
                    p.e[dst] = e_out[i];
                    p.info[dst] = inf_out[i];
                }
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
            p.tile_F[blk] = Fb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Fb;
            p.tile_total[blk] = Eb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Eb;
            if (Eb > 0xFFFFFFFFull) flag_route(p.cnt, p.health, 2u, 0u);
        }
        lds_barrier();  // the next tile rewrites wave_F / wave_E
    }
}

// One wave per block, one 64-message tile per wave (route config 13, an experiment of round 6): no
// block barrier, so a wave whose lanes finish early leaves its slot to the next tile at once instead
// of waiting for the block's slowest wave. The tile totals are per 64 messages (count_tile = 64;
// the emit's tile prefix addressing takes any count_tile dividing its 256-message blocks).
template <bool RAW_KEYS, int MINB>
__global__ __launch_bounds__(64, MINB) void count_wave_kernel(CountParams p) {
    const int lane = threadIdx.x;
    if (blockIdx.x == 0 && lane == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    const uint32_t nt = p.n_tiles ? p.n_tiles : gridDim.x;
    for (uint32_t blk = blockIdx.x; blk < nt; blk += gridDim.x) {
        const uint32_t m0 = blk * 64u;
        uint64_t F_local = 0;
        uint32_t E_local = 0;
        uint32_t e_out[1];
        uint2 inf_out[1];
        count_rows<RAW_KEYS, 1>(p.in, p.t, m0, e_out, inf_out, F_local, E_local);
        const uint32_t m = m0 + lane;
        if (m < p.in.M) {
            p.e[m] = e_out[0];
            p.info[m] = inf_out[0];
        }
        const uint64_t Fw = wave_sum_u64(F_local);
        const uint64_t Ew = wave_sum_u64(E_local);
        if (lane == 0) {
            p.tile_F[blk] = Fw > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Fw;
            p.tile_total[blk] = Ew > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Ew;
            if (Ew > 0xFFFFFFFFull) flag_route(p.cnt, p.health, 2u, 0u);
        }
    }
}

}  // namespace wq
