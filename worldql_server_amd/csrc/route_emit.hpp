// route_emit.hpp — pass 3 of the tick: emit_kernel (see wq_route.hip).
#pragma once
#include <type_traits>

#include "route_common.hpp"

namespace wq {

// ------------------------------------------------------------------------------------------
// 3. emit
// ------------------------------------------------------------------------------------------
struct EmitParams {
    const uint32_t* sender;
    uint32_t M;
    TableView t;
    const uint32_t* e;            // filtered counts (count pass)
    const uint32_t* tile_prefix;  // exclusive prefix of the count pass's block totals
    uint32_t count_tile;          // messages per count block (a multiple of the emit tile)
    uint32_t* offsets;            // out: CSR offsets[0 .. M)
    const uint2* info;
    uint32_t* peers;              // nullptr: offsets only (no capacity)
    uint32_t* msgs;
    uint64_t capacity;
};

template <int IPT, int STAGE>
struct EmitSmem {
    using Om = typename std::conditional<IPT == 1, uint8_t, uint16_t>::type;
    uint32_t op[STAGE];             // window of the tile's output: peers, in output order
    Om om[STAGE];                   // ... and the tile-local index of each output's message
    uint32_t start[kBlock * IPT];   // tile-local first output of the message
    uint32_t slot[kBlock * IPT];    // inline record slot, or kNone
    uint32_t meta[kBlock * IPT];    // inline: count | skipped index << 8 (0xFF: none)
    uint32_t gq_j[kBlock * IPT];    // messages whose list is read from `list` (> kInline peers)
    uint32_t gq_off[kBlock * IPT];  // ... its list offset (first peer)
    uint32_t gq_skip[kBlock * IPT]; // ... skipped list index or kNone
    uint32_t gq_e[kBlock * IPT];    // ... outputs
    uint32_t n_gq;
    uint32_t wave_tot[kWaves];
    uint32_t rowt[IPT + 1][kWaves]; // per-row wave totals of e (+ earlier messages of the count block)
};

// Pass 3. The tile's outputs [0, T) are produced in windows of STAGE positions: every message's
// peers are written straight into an LDS image of the window IN OUTPUT ORDER (the sender's own
// entry skipped while staging), together with the message's tile-local index, and the window is
// then copied out with coalesced stores. C2 tiles (256 messages, ~2,560 outputs) take one window.
//   inline records (<= kInline peers): eight lanes per record line, lane `part` reading chunk
//     `part` (peers 4*part-6 .. 4*part-3) only if it holds one of the message's peers;
//   longer lists: the block copies the list slice that falls in the window from `list`;
//   OnlySelf: the sender itself, written by the message's own lane.
template <int IPT, int STAGE, int U, int DBG = 0>
__global__ __launch_bounds__(kBlock) void emit_kernel(EmitParams p) {
    constexpr int TILE = kBlock * IPT;
    static_assert(IPT == 1 || IPT == 2, "tile-local message index must fit EmitSmem::Om");
    __shared__ EmitSmem<IPT, STAGE> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TableView& tv = p.t;
    const uint32_t m0 = blockIdx.x * TILE;

    // ---- A0: CSR offsets of the tile — count-block prefix + block-local scan in message order ----
    uint32_t e[IPT], st[IPT];
    uint2 inf[IPT];
    uint32_t g0 = 0, T = 0;  // global offset of the tile's first output; outputs in the tile
    if (tid == 0) sm.n_gq = 0;
    {
        uint32_t incl[IPT];
        // the locators are loaded with the counts, ahead of the offset stores (gfx9: a later
        // load-wait would otherwise also wait for those stores)
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            const uint32_t m = m0 + i * kBlock + tid;
            e[i] = m < p.M ? p.e[m] : 0u;
            inf[i] = (p.peers && m < p.M) ? p.info[m] : make_uint2(0, kNone);
        }
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            incl[i] = wave_incl_scan_add(e[i], lane);
            if (lane == 63) sm.rowt[i][wave] = incl[i];
        }
        const uint32_t ct0 = (m0 / p.count_tile) * p.count_tile;
        uint32_t part = 0;
        for (uint32_t m = ct0 + tid; m < m0; m += kBlock) part += p.e[m];
        part = (uint32_t)wave_sum_u64(part);
        if (lane == 0) sm.rowt[IPT][wave] = part;
        lds_barrier();
        uint32_t g = p.tile_prefix[m0 / p.count_tile], rows = 0;
#pragma unroll
        for (int u = 0; u < kWaves; ++u) g += sm.rowt[IPT][u];
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            uint32_t before = 0, tot = 0;
#pragma unroll
            for (int u = 0; u < kWaves; ++u) {
                const uint32_t t = sm.rowt[i][u];
                if (u < wave) before += t;
                tot += t;
            }
            st[i] = rows + before + incl[i] - e[i];
            rows += tot;
            const uint32_t m = m0 + i * kBlock + tid;
            if (m < p.M && !(DBG & 4)) p.offsets[m] = g + st[i];
        }
        g0 = g;
        T = rows;
    }
    if (!p.peers) return;  // counts-only call: offsets are all that is asked for

    // ---- A: per message — what to stage, and from where ----
    bool self[IPT];
    uint32_t self_peer[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t j = i * kBlock + tid;
        uint32_t slot = kNone, meta = 0;
        self[i] = e[i] && (inf[i].x & kLocSelf);
        self_peer[i] = self[i] ? p.sender[m0 + j] : 0u;
        if (e[i] && !(inf[i].x & kLocSelf)) {
            if (inf[i].x & kLocGlobal) {
                const uint32_t q = atomicAdd(&sm.n_gq, 1u);
                sm.gq_j[q] = j;
                sm.gq_off[q] = (inf[i].x & ~kLocGlobal) + 1;
                sm.gq_skip[q] = inf[i].y;
                sm.gq_e[q] = e[i];
            } else {
                const uint32_t s24 = inf[i].y & kSkipNone24;
                slot = inf[i].x;
                meta = (inf[i].y >> 24) | ((s24 == kSkipNone24 ? 0xFFu : s24) << 8);
            }
        }
        sm.start[j] = st[i];
        sm.slot[j] = slot;
        sm.meta[j] = meta;
    }
    lds_barrier();
    const uint32_t n_gq = sm.n_gq;

    const int grp = lane >> 3, part = lane & 7;
    const uint4* recs4 = reinterpret_cast<const uint4*>(tv.recs);
    const uint32_t first = part <= 1 ? 0u : 4u * part - 6u;  // first peer index in chunk `part`
    for (uint32_t w0 = 0; w0 < T; w0 += STAGE) {
        const uint32_t w1 = T - w0 < (uint32_t)STAGE ? T : w0 + STAGE;
        // OnlySelf: the message's own lane
#pragma unroll
        for (int i = 0; i < IPT; ++i)
            if (self[i] && st[i] >= w0 && st[i] < w1) {
                sm.op[st[i] - w0] = self_peer[i];
                sm.om[st[i] - w0] = (typename EmitSmem<IPT, STAGE>::Om)(i * kBlock + tid);
            }
        // inline records: eight lanes per line, U lines per lane in flight
        for (int r0 = 0; r0 < 8 * IPT; r0 += U) {
            uint4 v[U];
            uint32_t jj[U], sp[U], mt[U];
            bool act[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                jj[u] = wave_msg<IPT>(wave, 8 * (r0 + u) + grp);
                const uint32_t sl = sm.slot[jj[u]];
                sp[u] = sm.start[jj[u]];
                mt[u] = sm.meta[jj[u]];
                const uint32_t cnt = mt[u] & 0xFF, skip = mt[u] >> 8;
                const uint32_t ej = cnt - (skip != 0xFFu ? 1u : 0u);
                act[u] = sl != kNone && part >= 1 && first < cnt && sp[u] < w1 && sp[u] + ej > w0;
                if (act[u]) v[u] = (DBG & 1) ? make_uint4(sl, part, 0, 0) : recs4[(uint64_t)sl * 8 + part];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!act[u]) continue;
                const uint32_t cnt = mt[u] & 0xFF, skip = mt[u] >> 8;
                const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                    const int idx = 4 * part + e4 - kInlineWord0;
                    if (idx < 0 || (uint32_t)idx >= cnt || (uint32_t)idx == skip) continue;
                    const uint32_t pos = sp[u] + (uint32_t)idx - ((uint32_t)idx > skip && skip != 0xFFu ? 1u : 0u);
                    if (pos >= w0 && pos < w1) {
                        sm.op[pos - w0] = vv[e4];
                        sm.om[pos - w0] = (typename EmitSmem<IPT, STAGE>::Om)jj[u];
                    }
                }
            }
        }
        // long lists: the block copies each one's slice of the window from `list`
        for (uint32_t q = 0; q < n_gq; ++q) {
            const uint32_t j = sm.gq_j[q], s0 = sm.start[j], ej = sm.gq_e[q];
            const uint32_t lo = s0 > w0 ? s0 : w0, hi = s0 + ej < w1 ? s0 + ej : w1;
            const uint32_t off = sm.gq_off[q], skip = sm.gq_skip[q];
            for (uint32_t k = lo + tid; k < hi; k += kBlock) {
                const uint32_t o = k - s0;
                sm.op[k - w0] = tv.list[off + o + (o >= skip ? 1u : 0u)];
                sm.om[k - w0] = (typename EmitSmem<IPT, STAGE>::Om)j;
            }
        }
        lds_barrier();
        // copy-out: one coalesced stream per array
        const uint32_t n = w1 - w0;
        for (uint32_t k = tid; k < n; k += kBlock) {
            const uint64_t out = (uint64_t)g0 + w0 + k;
            if (out < p.capacity && !(DBG & 2)) {
                p.peers[out] = sm.op[k];
                if (p.msgs) p.msgs[out] = m0 + sm.om[k];
            }
        }
        if (w1 < T) lds_barrier();  // the next window reuses the image
    }
}

}  // namespace wq
