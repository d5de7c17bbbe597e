// route_emit.hpp — pass 3 of the tick: emit_kernel (see wq_route.hip).
#pragma once
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
    uint32_t rowt[IPT + 1][kWaves]; // per-row wave totals of e (+ earlier messages of the count block)
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

    // ---- A0: CSR offsets of the tile — count-block prefix + block-local scan in message order ----
    uint32_t e[IPT], st[IPT], sc[IPT];
    uint2 inf[IPT];
    uint32_t g0 = 0, T = 0;  // global offset of the tile's first output; outputs in the tile
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
            if (m < p.M) p.offsets[m] = g + st[i];
        }
        g0 = g;
        T = rows;
    }
    if (!p.peers) return;  // counts-only call: offsets are all that is asked for

    // ---- A: one lane per message — locators, stage positions ----
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
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
                // unconditional load, no drain between rounds; groups with no record read a dummy
                // line spread by message index (a shared line would serialise on one L2 channel)
                const uint64_t line = sl != kNone ? sl : ((m0 + j) & (uint32_t)tv.rec_mask);
                v[u] = recs4[line * 8 + part];
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

}  // namespace wq
