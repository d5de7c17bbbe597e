// route_emit.hpp — pass 3 of the tick: emit_kernel (see wq_route.hip).
#pragma once
#include "route_common.hpp"

namespace wq {

// ------------------------------------------------------------------------------------------
// 3. emit
// ------------------------------------------------------------------------------------------
struct EmitParams {
    const uint32_t* sender;
    const double* pos;    // radius mode only
    const uint8_t* repl;  // radius mode only
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
    uint32_t n_blocks = 0;  // emit_map_kernel: 256-message blocks (grid stride when > gridDim.x)
    uint32_t msg_base = 0;  // emit_map_kernel: msgs[] = msg_base + the message's index here (a chunk's first message)
    // emit_map_kernel in the sharded tick: rows whose info.x carries kLocPool read the received
    // cube-list pool at that word offset (wq_sharded.hip); nullptr everywhere else
    const uint32_t* pool = nullptr;
    // emit_map_kernel: OnlySelf rows read the sender at sender[m * sender_stride] (the owner form
    // of the sharded tick routes received slots: their sender is word 3 of 5)
    uint32_t sender_stride = 1;
};

// LDS of one emit row (256 messages): an image of a window of the row's output, aligned to
// 16-byte quads of the global output, and the messages whose list is read from `list`.
// The long-list queue of one row (messages with more than kInline peers or a full-key slot-table
// cube) and the row scan's wave totals.
struct EmitQueue {
    uint32_t gq_j[kBlock];    // message (row-local index)
    uint32_t gq_off[kBlock];  // ... index of the list's first peer in `list`
    uint32_t gq_skip[kBlock]; // ... skipped list index or kNone (radius mode: the list length)
    uint32_t gq_e[kBlock];    // ... outputs
    uint32_t gq_st[kBlock];   // ... row-local first output
    uint32_t gq_pre[kBlock + 1];  // ... prefix of their slices of the current window
    uint32_t scan_tot[kWaves];
    uint32_t n_gq;
};

template <int STAGE>
struct EmitRowSmem {
    alignas(16) uint32_t op[STAGE];  // peers of window positions, in output order
    alignas(16) uint8_t om[STAGE];   // ... and the row-local index of each position's message
    EmitQueue q;
};

struct EmitOut {
    const uint32_t* sender;
    uint32_t* peers;
    uint32_t* msgs;
    uint64_t capacity;
    const double* pos;     // message positions (radius mode)
    const uint8_t* repl;   // replication codes (radius mode)
    const uint32_t* pool = nullptr;  // radius mode in the sharded tick: rows with kLocPool read here
};

// Replication filter for one candidate (local_message.rs:60-86; replication.rs:34-43: every unknown
// code is ExceptSelf). Branch-free on purpose: written as nested selects, it was lowered to a switch
// whose unknown-code leaf inside count_radius_kernel's unrolled inline loop tested the radius
// against a stale register instead of the peer (codes >= 3 lost their recipients; ROCm 7.2 clang,
// gfx950) — tests/test_gpu_c345.py::test_radius_unknown_replication_codes.
__device__ __forceinline__ bool repl_keeps(uint8_t rp, uint32_t peer, uint32_t me) {
    const bool including = rp == WQ_REPL_INCLUDING_SELF, only = rp == WQ_REPL_ONLY_SELF;
    return including | (only == (peer == me));
}

// Row-local exclusive scan of e over the block's 256 threads; returns this thread's start and
// the row total.
__device__ __forceinline__ uint32_t row_scan(uint32_t e, uint32_t* wave_tot, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t incl = wave_incl_scan_add(e, lane);
    if (lane == 63) wave_tot[wave] = incl;
    lds_barrier();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int u = 0; u < kWaves; ++u) {
        const uint32_t t = wave_tot[u];
        if (u < wave) before += t;
        tot += t;
    }
    *total = tot;
    return before + incl - e;
}

// Kernel (3) for one row of 256 messages m0 + threadIdx.x whose filtered counts e, locators inf
// and row-local first outputs st the caller holds; the row's outputs go to [g0, g0 + T).
// The outputs are assembled in LDS in output order, in windows of STAGE positions aligned to the
// global output's 16-byte quads, then written with one 16-byte store per lane per array (the
// row's first and last quads, shared with the neighbouring rows, word by word).
//   inline records (<= kInline peers): eight lanes per record line, lane `part` < 6 reading chunk
//     2 + part = peers 4*part .. 4*part+3 only if it holds one of the message's peers; U rounds
//     of the wave's 64 messages in flight at once; the sender's own entry (radius mode: every
//     peer outside the locator's survivor mask) is dropped while staging;
//   longer lists: the window's slices of all of them are copied from `list` as one flat,
//     block-strided range (coalesced loads, four in flight per thread); in radius mode each list
//     is re-filtered chunk by chunk with a block-wide compaction;
//   OnlySelf: the sender, by its own lane.
// Every thread of the block must call it (it contains barriers); it ends with a barrier.
constexpr uint32_t kSlPool = 0x80000000u;  // emit_row_img, radius mode: sl is a pool word offset

template <int STAGE, int U = 8, bool RADIUS = false>
__device__ __forceinline__ void emit_row_img(uint32_t* op, uint8_t* om, EmitQueue& q_, const TableView& tv, const EmitOut& o, uint32_t m0,
                                         uint32_t e, uint2 inf, uint32_t st, uint64_t g0, uint32_t T) {
    static_assert(STAGE % 4 == 0, "STAGE: whole 16-byte quads");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) q_.n_gq = 0;
    lds_barrier();
    uint32_t sl = kNone, cnt = 0, skip = kNone;  // radius mode: skip holds the survivor mask
    // OnlySelf rows; in radius mode only the sharded tick's (count_radius folds OnlySelf into masks)
    const bool self = e && (RADIUS ? (inf.x & kLocPool) == kLocSelf : (inf.x & kLocSelf) != 0);
    const uint32_t self_peer = self ? o.sender[m0 + tid] : 0u;
    if (e && !self) {
        // radius mode: a row of the sharded tick's received pools (kLocPool | word offset): a short one
        // is staged like an inline record (sl = kSlPool | offset), a longer one re-filtered from the pool
        const bool from_pool = RADIUS && (inf.x & kLocPool) == kLocPool;
        if (from_pool && (inf.y & kPoolShort)) {
            sl = kSlPool | (inf.x & ~kLocPool);
            cnt = (inf.y >> 24) & 0x1Fu;
            skip = inf.y & kSkipNone24;
        } else if (inf.x & kLocGlobal) {
            const uint32_t q = atomicAdd(&q_.n_gq, 1u);
            q_.gq_j[q] = tid | (from_pool ? 0x100u : 0u);
            q_.gq_off[q] = from_pool ? (inf.x & ~kLocPool) : (inf.x & ~kLocGlobal) + 1;
            q_.gq_skip[q] = inf.y;
            q_.gq_e[q] = e;
            q_.gq_st[q] = st;
        } else {
            const uint32_t s24 = inf.y & kSkipNone24;
            sl = inf.x;
            cnt = inf.y >> 24;
            skip = RADIUS ? s24 : (s24 == kSkipNone24 ? kNone : s24);
        }
    }
    // record chunks of the wave's 64 messages: message q by lanes 8*(q%8) .. +7, round q/8,
    // U rounds of loads in flight at a time
    const int grp = lane >> 3, part = lane & 7;
    const uint4* recs4 = reinterpret_cast<const uint4*>(tv.recs);
    lds_barrier();
    const uint32_t n_gq = q_.n_gq;
    // window w covers global outputs [gA + w0, gA + w0 + STAGE), gA = g0 rounded down to a quad
    const uint64_t gA = g0 & ~3ull;
    const uint32_t lead = (uint32_t)(g0 - gA);  // row output r sits at image index lead + r - w0
    const uint32_t span = lead + T;
    for (uint32_t w0 = 0; w0 < span; w0 += STAGE) {
        const uint32_t w1 = span - w0 < (uint32_t)STAGE ? span : w0 + STAGE;
        if (self && lead + st >= w0 && lead + st < w1) {
            op[lead + st - w0] = self_peer;
            om[lead + st - w0] = (uint8_t)tid;
        }
#pragma unroll 1
        for (int r0 = 0; r0 < 8; r0 += U) {
            uint4 v[U];
            uint32_t q_cnt[U], q_skip[U], q_st[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int src = 8 * (r0 + u) + grp;
                const uint32_t qs = __shfl(sl, src, 64);
                q_cnt[u] = __shfl(cnt, src, 64);
                q_skip[u] = __shfl(skip, src, 64);
                q_st[u] = __shfl(st, src, 64);
                if (part < 6 && qs != kNone && 4u * part < q_cnt[u]) {
                    if (RADIUS && (qs & kSlPool)) {  // a short pool row: its words, none past its end
                        const uint32_t* pw = o.pool + (qs & ~kSlPool) + 4u * part;
                        const uint32_t i0 = 4u * part;
                        v[u] = make_uint4(pw[0], i0 + 1 < q_cnt[u] ? pw[1] : 0u, i0 + 2 < q_cnt[u] ? pw[2] : 0u,
                                          i0 + 3 < q_cnt[u] ? pw[3] : 0u);
                    } else {
                        v[u] = recs4[(uint64_t)qs * 8 + 2 + part];
                    }
                } else {
                    q_cnt[u] = 0;  // nothing to stage from this lane
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!q_cnt[u]) continue;
                const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                const uint8_t j = (uint8_t)(wave * 64 + 8 * (r0 + u) + grp);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t idx = 4u * part + i;  // peer index in the cube's list
                    uint32_t pos;
                    if (RADIUS) {
                        if (idx >= q_cnt[u] || !((q_skip[u] >> idx) & 1u)) continue;
                        pos = lead + q_st[u] + (uint32_t)__popc(q_skip[u] & ((1u << idx) - 1u));
                    } else {
                        if (idx >= q_cnt[u] || idx == q_skip[u]) continue;
                        pos = lead + q_st[u] + idx - (idx > q_skip[u] && q_skip[u] != kNone ? 1u : 0u);
                    }
                    if (pos >= w0 && pos < w1) {
                        op[pos - w0] = vv[i];
                        om[pos - w0] = j;
                    }
                }
            }
        }
        if (n_gq) {
            if (RADIUS) {
                // re-filter each long list chunk by chunk, compacting survivors block-wide
                for (uint32_t q = 0; q < n_gq; ++q) {
                    const uint32_t jq = q_.gq_j[q], j = jq & 0xFFu, s0 = lead + q_.gq_st[q], ej = q_.gq_e[q];
                    if (s0 >= w1 || s0 + ej <= w0) continue;  // block-uniform
                    const uint32_t off = q_.gq_off[q], len = q_.gq_skip[q];
                    const uint32_t* src = (jq & 0x100u) ? o.pool : tv.list;
                    const uint32_t m = m0 + j, me = o.sender[m];
                    const uint8_t rp = o.repl[m];
                    const double mx = o.pos[3ull * m], my = o.pos[3ull * m + 1], mz = o.pos[3ull * m + 2];
                    uint32_t run = 0;
                    for (uint32_t b = 0; b < len; b += kBlock) {
                        const uint32_t i = b + tid;
                        const uint32_t peer = i < len ? src[off + i] : 0u;
                        const bool ok = i < len && repl_keeps(rp, peer, me) && within_radius(tv, mx, my, mz, peer);
                        uint32_t tot;
                        const uint32_t at = row_scan(ok ? 1u : 0u, q_.scan_tot, &tot);
                        const uint32_t pos = s0 + run + at;
                        if (ok && pos >= w0 && pos < w1) {
                            op[pos - w0] = peer;
                            om[pos - w0] = (uint8_t)j;
                        }
                        run += tot;
                        lds_barrier();  // scan_tot reuse
                    }
                }
            } else {
                // the window's slices of every long list as one flat, block-strided range
                if (tid == 0) {
                    uint32_t acc = 0;
                    for (uint32_t q = 0; q < n_gq; ++q) {
                        const uint32_t s0 = lead + q_.gq_st[q], ej = q_.gq_e[q];
                        const uint32_t lo = s0 > w0 ? s0 : w0, hi = s0 + ej < w1 ? s0 + ej : w1;
                        q_.gq_pre[q] = acc;
                        acc += hi > lo ? hi - lo : 0u;
                    }
                    q_.gq_pre[n_gq] = acc;
                }
                lds_barrier();
                const uint32_t W = q_.gq_pre[n_gq];
                uint32_t q = 0;
                for (uint32_t k0 = tid; k0 < W; k0 += 4 * kBlock) {
                    uint32_t val[4], dst[4], jj[4];
                    bool ok[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t k = k0 + u * kBlock;
                        ok[u] = k < W;
                        if (!ok[u]) continue;
                        while (q_.gq_pre[q + 1] <= k) ++q;  // owners ascend with k
                        const uint32_t s0 = lead + q_.gq_st[q];
                        const uint32_t lo = s0 > w0 ? s0 : w0;
                        const uint32_t posn = lo + (k - q_.gq_pre[q]);  // image-space position
                        const uint32_t oi = posn - s0, sk = q_.gq_skip[q];
                        val[u] = tv.list[q_.gq_off[q] + oi + (oi >= sk ? 1u : 0u)];
                        dst[u] = posn - w0;
                        jj[u] = q_.gq_j[q];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (!ok[u]) continue;
                        op[dst[u]] = val[u];
                        om[dst[u]] = (uint8_t)jj[u];
                    }
                }
            }
        }
        lds_barrier();
        // copy-out, quad t of the window by thread t % 256
        for (uint32_t qd = w0 + 4u * tid; qd < w1; qd += 4u * kBlock) {
            const uint4 pv = *reinterpret_cast<const uint4*>(&op[qd - w0]);
            const uint32_t mv = *reinterpret_cast<const uint32_t*>(&om[qd - w0]);
            const uint64_t out0 = gA + qd;
            const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
            const uint32_t mw[4] = {m0 + (mv & 0xFF), m0 + ((mv >> 8) & 0xFF), m0 + ((mv >> 16) & 0xFF), m0 + (mv >> 24)};
            if (qd >= lead && qd + 4 <= span && out0 + 4 <= o.capacity) {
                *reinterpret_cast<uint4*>(o.peers + out0) = pv;
                if (o.msgs) *reinterpret_cast<uint4*>(o.msgs + out0) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i) {
                    if (qd + i >= lead && qd + i < span && out0 + i < o.capacity) {
                        o.peers[out0 + i] = pw[i];
                        if (o.msgs) o.msgs[out0 + i] = mw[i];
                    }
                }
            }
        }
        lds_barrier();  // the next window (or the caller's next row) reuses the image
    }
}

template <int STAGE, int U = 8, bool RADIUS = false>
__device__ __forceinline__ void emit_row(EmitRowSmem<STAGE>& sm, const TableView& tv, const EmitOut& o, uint32_t m0,
                                         uint32_t e, uint2 inf, uint32_t st, uint64_t g0, uint32_t T) {
    emit_row_img<STAGE, U, RADIUS>(sm.op, sm.om, sm.q, tv, o, m0, e, inf, st, g0, T);
}


// Heavy fan-out (T > STAGE, e.g. C3's hotspots): instead of emit_row's windows, which re-read the
// block's 256 record lines once per STAGE outputs, the block's outputs are written straight to
// the global output, one output per thread and pass: output r (row-local) belongs to the message
// j with st[j] <= r < st[j] + e[j] (binary search over the row's exclusive prefixes in LDS), and
// its peer comes from the record's inline words (L2-resident since the count read them), the
// cube's list, or the sender (OnlySelf). Consecutive threads write consecutive outputs, so every
// store instruction is one contiguous 256-word run. The image's LDS is reused for the per-message
// descriptors: op[0..255] st, op[256..511] source, op[512..767] skipped index, om[0..255] kind.
constexpr uint8_t kDirNone = 0, kDirInline = 1, kDirList = 2, kDirSelf = 3;

// The descriptors' LDS on its own (the heavy-row emit kernel needs nothing else): 4 KB per block.
struct DirectSmem {
    alignas(16) uint32_t op[3 * kBlock];
    uint8_t om[kBlock];
};

template <class SM>
__device__ __forceinline__ void direct_meta(SM& es, const EmitOut& out, uint32_t m, uint32_t e, uint2 inf,
                                            uint32_t st) {
    static_assert(sizeof(es.op) >= 3 * kBlock * sizeof(uint32_t), "room for three descriptor arrays");
    const int tid = threadIdx.x;
    uint8_t kind = kDirNone;
    uint32_t src = 0, skip = kNone;
    if (e) {
        if (inf.x & kLocSelf) {
            kind = kDirSelf;
            src = out.sender[m];
        } else if (inf.x & kLocGlobal) {
            kind = kDirList;
            src = (inf.x & ~kLocGlobal) + 1;
            skip = inf.y;
        } else {
            kind = kDirInline;
            src = inf.x;
            const uint32_t s24 = inf.y & kSkipNone24;
            skip = s24 == kSkipNone24 ? kNone : s24;
        }
    }
    es.op[tid] = st;
    es.op[kBlock + tid] = src;
    es.op[2 * kBlock + tid] = skip;
    es.om[tid] = kind;
}

template <int R, class SM>
__device__ __forceinline__ void emit_direct(const SM& es, const TableView& tv, const EmitOut& out, uint32_t m0,
                                            uint64_t g0, uint32_t T) {
    // R: outputs per thread per pass. The R binary searches run in lockstep (each of the 8 rounds
    // issues R LDS reads, then waits once) and the peer loads are branch-free (one address select,
    // R loads in flight): written as R independent loops with per-output branches, the compiler
    // serialised them — 8 dependent LDS round trips per output, the emit's main cost on C3.
    const uint32_t* recs32 = reinterpret_cast<const uint32_t*>(tv.recs);
    for (uint32_t r0 = threadIdx.x; r0 < T; r0 += R * kBlock) {
        uint32_t rr[R], lo[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t r = r0 + u * kBlock;
            rr[u] = r < T ? r : T - 1;  // clamped: a valid output, its store is masked below
            lo[u] = 0;                  // last j with st[j] <= r (st[0] = 0)
        }
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const uint32_t half = 128u >> it;
            uint32_t t[R];
#pragma unroll
            for (int u = 0; u < R; ++u) t[u] = es.op[lo[u] + half];
#pragma unroll
            for (int u = 0; u < R; ++u) lo[u] += t[u] <= rr[u] ? half : 0u;
        }
        uint32_t peer[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t j = lo[u];
            const uint32_t k = rr[u] - es.op[j], src = es.op[kBlock + j], sk = es.op[2 * kBlock + j];
            const uint32_t idx = k + (k >= sk ? 1u : 0u);
            const uint8_t kind = es.om[j];
            const uint32_t* a = kind == kDirList     ? tv.list + ((uint64_t)src + idx)
                                : kind == kDirInline ? recs32 + ((uint64_t)src * 32 + kInlineWord0 + idx)
                                                     : tv.list;  // OnlySelf / none: a safe dummy load
            peer[u] = *a;
            if (kind == kDirSelf) peer[u] = src;
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t r = r0 + u * kBlock;
            const uint64_t o = g0 + r;
            if (r < T && o < out.capacity) {
                out.peers[o] = peer[u];
                if (out.msgs) out.msgs[o] = m0 + lo[u];
            }
        }
    }
}

// Pass 3 of the three-launch tick: one 256-message row per block. CSR offsets = count-block
// prefix (tile_scan) + the in-block prefix, then emit_row.
template <int STAGE, int U, bool RADIUS = false>
__global__ __launch_bounds__(kBlock) void emit_kernel(EmitParams p) {
    __shared__ EmitRowSmem<STAGE> sm;
    __shared__ uint32_t wave_tot[kWaves];
    __shared__ uint32_t part_tot[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t m0 = blockIdx.x * kBlock;
    const uint32_t m = m0 + tid;
    const uint32_t e = m < p.M ? p.e[m] : 0u;
    const uint2 inf = (p.peers && m < p.M) ? p.info[m] : make_uint2(0, kNone);
    const uint32_t ct0 = (m0 / p.count_tile) * p.count_tile;
    uint32_t g = p.tile_prefix[m0 / p.count_tile];
    // earlier rows of the same count block
    uint32_t part = 0;
    for (uint32_t k = ct0 + tid; k < m0; k += kBlock) part += p.e[k];
    part = (uint32_t)wave_sum_u64(part);
    if (lane == 0) part_tot[wave] = part;
    uint32_t T;
    const uint32_t st = row_scan(e, wave_tot, &T);  // (its barrier also publishes part_tot)
#pragma unroll
    for (int u = 0; u < kWaves; ++u) g += part_tot[u];
    if (m < p.M) p.offsets[m] = g + st;
    if (!p.peers) return;  // counts-only call: offsets are all that is asked for
    if (!RADIUS && T > (uint32_t)STAGE) {  // block-uniform: heavy fan-out, no windows
        direct_meta(sm, EmitOut{p.sender, p.peers, p.msgs, p.capacity, p.pos, p.repl, p.pool}, m, e, inf, st);
        lds_barrier();
        emit_direct<16>(sm, p.t, EmitOut{p.sender, p.peers, p.msgs, p.capacity, p.pos, p.repl, p.pool}, m0, g, T);
        return;
    }
    emit_row<STAGE, U, RADIUS>(sm, p.t, EmitOut{p.sender, p.peers, p.msgs, p.capacity, p.pos, p.repl, p.pool}, m0, e, inf,
                               st, g, T);
}

// Pass 3 for heavy fan-out (wq_set_fanout_hint, C3): every row through emit_direct, whatever its
// size, so the block needs only the 4 KB of descriptors instead of emit_kernel's 27 KB image — 8
// blocks (32 waves) per CU instead of 5, i.e. more peer loads in flight. Offsets as emit_kernel.
template <int R>
__global__ __launch_bounds__(kBlock) void emit_heavy_kernel(EmitParams p) {
    __shared__ DirectSmem sm;
    __shared__ uint32_t wave_tot[kWaves];
    __shared__ uint32_t part_tot[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t m0 = blockIdx.x * kBlock;
    const uint32_t m = m0 + tid;
    const uint32_t e = m < p.M ? p.e[m] : 0u;
    const uint2 inf = (p.peers && m < p.M) ? p.info[m] : make_uint2(0, kNone);
    const uint32_t ct0 = (m0 / p.count_tile) * p.count_tile;
    uint32_t g = p.tile_prefix[m0 / p.count_tile];
    uint32_t part = 0;
    for (uint32_t k = ct0 + tid; k < m0; k += kBlock) part += p.e[k];
    part = (uint32_t)wave_sum_u64(part);
    if (lane == 0) part_tot[wave] = part;
    uint32_t T;
    const uint32_t st = row_scan(e, wave_tot, &T);
#pragma unroll
    for (int u = 0; u < kWaves; ++u) g += part_tot[u];
    if (m < p.M) p.offsets[m] = g + st;
    if (!p.peers) return;
    const EmitOut out{p.sender, p.peers, p.msgs, p.capacity, p.pos, p.repl};
    direct_meta(sm, out, m, e, inf, st);
    lds_barrier();
    emit_direct<R>(sm, p.t, out, m0, g, T);
}

// Pass 3 for heavy fan-out, owner-map form (C3): per message one 16-byte descriptor {row start,
// skipped index, pointer to its first recipient word} — the cube's list, the record's inline
// peers, or the sender itself for OnlySelf — so each output is one LDS descriptor read, a
// subtract, a compare and one global load. Outputs go in windows of W = R * 256: every message
// marks where its range enters the window in a u16 owner map (index + 1), a block-wide max-scan
// carries each owner over its outputs, and thread t then writes outputs t, t + 256, ... of the
// window (one contiguous 256-word run per store instruction). Against emit_direct's per-output
// binary search (8 dependent LDS rounds, ~70 VALU per output, issue-bound on C3) this is a few
// VALU per output plus the scan's share.
template <int R>
struct MapSmem {
    alignas(16) uint4 desc[kBlock];
    alignas(16) uint16_t map[R * kBlock];
    uint32_t wave_max[kWaves];
};

template <int R>
__global__ __launch_bounds__(kBlock) void emit_map_kernel(EmitParams p) {
    static_assert(R % 8 == 0, "map rows of whole 16-byte words");
    constexpr uint32_t W = R * kBlock;
    __shared__ MapSmem<R> sm;
    __shared__ uint32_t wave_tot[kWaves];
    __shared__ uint32_t part_tot[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nbk = p.n_blocks ? p.n_blocks : gridDim.x;
    for (uint32_t blk = blockIdx.x; blk < nbk; blk += gridDim.x) {
    const uint32_t m0 = blk * kBlock;
    const uint32_t m = m0 + tid;
    const uint32_t e = m < p.M ? p.e[m] : 0u;
    const uint2 inf = (p.peers && m < p.M) ? p.info[m] : make_uint2(0, kNone);
    const uint32_t ct0 = (m0 / p.count_tile) * p.count_tile;
    uint32_t g = p.tile_prefix[m0 / p.count_tile];
    uint32_t part = 0;
    for (uint32_t k = ct0 + tid; k < m0; k += kBlock) part += p.e[k];
    part = (uint32_t)wave_sum_u64(part);
    if (lane == 0) part_tot[wave] = part;
    uint32_t T;
    const uint32_t st = row_scan(e, wave_tot, &T);
#pragma unroll
    for (int u = 0; u < kWaves; ++u) g += part_tot[u];
    if (m < p.M) p.offsets[m] = g + st;
    if (p.peers && T != 0) {
    // the descriptor: recipient k of the message is word k + (k >= skip) from `base`
    const uint32_t* base = p.t.list;
    uint32_t skip = kNone;
    if (e) {
        if (p.pool && (inf.x & kLocPool) == kLocPool) {
            base = p.pool + (inf.x & kLocMask);
            skip = inf.y;
        } else if (inf.x & kLocSelf) {
            base = p.sender + (uint64_t)m * p.sender_stride;
        } else if (inf.x & kLocGlobal) {
            base = p.t.list + (inf.x & ~kLocGlobal) + 1;
            skip = inf.y;
        } else {
            base = reinterpret_cast<const uint32_t*>(p.t.recs) + ((uint64_t)inf.x * 32 + kInlineWord0);
            const uint32_t s24 = inf.y & kSkipNone24;
            skip = s24 == kSkipNone24 ? kNone : s24;
        }
    }
    const uint64_t bp = reinterpret_cast<uint64_t>(base);
    sm.desc[tid] = make_uint4(st, skip, (uint32_t)bp, (uint32_t)(bp >> 32));
    uint4* my_map = reinterpret_cast<uint4*>(sm.map) + tid * (R / 8);
    for (uint32_t w0 = 0; w0 < T; w0 += W) {
#pragma unroll
        for (int q = 0; q < R / 8; ++q) my_map[q] = make_uint4(0, 0, 0, 0);
        lds_barrier();
        // the message whose range enters the window at position x marks map[x]
        if (e && st + e > w0 && st < w0 + W) sm.map[(st > w0 ? st : w0) - w0] = (uint16_t)(tid + 1);
        lds_barrier();
        // block-wide inclusive max-scan of the map (owners only grow along the row)
        uint4 v[R / 8];
#pragma unroll
        for (int q = 0; q < R / 8; ++q) v[q] = my_map[q];
        uint32_t run = 0;
#pragma unroll
        for (int q = 0; q < R / 8; ++q) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&v[q]);
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                uint32_t lo = w[h] & 0xFFFFu, hi = w[h] >> 16;
                run = lo > run ? lo : run;
                lo = run;
                run = hi > run ? hi : run;
                w[h] = lo | (run << 16);
            }
        }
        const uint32_t incl = wave_incl_scan_max(run, lane);
        uint32_t pre = __shfl_up(incl, 1, 64);
        if (lane == 0) pre = 0;
        if (lane == 63) sm.wave_max[wave] = incl;
        lds_barrier();
#pragma unroll
        for (int u = 0; u < kWaves; ++u)
            if (u < wave) pre = sm.wave_max[u] > pre ? sm.wave_max[u] : pre;
#pragma unroll
        for (int q = 0; q < R / 8; ++q) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&v[q]);
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t lo = w[h] & 0xFFFFu, hi = w[h] >> 16;
                w[h] = (lo > pre ? lo : pre) | ((hi > pre ? hi : pre) << 16);
            }
            my_map[q] = v[q];
        }
        lds_barrier();
        // outputs w0 + tid + 256 u; past the row's end a clamped position (valid owner, no store)
        const uint32_t last = (T - 1 - w0) < W - 1 ? (T - 1 - w0) : W - 1;
        uint32_t peer[R], own[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t x = (uint32_t)(u * kBlock + tid) < last ? (uint32_t)(u * kBlock + tid) : last;
            const uint32_t j = (uint32_t)sm.map[x] - 1u;
            const uint4 d = sm.desc[j];
            const uint32_t k = w0 + x - d.x;
            const uint32_t* a = reinterpret_cast<const uint32_t*>(((uint64_t)d.w << 32) | d.z);
            peer[u] = a[k + (k >= d.y ? 1u : 0u)];
            own[u] = j;
        }
        // both stores after all R loads: storing the message index first, between the loads,
        // measured 14% slower on C3
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t r = w0 + u * kBlock + tid;
            const uint64_t o = (uint64_t)g + r;
            if (r < T && o < p.capacity) {
                p.peers[o] = peer[u];
                if (p.msgs) p.msgs[o] = p.msg_base + m0 + own[u];
            }
        }
        lds_barrier();  // the next window rewrites the map
    }
    }  // outputs
    lds_barrier();  // the next block's scan and descriptors reuse the LDS
    }  // blocks
}

}  // namespace wq
