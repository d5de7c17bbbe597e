// wq_route.hip — the LocalMessage hot path on gfx950: launch selection for one tick.
//
// Replaces, per message, worldql_server/src/processing/local_message.rs:52-86:
//   world_map.get(world) -> Vector3::to_cube_area (cube_area.rs:72-77 -> coord_clamp :23-44)
//   -> AreaMap::get_subscribed_peers (area_map.rs:52-60) -> replication filter (:60-86).
//
// Default: ONE launch (route_tick.hpp: count from the whole record line held in registers, block
// scan, LDS image of the block's outputs, decoupled look-back, aligned 16-byte copy-out). Other
// compiled shapes, selectable with wq_debug_set_route_config and identical in output: the same
// single launch with other image sizes, and three launches (route_count.hpp count_kernel,
// route_scan.hpp tile_scan_kernel, route_emit.hpp emit_kernel) which re-read the record lines
// once but never wait on another block. The radius filter (route_radius.hpp) always takes three
// launches. DESIGN.md §4-5 has the measurements behind each choice.
// Output: CSR offsets[M+1] (message-major), peers[P], optional msgs[P].
#include <algorithm>
#include <cstdlib>

#include "route_count.hpp"
#include "route_emit.hpp"
#include "route_scan.hpp"
#include "route_tick.hpp"
#include "route_radius.hpp"
#include "route_spill.hpp"

namespace wq {

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
namespace {
constexpr int kSpillStage = 2816;

struct Cfg {
    int count_tile;  // messages per tile_total entry
    void (*count)(const CountParams&, hipStream_t, unsigned);
    int emit_stage;  // emit window positions (4096 or 8192)
    // single-launch tick (route_tick.hpp): its LDS image positions, or 0 for three launches
    int tick_stage;
    void (*tick)(const TickParams&, hipStream_t, unsigned);
    // count+spill / tile_scan / copy (route_spill.hpp): image positions per block, or 0
    int spill_stage;
    // three launches: 0 = emit_kernel (windowed image, heavy rows through emit_direct), the
    // outputs in flight per thread of emit_heavy_kernel (every row through emit_direct, 4 KB LDS),
    // or 100 + outputs per thread per window of emit_map_kernel (owner map)
    int emit_heavy;
};

template <int IPT, int MINW, bool FULL = false>
void launch_count(const CountParams& p, hipStream_t s, unsigned grid) {
    if (p.in.keys)
        hipLaunchKernelGGL((count_kernel<true, IPT, MINW, 0, FULL>), dim3(grid), dim3(kBlock), 0, s, p);
    else
        hipLaunchKernelGGL((count_kernel<false, IPT, MINW, 0, FULL>), dim3(grid), dim3(kBlock), 0, s, p);
}

// route config 13: one-wave count blocks of 64 messages (route_count.hpp count_wave_kernel)
void launch_count_wave(const CountParams& p, hipStream_t s, unsigned grid) {
    if (p.in.keys)
        hipLaunchKernelGGL((count_wave_kernel<true, 32>), dim3(grid), dim3(64), 0, s, p);
    else
        hipLaunchKernelGGL((count_wave_kernel<false, 32>), dim3(grid), dim3(64), 0, s, p);
}

template <int STAGE, int U, bool NT = false>
void launch_tick(const TickParams& p, hipStream_t s, unsigned grid) {
    if (p.in.keys)
        hipLaunchKernelGGL((tick_kernel<true, STAGE, U, NT>), dim3(grid), dim3(kBlock), 0, s, p);
    else
        hipLaunchKernelGGL((tick_kernel<false, STAGE, U, NT>), dim3(grid), dim3(kBlock), 0, s, p);
}

#define WQ_CFG3(cipt, minw, stage) {kBlock * cipt, &launch_count<cipt, minw>, stage, 0, nullptr, 0, 0}
#define WQ_CFG3H(r) {kBlock, &launch_count<1, 8>, 4096 + 2, 0, nullptr, 0, r}
#define WQ_CFG1(stage, u) {kBlock, &launch_count<1, 8>, 4096, stage, &launch_tick<stage, u, true>, 0, 0}
#define WQ_CFGS(stage) {kBlock, &launch_count<1, 8>, 4096, 0, nullptr, stage, 0}
// Three launches: count (messages per lane, min waves per SIMD) / tile_scan / emit. One launch:
// messages per block; its three-launch fallback (too many blocks to be resident) is count 4/2.
const Cfg kCfgs[] = {
    WQ_CFG1(2816, 2),         // 0: default, single launch; 20.3 KB LDS -> 8 blocks per CU (63.3 us on C2);
                              //    the image leaves by non-temporal 16-byte stores (streamed, never re-read)
    WQ_CFG3(1, 8, 4096 + 2),  // 1: three launches (73 us on C2)
    WQ_CFG1(4096, 2),         // 2
    WQ_CFG3(1, 8, 4096 + 8),  // 3
    WQ_CFG3(4, 2, 4096 + 2),  // 4
    WQ_CFG1(3072, 2),         // 5: 21.6 KB LDS -> 7 blocks per CU (65.6 us)
    WQ_CFG1(2560, 2),         // 6: C2 blocks overflow the image (78 us)
    WQ_CFGS(kSpillStage),     // 7: count+spill / tile_scan / copy, no block waits on another
    WQ_CFG3H(16),             // 8: three launches, emit_heavy_kernel (16 outputs in flight per thread)
    WQ_CFG3H(8),              // 9: ... 8 in flight
    // 10: three launches, emit_map_kernel (owner map, 16 outputs per thread per window): C3 1288 us
    //     against cfg 8's 1472 us on one box (R = 8: 1366, R = 32: 1412; storing the message index
    //     before the peer loads land: 1467)
    WQ_CFG3H(116),
    WQ_CFG3H(108),            // 11: ... 8 per window
    // 12: cfg 0 with plain (not non-temporal) copy-out stores: C2 64.8 us against cfg 0's 63.2
    //     (tools/tune_route.py, 4 rounds; a non-temporal emit_map on C3 was 4% slower, not kept)
    {kBlock, &launch_count<1, 8>, 4096, 2816, &launch_tick<2816, 2, false>, 0, 0},
    // 13: cfg 10 with one-wave count blocks of 64 messages (count_wave_kernel; round-6 experiment)
    {64, &launch_count_wave, 4096 + 2, 0, nullptr, 0, 116},
};
#undef WQ_CFG1
#undef WQ_CFGS
#undef WQ_CFG3
#undef WQ_CFG3H
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);
constexpr int kCfgHeavy = 10;                // the default shape under wq_set_fanout_hint >= WQ_HEAVY_FANOUT (emit_map_kernel)
constexpr uint32_t kShortTickTiles = 12288;  // 256-message tiles up to which a tick is "short" (above)

}  // namespace

int route_config_count() { return kNumCfgs; }
uint32_t route_tiles_per_block(uint32_t tiles) { return tiles <= kShortTickTiles ? 1u : 2u; }

int route_counters(wq_router* h, size_t M, uint32_t* d_offsets, wq_route_counters** cur_out,
                   wq_route_counters** nxt_out) {
    hipStream_t s = h->stream;
    RouteWs& rw = h->rws;
    // workspace: [health u32 x2, pad to 64][counters x2 (24 B each)] — each call's count pass
    // zeroes the next slot; the health words are only cleared by wq_route_health
    if (!rw.buf.p) {
        WQ_ALLOC(h, rw.buf, 128);
        WQ_HIP(h, hipMemsetAsync(rw.buf.p, 0, 128, s));
        rw.calls = 0;
    }
    char* base = rw.buf.as<char>();
    wq_route_counters* ring = reinterpret_cast<wq_route_counters*>(base + 64);
    wq_route_counters* cur = ring + (rw.calls & 1);
    wq_route_counters* nxt = ring + ((rw.calls + 1) & 1);
    rw.last = cur;
    *cur_out = cur;
    *nxt_out = nxt;
    if (M == 0) {
        WQ_HIP(h, hipMemsetAsync(d_offsets, 0, 4, s));
        WQ_HIP(h, hipMemsetAsync(cur, 0, sizeof(wq_route_counters), s));
        WQ_HIP(h, hipMemsetAsync(nxt, 0, sizeof(wq_route_counters), s));
        rw.calls++;
        *cur_out = nullptr;  // nothing to launch
    }
    return WQ_OK;
}

int launch_route(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                 const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                 uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    hipStream_t s = h->stream;
    RouteWs& rw = h->rws;
    // fold in a finished incremental batch (never waits: an unfinished one that turns out not to
    // be applied shows as error bit 8 in this tick's counters)
    if (int rc = table_resolve(h, false)) return rc;
    const Cfg& cfg = kCfgs[h->route_cfg == 0 && h->heavy_fanout ? kCfgHeavy : h->route_cfg];
    wq_route_counters *cur, *nxt;
    int rc0 = route_counters(h, M, d_offsets, &cur, &nxt);
    if (rc0 || !cur) return rc0;
    const TableView tv = table_view(h);
    ProfileEvents& pr = h->prof;
    if (pr.enabled) {
        if (pr.used == pr.start.size()) {
            hipEvent_t a, b, c, d;
            WQ_HIP(h, hipEventCreate(&a));
            WQ_HIP(h, hipEventCreate(&b));
            WQ_HIP(h, hipEventCreate(&c));
            WQ_HIP(h, hipEventCreate(&d));
            pr.start.push_back(a);
            pr.stop.push_back(b);
            pr.mid1.push_back(c);
            pr.mid2.push_back(d);
            pr.phased.push_back(0);
        }
        pr.phased[pr.used] = 0;
        WQ_HIP(h, hipEventRecord(pr.start[pr.used], s));
    }
    const RouteIn in{d_pos, d_keys, d_world, d_sender, d_repl, (uint32_t)M, (int64_t)h->cube_size};

    const bool radius = h->radius > 0.0;
    if (radius && !d_pos) return set_error(h, WQ_E_INVALID, "the radius filter needs message positions");
    if (cfg.tick && !radius) {  // single launch: one block per 256 messages, decoupled look-back
        const uint64_t nb = (M + kBlock - 1) / kBlock;
        WQ_ALLOC(h, rw.agg, 2 * nb * 8);
        if (rw.agg_zeroed < 2 * nb) {  // fresh granules: tag 0 never matches a call's tag
            WQ_HIP(h, hipMemsetAsync(rw.agg.p, 0, rw.agg.bytes, s));
            rw.agg_zeroed = rw.agg.bytes / 8;
        }
        TickParams tp;
        tp.in = in;
        tp.t = tv;
        tp.offsets = d_offsets;
        tp.out = EmitOut{d_sender, capacity ? d_peers : nullptr, d_msgs, capacity, d_pos, d_repl};
        tp.look = rw.agg.as<uint64_t>();
        tp.fgran = tp.look + nb;
        tp.tag = (uint32_t)(rw.calls % ((1ull << 30) - 1)) + 1u;
        tp.cnt = cur;
        tp.cnt_next = nxt;
        tp.health = route_health(h);
        tp.stamps = rw.stamps;
        tp.n_tiles = (uint32_t)nb;
        // the caller's counters: a copy launch after the tick by default. The tick's last block can
        // write them itself (WQ_TICK_OUTCNT=1), one launch fewer, but its extra tail made C2 slower:
        // 62.8-63.4 against 62.5-62.8 us, alternating on one box (profiles/r06_tick_outcnt_ab.json)
        static const bool outcnt_in_tick = getenv("WQ_TICK_OUTCNT") && atoi(getenv("WQ_TICK_OUTCNT")) != 0;
        tp.out_cnt = outcnt_in_tick ? rw.out : nullptr;
        cfg.tick(tp, s, (unsigned)nb);
        WQ_HIP(h, hipGetLastError());
        rw.out_done = tp.out_cnt != nullptr;
        if (pr.enabled) {
            WQ_HIP(h, hipEventRecord(pr.stop[pr.used], s));
            pr.used++;
        }
        rw.calls++;
        return WQ_OK;
    }

    if (cfg.spill_stage && !radius) {  // count+spill / tile_scan / copy
        const uint64_t nb = (M + kBlock - 1) / kBlock;
        WQ_ALLOC(h, rw.info, M * sizeof(uint2));
        WQ_ALLOC(h, rw.e, M * 4);
        WQ_ALLOC(h, rw.tiles, nb * 12);
        if (capacity) WQ_ALLOC(h, rw.spill, nb * (uint64_t)kSpillStage * 5);
        SpillParams sp;
        sp.in = in;
        sp.t = tv;
        sp.out = EmitOut{d_sender, capacity ? d_peers : nullptr, d_msgs, capacity, d_pos, d_repl};
        sp.offsets = d_offsets;
        sp.e = rw.e.as<uint32_t>();
        sp.info = rw.info.as<uint2>();
        sp.tile_total = rw.tiles.as<uint32_t>();
        sp.tile_F = sp.tile_total + 2 * nb;
        sp.tile_prefix = sp.tile_total + nb;
        sp.spill_p = capacity ? rw.spill.as<uint32_t>() : nullptr;
        sp.spill_m = capacity ? reinterpret_cast<uint8_t*>(sp.spill_p + nb * kSpillStage) : nullptr;
        sp.cnt_next = nxt;
        if (in.keys)
            hipLaunchKernelGGL((spill_count_kernel<true, kSpillStage>), dim3(nb), dim3(kBlock), 0, s, sp);
        else
            hipLaunchKernelGGL((spill_count_kernel<false, kSpillStage>), dim3(nb), dim3(kBlock), 0, s, sp);
        WQ_HIP(h, hipGetLastError());
        TileScanParams tsp;
        tsp.tile_total = sp.tile_total;
        tsp.tile_F = sp.tile_F;
        tsp.tile_prefix = rw.tiles.as<uint32_t>() + nb;
        tsp.n_tiles = (uint32_t)nb;
        tsp.offsets = d_offsets;
        tsp.M = (uint32_t)M;
        tsp.capacity = capacity;
        tsp.cnt = cur;
        tsp.health = route_health(h);
        tsp.stale = tv.stale;
        if (int rc = launch_tile_scan(h, tsp)) return rc;
        hipLaunchKernelGGL((spill_copy_kernel<kSpillStage, 2>), dim3(nb), dim3(kBlock), 0, s, sp);
        WQ_HIP(h, hipGetLastError());
        if (pr.enabled) {
            WQ_HIP(h, hipEventRecord(pr.stop[pr.used], s));
            pr.used++;
        }
        rw.calls++;
        return WQ_OK;
    }

    const uint32_t count_tile = radius ? (uint32_t)kBlock : (uint32_t)cfg.count_tile;
    const uint32_t n_count = (uint32_t)((M + count_tile - 1) / count_tile);
    WQ_ALLOC(h, rw.info, M * sizeof(uint2));
    WQ_ALLOC(h, rw.e, M * 4);
    WQ_ALLOC(h, rw.tiles, (uint64_t)n_count * 12);
    uint32_t* tile_total = rw.tiles.as<uint32_t>();
    uint32_t* tile_prefix = tile_total + n_count;
    uint32_t* tile_F = tile_prefix + n_count;

    // Pipelined heavy tick: the messages in C chunks of whole count tiles; the chunks' counts run
    // back to back on a side stream while the launch stream scans and emits the chunks before them
    // (the scans carry {P, F} from chunk to chunk), so a latency-bound count overlaps a
    // bandwidth-bound emit. WQ_ROUTE_CHUNKS sets C (1 = the plain three launches).
    static const uint32_t chunks_env =
        getenv("WQ_ROUTE_CHUNKS") ? (uint32_t)std::max(1, atoi(getenv("WQ_ROUTE_CHUNKS"))) : 1u;
    const uint32_t want = h->route_chunks ? h->route_chunks : chunks_env;
    const uint32_t nchunk = (!radius && cfg.emit_heavy == 116 && count_tile == (uint32_t)kBlock && want > 1 &&
                             n_count >= 2 * want && (n_count + want - 1) / want <= kScanOneBlockMax)
                                ? want
                                : 1u;
    if (nchunk > 1) {
        if (!rw.side) WQ_HIP(h, hipStreamCreateWithFlags(&rw.side, hipStreamNonBlocking));
        if (!rw.ev_in) WQ_HIP(h, hipEventCreateWithFlags(&rw.ev_in, hipEventDisableTiming | hipEventReleaseToDevice));
        while (rw.cev.size() < nchunk) {
            hipEvent_t ev;
            WQ_HIP(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice));
            rw.cev.push_back(ev);
        }
        WQ_ALLOC(h, rw.carry, 16);
        // the side stream starts where the caller's stream is: inputs complete, the previous tick's
        // emit (which read e / info) done
        WQ_HIP(h, hipEventRecord(rw.ev_in, s));
        WQ_HIP(h, hipStreamWaitEvent(rw.side, rw.ev_in, 0));
        auto bounds = [&](uint32_t c, uint32_t* t0, uint32_t* t1, uint64_t* lo, uint64_t* hi) {
            *t0 = (uint32_t)((uint64_t)n_count * c / nchunk);
            *t1 = (uint32_t)((uint64_t)n_count * (c + 1) / nchunk);
            *lo = (uint64_t)*t0 * kBlock;
            *hi = std::min<uint64_t>(M, (uint64_t)*t1 * kBlock);
        };
        for (uint32_t c = 0; c < nchunk; ++c) {
            uint32_t t0, t1;
            uint64_t lo, hi;
            bounds(c, &t0, &t1, &lo, &hi);
            CountParams cp;
            cp.in = RouteIn{d_pos ? d_pos + 3 * lo : nullptr, d_keys ? d_keys + 3 * lo : nullptr, d_world + lo,
                            d_sender + lo, d_repl + lo, (uint32_t)(hi - lo), (int64_t)h->cube_size};
            cp.t = tv;
            cp.e = rw.e.as<uint32_t>() + lo;
            cp.info = rw.info.as<uint2>() + lo;
            cp.tile_total = tile_total + t0;
            cp.tile_F = tile_F + t0;
            cp.cnt = cur;
            cp.cnt_next = nxt;
            cp.health = route_health(h);
            cp.n_tiles = t1 - t0;
            cfg.count(cp, rw.side, t1 - t0);
            WQ_HIP(h, hipGetLastError());
            WQ_HIP(h, hipEventRecord(rw.cev[c], rw.side));
        }
        for (uint32_t c = 0; c < nchunk; ++c) {
            uint32_t t0, t1;
            uint64_t lo, hi;
            bounds(c, &t0, &t1, &lo, &hi);
            WQ_HIP(h, hipStreamWaitEvent(s, rw.cev[c], 0));
            TileScanParams sp;
            sp.tile_total = tile_total + t0;
            sp.tile_F = tile_F + t0;
            sp.tile_prefix = tile_prefix + t0;
            sp.n_tiles = t1 - t0;
            sp.offsets = d_offsets;
            sp.M = (uint32_t)M;
            sp.capacity = capacity;
            sp.cnt = cur;
            sp.health = route_health(h);
            sp.stale = tv.stale;
            sp.carry = rw.carry.as<uint64_t>();
            sp.chunk = (c > 0 ? 1u : 0u) | (c + 1 < nchunk ? 2u : 0u);
            hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, sp);
            EmitParams ep;
            ep.sender = d_sender + lo;
            ep.pos = d_pos ? d_pos + 3 * lo : nullptr;
            ep.repl = d_repl + lo;
            ep.M = (uint32_t)(hi - lo);
            ep.t = tv;
            ep.e = rw.e.as<uint32_t>() + lo;
            ep.tile_prefix = tile_prefix + t0;
            ep.count_tile = count_tile;
            ep.offsets = d_offsets + lo;
            ep.info = rw.info.as<uint2>() + lo;
            ep.peers = capacity ? d_peers : nullptr;
            ep.msgs = d_msgs;
            ep.capacity = capacity;
            ep.n_blocks = t1 - t0;
            ep.msg_base = (uint32_t)lo;
            hipLaunchKernelGGL((emit_map_kernel<16>), dim3(t1 - t0), dim3(kBlock), 0, s, ep);
            WQ_HIP(h, hipGetLastError());
        }
        if (pr.enabled) {
            WQ_HIP(h, hipEventRecord(pr.stop[pr.used], s));
            pr.used++;
        }
        rw.calls++;
        return WQ_OK;
    }

    CountParams cp;
    cp.in = in;
    cp.t = tv;
    cp.e = rw.e.as<uint32_t>();
    cp.info = rw.info.as<uint2>();
    cp.tile_total = tile_total;
    cp.tile_F = tile_F;
    cp.cnt = cur;
    cp.cnt_next = nxt;
    cp.health = route_health(h);
    if (radius)
        hipLaunchKernelGGL(count_radius_kernel<false>, dim3(n_count), dim3(kBlock), 0, s, cp);
    else
        {
        // two count tiles per block (grid stride): C3's 39,063 short blocks turn over less (with
        // two emit blocks per workgroup, 1,294-1,303 vs 1,320-1,328 us per tick on one box; 3 or 4
        // no better); a tick of a few rounds of resident blocks (an 8-GPU rank's replicated C3
        // slice: 4,883 tiles) is faster with one (212-213 vs 221-222 us, with one emit block per
        // workgroup too; 2.5M messages 383-384 vs 389-390). WQ_DEBUG_COUNT_TPB overrides (diagnostics)
        static const uint32_t tpb_env = getenv("WQ_DEBUG_COUNT_TPB") ? (uint32_t)std::max(1, atoi(getenv("WQ_DEBUG_COUNT_TPB"))) : 0u;
        const uint32_t tpb = tpb_env ? tpb_env : ((uint64_t)n_count * count_tile <= (uint64_t)kShortTickTiles * kBlock ? 1u : 2u);
        cp.n_tiles = n_count;
        cfg.count(cp, s, (n_count + tpb - 1) / tpb);
    }
    WQ_HIP(h, hipGetLastError());
    if (pr.enabled) WQ_HIP(h, hipEventRecord(pr.mid1[pr.used], s));

    TileScanParams sp;
    sp.tile_total = tile_total;
    sp.tile_F = tile_F;
    sp.tile_prefix = tile_prefix;
    sp.n_tiles = n_count;
    sp.offsets = d_offsets;
    sp.M = (uint32_t)M;
    sp.capacity = capacity;
    sp.cnt = cur;
    sp.health = route_health(h);
    sp.stale = tv.stale;
    sp.out = rw.out;
    if (int rc = launch_tile_scan(h, sp, nullptr, &rw.out_done)) return rc;
    if (pr.enabled) {
        WQ_HIP(h, hipEventRecord(pr.mid2[pr.used], s));
        pr.phased[pr.used] = 1;
    }

    EmitParams ep;
    ep.sender = d_sender;
    ep.pos = d_pos;
    ep.repl = d_repl;
    ep.M = (uint32_t)M;
    ep.t = tv;
    ep.e = rw.e.as<uint32_t>();
    ep.tile_prefix = tile_prefix;
    ep.count_tile = count_tile;
    ep.offsets = d_offsets;
    ep.info = rw.info.as<uint2>();
    ep.peers = capacity ? d_peers : nullptr;
    ep.msgs = d_msgs;
    ep.capacity = capacity;
    const dim3 eg((unsigned)((M + kBlock - 1) / kBlock));
    if (radius)
        hipLaunchKernelGGL((emit_kernel<4096, 2, true>), eg, dim3(kBlock), 0, s, ep);
    else if (cfg.emit_heavy == 16)
        hipLaunchKernelGGL((emit_heavy_kernel<16>), eg, dim3(kBlock), 0, s, ep);
    else if (cfg.emit_heavy == 8)
        hipLaunchKernelGGL((emit_heavy_kernel<8>), eg, dim3(kBlock), 0, s, ep);
    else if (cfg.emit_heavy == 116) {
        // diagnostics only: extra LDS per block caps the emit's blocks per CU (occupancy sweeps)
        static const size_t emit_lds = getenv("WQ_DEBUG_EMIT_LDS") ? strtoull(getenv("WQ_DEBUG_EMIT_LDS"), nullptr, 10) : 0;
        // two 256-message blocks per workgroup (grid stride, see the count above; one for a short
        // tick); WQ_DEBUG_EMIT_BPB overrides
        static const uint32_t bpb_env = getenv("WQ_DEBUG_EMIT_BPB") ? (uint32_t)std::max(1, atoi(getenv("WQ_DEBUG_EMIT_BPB"))) : 0u;
        const uint32_t bpb = bpb_env ? bpb_env : (eg.x <= kShortTickTiles ? 1u : 2u);
        ep.n_blocks = eg.x;
        hipLaunchKernelGGL((emit_map_kernel<16>), dim3((eg.x + bpb - 1) / bpb), dim3(kBlock), emit_lds, s, ep);
    }
    else if (cfg.emit_heavy == 108)
        hipLaunchKernelGGL((emit_map_kernel<8>), eg, dim3(kBlock), 0, s, ep);
    else if (cfg.emit_stage == 4096 + 2)
        hipLaunchKernelGGL((emit_kernel<4096, 2>), eg, dim3(kBlock), 0, s, ep);
    else if (cfg.emit_stage == 4096 + 4)
        hipLaunchKernelGGL((emit_kernel<4096, 4>), eg, dim3(kBlock), 0, s, ep);
    else
        hipLaunchKernelGGL((emit_kernel<4096, 8>), eg, dim3(kBlock), 0, s, ep);
    WQ_HIP(h, hipGetLastError());
    if (pr.enabled) {
        WQ_HIP(h, hipEventRecord(pr.stop[pr.used], s));
        pr.used++;
    }
    rw.calls++;
    return WQ_OK;
}

}  // namespace wq
