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
//                   in parallel and reduced with lane shuffles. Writes the filtered count e_m,
//                   an 8-byte locator (record slot + count / list offset / "the sender itself",
//                   skipped index) and the block's total. No inter-block waits.
// 2. tile_scan      one block scans the block totals (C2: 1,954 values) -> tile_prefix[], P.
// 3. emit_kernel    CSR offsets = tile_prefix + a block-local scan of e_m, then the
//                   load-balanced expand + compaction (kernel 3): a tile stages its messages'
//                   inline peer lists in LDS (8 lanes per record line again; the table is
//                   Infinity-Cache resident since pass 1), marks each message's first output in
//                   an LDS owner array, max-scans it, and writes output j with thread j % 256 —
//                   one coalesced stream per tile whatever the fan-out skew.
// A single fused launch was measured first: its decoupled look-back made
// every tile wait for the slowest earlier tile's probes (p50 13 us, max 47 us per tile), capping
// it at 115-135 us per C2 tick. The split re-reads the record lines once and removes every wait.
// Output: CSR offsets[M+1] (message-major), peers[P], optional msgs[P].
#include <algorithm>

#include "route_count.hpp"
#include "route_emit.hpp"
#include "route_scan.hpp"

namespace wq {

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

template <int IPT, int MINW>
void launch_count(const CountParams& p, hipStream_t s, unsigned grid) {
    if (p.in.keys)
        hipLaunchKernelGGL((count_kernel<true, IPT, MINW>), dim3(grid), dim3(kBlock), 0, s, p);
    else
        hipLaunchKernelGGL((count_kernel<false, IPT, MINW>), dim3(grid), dim3(kBlock), 0, s, p);
}

template <int IPT, int STAGE, int U, int DBG = 0>
void launch_emit(const EmitParams& p, hipStream_t s, unsigned grid) {
    hipLaunchKernelGGL((emit_kernel<IPT, STAGE, U, DBG>), dim3(grid), dim3(kBlock), 0, s, p);
}

#define WQ_CFG(cipt, minw, eipt, stage, eu) \
    {cipt, eipt, &launch_count<cipt, minw>, &launch_emit<eipt, stage, eu>}
// count: (messages per lane, min waves per SIMD); emit: (messages per thread, window positions,
// record lines per lane in flight)
const Cfg kCfgs[] = {
    WQ_CFG(4, 2, 1, 4096, 8),  // 0: default
    WQ_CFG(4, 2, 1, 3072, 8),  // 1
    WQ_CFG(4, 2, 2, 6144, 8),  // 2
    WQ_CFG(2, 4, 1, 4096, 8),  // 3
    WQ_CFG(4, 2, 1, 2048, 8),  // 4
    WQ_CFG(4, 2, 1, 4096, 4),  // 5
    {4, 1, &launch_count<4, 2>, &launch_emit<1, 3072, 8, 1>},  // 6 timing only: no record loads
    {4, 1, &launch_count<4, 2>, &launch_emit<1, 3072, 8, 2>},  // 7 timing only: no output stores
    {4, 1, &launch_count<4, 2>, &launch_emit<1, 3072, 8, 4>},  // 8 timing only: no offset stores
    {4, 1, &launch_count<4, 2>, &launch_emit<1, 3072, 8, 7>},  // 9 timing only: none
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
    // workspace: [pad 64][counters x2 (32 B each)] — each call's count pass zeroes the next slot
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
    if (M == 0) {
        WQ_HIP(h, hipMemsetAsync(d_offsets, 0, 4, s));
        WQ_HIP(h, hipMemsetAsync(cur, 0, sizeof(wq_route_counters), s));
        WQ_HIP(h, hipMemsetAsync(nxt, 0, sizeof(wq_route_counters), s));
        rw.calls++;
        return WQ_OK;
    }
    const uint32_t count_tile = kBlock * cfg.count_ipt;
    const uint32_t n_count = (uint32_t)((M + count_tile - 1) / count_tile);
    WQ_ALLOC(h, rw.info, M * sizeof(uint2));
    WQ_ALLOC(h, rw.e, M * 4);
    WQ_ALLOC(h, rw.tiles, (uint64_t)n_count * 8);
    uint32_t* tile_total = rw.tiles.as<uint32_t>();
    uint32_t* tile_prefix = tile_total + n_count;

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
    cp.e = rw.e.as<uint32_t>();
    cp.info = rw.info.as<uint2>();
    cp.tile_total = tile_total;
    cp.cnt = cur;
    cp.cnt_next = nxt;
    cfg.count(cp, s, n_count);
    WQ_HIP(h, hipGetLastError());

    TileScanParams sp;
    sp.tile_total = tile_total;
    sp.tile_prefix = tile_prefix;
    sp.n_tiles = n_count;
    sp.offsets = d_offsets;
    sp.M = (uint32_t)M;
    sp.capacity = capacity;
    sp.cnt = cur;
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, sp);
    WQ_HIP(h, hipGetLastError());

    EmitParams ep;
    ep.sender = d_sender;
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
    const uint32_t emit_tile = kBlock * cfg.emit_ipt;
    cfg.emit(ep, s, (unsigned)((M + emit_tile - 1) / emit_tile));
    WQ_HIP(h, hipGetLastError());
    if (pr.enabled) {
        WQ_HIP(h, hipEventRecord(pr.stop[pr.used], s));
        pr.used++;
    }
    rw.calls++;
    return WQ_OK;
}

}  // namespace wq
