// wq_global.hip — GlobalMessage to a named world, on the same table.
//
// Replaces worldql_server/src/processing/global_message.rs:36-84: for a world that exists, the
// recipients are AreaMap::get_subscribed_any_peers (worldql_server/src/subscriptions/area_map.rs:65-67) — every peer holding at
// least one cube in that world — under the LocalMessage replication filter (ExceptSelf drops the
// sender, OnlySelf keeps only the sender, IncludingSelf keeps everyone). The "@global" broadcast
// (global_message.rs:18-35) goes to every connected peer, a PeerMap operation outside the table.
//
// The table keeps the sorted unique (world << 32 | peer) keys ("any-keys", wq_table.hip), so a
// world's peer set is one contiguous range of it. A tick of GlobalMessages is
//   count   one lane per message: two binary searches give the world's range and the sender's
//           rank inside it; e and a locator {range start, skipped rank};
//   scan    tile_scan_kernel over the 256-message tiles (route_scan.hpp);
//   offsets one block per tile: the tile prefix + an in-tile scan;
//   copy    the whole tick's outputs as one flat range over a persistent grid (owner by binary
//           search over the offsets), copied from the any-keys with coalesced loads and stores —
//           a world's range is contiguous, so even one message to a 50k-peer world is a streaming
//           copy spread over every CU.
#include "route_scan.hpp"
#include "wq_internal.hpp"

namespace wq {

namespace {

constexpr unsigned kCopyGrid = 2048;  // persistent copy grid: 8 blocks per CU

__device__ __forceinline__ uint64_t lower_bound_u64(const uint64_t* a, uint64_t n, uint64_t v) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t upper_bound_u64(const uint64_t* a, uint64_t n, uint64_t v) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] <= v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

struct GlobalParams {
    const uint32_t* world;
    const uint32_t* sender;
    const uint8_t* repl;
    uint32_t M;
    const uint64_t* any;
    uint64_t n_any;
    uint32_t* e;
    uint2* info;  // {first any-key index of the world, skipped rank or kNone} (OnlySelf: kLocSelf)
    uint32_t* tile_total;
    uint32_t* tile_F;
    uint32_t* tile_prefix;
    uint32_t* offsets;
    uint32_t* peers;
    uint32_t* msgs;
    uint64_t capacity;
    wq_route_counters* cnt_next;
};

__global__ __launch_bounds__(kBlock) void global_count_kernel(GlobalParams p) {
    __shared__ uint64_t wave_F[kWaves];
    __shared__ uint64_t wave_E[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (blockIdx.x == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    const uint32_t m = blockIdx.x * kBlock + tid;
    uint32_t e = 0, cnt = 0;
    uint2 info = make_uint2(0, kNone);
    if (m < p.M) {
        const uint64_t w = p.world[m], me = p.sender[m];
        const uint8_t rp = p.repl[m];
        // the world's range [lo, hi): hi is the upper bound of (w << 32) | 0xFFFFFFFF, which —
        // unlike (w + 1) << 32 — does not wrap for w = 0xFFFFFFFF (WQ_WORLD_INVALID: no keys, empty)
        const uint64_t lo = lower_bound_u64(p.any, p.n_any, w << 32);
        const uint64_t hi = upper_bound_u64(p.any, p.n_any, (w << 32) | 0xFFFFFFFFull);
        cnt = (uint32_t)(hi - lo);
        const uint64_t at = lower_bound_u64(p.any, p.n_any, (w << 32) | me);
        const bool has = at < hi && p.any[at] == ((w << 32) | me);
        if (rp == WQ_REPL_INCLUDING_SELF) {
            e = cnt;
            info = make_uint2((uint32_t)lo, kNone);
        } else if (rp == WQ_REPL_ONLY_SELF) {
            e = has ? 1u : 0u;
            info = make_uint2(kLocSelf, kNone);
        } else {  // ExceptSelf and unknown codes (replication.rs:40)
            e = cnt - (has ? 1u : 0u);
            info = make_uint2((uint32_t)lo, has ? (uint32_t)(at - lo) : kNone);
        }
        p.e[m] = e;
        p.info[m] = info;
    }
    const uint64_t Fw = wave_sum_u64(cnt);
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

// CSR offsets: the tile's prefix (tile_scan) + an in-tile exclusive scan of e.
__global__ __launch_bounds__(kBlock) void global_offsets_kernel(GlobalParams p) {
    __shared__ uint32_t s_wave[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t m = blockIdx.x * kBlock + tid;
    const uint32_t e = m < p.M ? p.e[m] : 0u;
    const uint32_t incl = wave_incl_scan_add(e, lane);
    if (lane == 63) s_wave[wave] = incl;
    lds_barrier();
    uint32_t before = 0;
#pragma unroll
    for (int u = 0; u < kWaves; ++u)
        if (u < wave) before += s_wave[u];
    if (m < p.M) p.offsets[m] = p.tile_prefix[blockIdx.x] + before + incl - e;
}

// The outputs as one flat range over a persistent grid: output k belongs to the last message whose
// offset is <= k (binary search over the offsets, L2-resident), and is copied from that world's
// contiguous any-key range — so one message to a 50k-peer world spreads over the whole GPU.
__global__ __launch_bounds__(kBlock) void global_copy_kernel(GlobalParams p) {
    const uint32_t P = p.offsets[p.M];
    const uint64_t lim = P < p.capacity ? P : p.capacity;
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < lim; k += (uint64_t)gridDim.x * kBlock) {
        uint32_t lo = 0, hi = p.M - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (p.offsets[mid] <= k)
                lo = mid;
            else
                hi = mid - 1;
        }
        const uint2 f = p.info[lo];
        const uint32_t oi = (uint32_t)k - p.offsets[lo];
        p.peers[k] = f.x == kLocSelf ? p.sender[lo] : (uint32_t)p.any[(uint64_t)f.x + oi + (oi >= f.y ? 1u : 0u)];
        if (p.msgs) p.msgs[k] = lo;
    }
}

}  // namespace

// wq_route_global(_device) body; wq_router.hip validates the arguments.
int launch_route_global(wq_router* h, const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                        size_t M, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    hipStream_t s = h->stream;
    RouteWs& rw = h->rws;
    wq_route_counters *cur, *nxt;
    int rc = route_counters(h, M, d_offsets, &cur, &nxt);
    if (rc || !cur) return rc;
    const uint32_t n_tiles = (uint32_t)((M + kBlock - 1) / kBlock);
    WQ_ALLOC(h, rw.info, M * sizeof(uint2));
    WQ_ALLOC(h, rw.e, M * 4);
    WQ_ALLOC(h, rw.tiles, (uint64_t)n_tiles * 12);
    GlobalParams gp;
    gp.world = d_world;
    gp.sender = d_sender;
    gp.repl = d_repl;
    gp.M = (uint32_t)M;
    gp.any = h->tab.any.as<uint64_t>();
    gp.n_any = h->tab.n_any;
    gp.e = rw.e.as<uint32_t>();
    gp.info = rw.info.as<uint2>();
    gp.tile_total = rw.tiles.as<uint32_t>();
    gp.tile_prefix = gp.tile_total + n_tiles;
    gp.tile_F = gp.tile_prefix + n_tiles;
    gp.offsets = d_offsets;
    gp.peers = capacity ? d_peers : nullptr;
    gp.msgs = d_msgs;
    gp.capacity = capacity;
    gp.cnt_next = nxt;
    hipLaunchKernelGGL(global_count_kernel, dim3(n_tiles), dim3(kBlock), 0, s, gp);
    WQ_HIP(h, hipGetLastError());
    TileScanParams sp;
    sp.tile_total = gp.tile_total;
    sp.tile_F = gp.tile_F;
    sp.tile_prefix = gp.tile_prefix;
    sp.n_tiles = n_tiles;
    sp.offsets = d_offsets;
    sp.M = (uint32_t)M;
    sp.capacity = capacity;
    sp.cnt = cur;
    sp.health = route_health(h);
    sp.stale = h->tab.stale.as<uint32_t>();
    if ((rc = launch_tile_scan(h, sp))) return rc;
    hipLaunchKernelGGL(global_offsets_kernel, dim3(n_tiles), dim3(kBlock), 0, s, gp);
    if (gp.peers) hipLaunchKernelGGL(global_copy_kernel, dim3(kCopyGrid), dim3(kBlock), 0, s, gp);
    WQ_HIP(h, hipGetLastError());
    rw.calls++;
    return WQ_OK;
}

}  // namespace wq
