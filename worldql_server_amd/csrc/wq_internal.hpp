// wq_internal.hpp — host-side state of one router handle (one GPU, one owner thread).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/wq_router.h"
#include "wq_device.hpp"

namespace wq {

// wq_route_health error bit 16: a device op batch held an invalid op and was not applied.
constexpr uint32_t kErrBadBatch = 16u;

// Grow-only device buffer.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    // hipExtMallocWithFlags flags for the next allocation (0: hipMalloc); a flagged allocation that
    // fails falls back to hipMalloc
    unsigned flags = 0;
    bool flagged = false;  // the current allocation came from hipExtMallocWithFlags
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            bytes = 0;
        }
        size_t cap = need < 4096 ? 4096 : need + need / 4;
        hipError_t e = flags ? hipExtMallocWithFlags(&p, cap, flags) : hipMalloc(&p, cap);
        flagged = flags && e == hipSuccess;
        if (e != hipSuccess && flags) {
            (void)hipGetLastError();
            p = nullptr;
            e = hipMalloc(&p, cap);
        }
        if (e == hipSuccess) bytes = cap;
        return e;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// The live subscription set, sorted by (hash, world, key, peer): one entry per
// (world, cube, peer) triple. Everything the route kernel reads is derived from it.
struct State {
    DevBuf h, w, kx, ky, kz, p;  // u64, u32, i64 x3, u32
    uint64_t n = 0;
};

struct Table {
    DevBuf recs;      // Record[rec_cap]: regular cubes (wq_device.hpp), load <= 0.3
    DevBuf rclaim;    // u32[rec_cap] (build scratch)
    uint64_t rec_cap = 0;
    int rec_shift = 64;
    DevBuf slots;     // Slot[cap]: cubes without a packed key
    DevBuf claim;     // u32[cap] (build scratch)
    DevBuf list;      // u32 words: per cube [count, peers...] (+ room for relocated lists)
    DevBuf any;       // u64[n_any] sorted (world << 32 | peer)
    uint64_t cap = 0;
    int shift = 64;
    uint64_t n_cubes = 0, n_any = 0;
    // incremental updates (wq_delta.hip): list words in use (lists are bump-allocated past the
    // build's dense region when they outgrow their capacity) and record slots in use (including
    // records whose cube emptied: they keep their key, count 0)
    uint64_t list_used = 0, list_cap = 0, n_recs = 0;
    // per-peer boxes (wq_device.hpp PeerBox): kBoxWords words per peer, then the valid word
    DevBuf pbox;
    uint32_t n_pbox = 0;
    // u32: non-zero while the last incremental batch could not be applied on the device (the
    // next host call re-applies it); route kernels report error bit 8 meanwhile
    DevBuf stale;
    // dense record headers (TableView::hdr): 32 B per record slot, refreshed by every full build;
    // off (hdr_ok false) from the first in-place change until the next build
    DevBuf hdr;
    bool hdr_ok = false;
    // compact headers (round 6, default): their own open-addressed table at load <= 1/2 (hdr_cap
    // slots), each header's cap word replaced by its record slot; hdr_cap == 0: the round-4 layout
    // (header i = record i's first 32 bytes, WQ_HDR_COMPACT=0)
    uint64_t hdr_cap = 0;
    int hdr_shift = 64;
    uint32_t hdr_blk = 0;  // wq_device.hpp hdr_home (WQ_HDR_BLOCK)
};

// The last incremental batch (wq_delta.hip), in flight: its status and stat deltas arrive in
// pinned memory; the next host call folds them in (and re-applies the batch if it was not
// applied) — the update itself never waits for the GPU.
struct PendingDelta {
    bool active = false;
    hipEvent_t ev = nullptr;
    void* pinned = nullptr;     // DeltaStatus (32 B) + i64 {entries, live cubes} deltas
    const wq_op* ops = nullptr; // the batch (h->d_ops or the caller's device array)
    size_t n = 0;
    uint64_t list_room = 0;
};

// Scratch of the incremental update (wq_delta.hip).
struct DeltaWs {
    DevBuf part, summ;      // REMOVE_PEER per-block partial sums; a batch's DeltaStatus
    DevBuf dstat;           // i64 x2: entry / live-cube deltas of batches not yet read back
    DevBuf rm_bits;         // REMOVE_PEER from every world: bitmap over peer ids
    DevBuf sort_cnt;        // bucket sort: per (digit, tile) key counts, then their row prefixes
    DevBuf sort_tot;        // bucket sort: per digit key totals
};

// Route workspace, persistent across calls so a tick needs no memset: two counter slots (each
// call's count pass zeroes the next call's) and the per-message state the count pass hands to
// the scan and emit passes.
struct RouteWs {
    DevBuf buf;    // [pad 64][wq_route_counters x2]
    DevBuf info;   // uint2[M]: locators, count pass -> emit pass
    DevBuf e;      // u32[M]: filtered counts
    DevBuf tiles;  // u32[2 * n_count_blocks]: block totals, then their exclusive prefix
    DevBuf spill;  // per-block output images of the count+spill tick (route config 7)
    DevBuf agg;    // u64[2 * blocks]: look-back and candidate granules of the single-launch tick
    DevBuf scan_tmp;  // rocPRIM temporary storage of the many-tile scan (WQ_SCAN_MULTI=0)
    DevBuf sgran;     // u64[2 * blocks]: the multi-block tile scan's tagged block aggregates {E, F}
    uint64_t sgran_zeroed = 0;  // granules zeroed so far (a fresh one never matches a tag)
    uint64_t scan_calls = 0;    // multi-block scans so far (their tags)
    uint64_t agg_zeroed = 0;
    uint64_t* stamps = nullptr;  // wq_debug_set_timeline
    // the pipelined heavy tick (wq_route.hip, short ticks): count chunks on `side` while the launch
    // stream scans and emits the previous chunk; {P, F} carried across the chunks' scans
    hipStream_t side = nullptr;
    hipEvent_t ev_in = nullptr;
    std::vector<hipEvent_t> cev;
    DevBuf carry;
    uint64_t calls = 0;
    wq_route_counters* last = nullptr;  // counters of the most recent call (device)
    // wq_route_tick_device's caller counters: the three-launch tick's scan writes them itself when it
    // can (out_done), instead of a copy launch after the tick
    wq_route_counters* out = nullptr;
    bool out_done = false;
};

struct ProfileEvents {
    std::vector<hipEvent_t> start, stop;
    // the three-launch shape (count / tile scan / emit) also records an event after the count and
    // one after the scan, so wq_profile_read_phases can split a launch's time per kernel
    std::vector<hipEvent_t> mid1, mid2;
    std::vector<char> phased;
    size_t used = 0;
    bool enabled = false;
};

struct ShardCtx;  // wq_sharded.hip: the exchange a sharded tick uses, and its workspace
struct MultiCtx;  // wq_multi.hip: a handle over G GPUs (wq_router_create_multi)

}  // namespace wq

struct wq_router {
    int device = 0;
    uint16_t cube_size = 16;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    uint64_t hash_mask = ~0ull;
    uint32_t rec_slack = 8;  // record slots per cube at build (load <= 1/rec_slack)
    bool rec_slack_set = false;  // set by wq_debug_set_record_slack (then no footprint cap)
    uint64_t hash_fallbacks = 0;
    std::string err;

    wq::State st, st_next;
    wq::Table tab;
    // After incremental updates the sorted state `st` and the any-keys are stale; they are
    // regenerated from the records on demand (table_materialize / table_ensure_any).
    bool st_stale = false, any_stale = false;
    wq::DeltaWs dws;
    wq::PendingDelta pend;
    // incremental batches applied, batches that fell back to the rebuild, applied batches in which
    // some cube took the wave path (lists longer than kLaneList)
    uint64_t n_delta_applies = 0, n_delta_fallbacks = 0, n_delta_wave_batches = 0;
    uint64_t n_delta_batches = 0;  // batch tags of the record claims (wq_delta.hip)
    bool dstat_pending = false;
    // bumped by every change of the table (an op batch, a removal, a re-applied device batch):
    // results that point into the table (the slot tick's kept rows) are valid for one generation
    uint64_t table_gen = 0;

    // build scratch
    wq::DevBuf ev_h, ev_w, ev_kx, ev_ky, ev_kz, ev_p, ev_kind, d_ops;
    const wq_op* cur_ops = nullptr;  // the batch being applied (h->d_ops, or the caller's device array)
    wq::DevBuf idx_a, idx_b, key32_a, key32_b, key64_a, key64_b, flags, scan, sort_tmp, small;
    wq::DevBuf cube_id, cube_start;

    wq::RouteWs rws;
    // sharded ticks (wq_shard.hip): owner histograms, unpacked received records
    wq::DevBuf shard_hist, rec_keys, rec_w, rec_s, rec_r;
    // the one-pass slot grouping (wq_shard.hip slot_group_kernel): tagged look-back granules per
    // (owner, block), zeroed once per allocation (tag 0 never matches), and the launches so far
    wq::DevBuf shard_look;
    uint64_t shard_look_zeroed = 0, shard_look_calls = 0;
    int route_cfg = 0;  // route kernel shapes (wq_route.hip kCfgs)
    uint32_t route_chunks = 0;  // wq_debug_set_route_chunks: chunks of the pipelined heavy tick (0 = default)
    bool heavy_fanout = false;  // wq_set_fanout_hint: default shape -> kCfgHeavy
    bool fanout_auto = true;    // until wq_set_fanout_hint: wq_route_tick sets heavy_fanout from its P / M
    // host-pointer convenience buffers
    wq::DevBuf h_in, h_out;
    // C5 radius filter (wq_set_radius / wq_set_peer_positions)
    wq::DevBuf ppos;
    wq::DevBuf ppos4;  // f32 copy (float4 per peer) for the radius filter's second test
    wq::DevBuf pcode;  // 4-byte position codes (the first test) and their box (wq_device.hpp)
    wq::DevBuf qbox;   // u64 box keys [0, 6), then {lo, step} doubles [6, 12), the second box slot [12, 18)
    int qbox_phase = -1;  // the box slot the next wq_set_peer_positions accumulates into (-1: not reset yet)
    uint64_t n_ppos = 0;
    double radius = 0.0;
    wq::ProfileEvents prof;
    wq::ShardCtx* shard = nullptr;  // wq_shard_attach_*: this handle is one shard of G
    bool shard_expanded = false;    // wq_debug_set_shard_form: expanded pairs back instead of row references
    int shard_inject = 0;           // wq_debug_inject_shard_failure: fail the next sharded tick's step 1 or 3
    wq::MultiCtx* multi = nullptr;  // wq_router_create_multi: this handle drives G shard handles
};

namespace wq {
inline TableView table_view(const wq_router* h) {
    TableView v;
    v.recs = h->tab.recs.as<Record>();
    v.rec_mask = h->tab.rec_cap - 1;
    v.rec_shift = h->tab.rec_shift;
    v.slots = h->tab.slots.as<Slot>();
    v.slot_mask = h->tab.cap - 1;
    v.slot_shift = h->tab.shift;
    v.hash_mask = h->hash_mask;
    v.list = h->tab.list.as<uint32_t>();
    v.sf = (double)h->cube_size;
    v.ppos = h->ppos.as<double>();
    v.ppos4 = h->ppos4.as<float4>();
    v.pcode = h->n_ppos ? h->pcode.as<uint32_t>() : nullptr;
    v.qbox = h->qbox.p ? reinterpret_cast<const double*>(h->qbox.as<uint64_t>() + 6) : nullptr;
    v.n_ppos = (uint32_t)h->n_ppos;
    v.r2 = h->radius > 0.0 ? h->radius * h->radius : -1.0;
    v.n_pbox = h->tab.n_pbox;
    v.pbox = h->tab.n_pbox ? h->tab.pbox.as<uint32_t>() : nullptr;
    v.pbox_valid = h->tab.n_pbox ? h->tab.pbox.as<uint32_t>() + (uint64_t)kBoxWords * h->tab.n_pbox : nullptr;
    v.stale = h->tab.stale.as<uint32_t>();
    v.hdr = h->tab.hdr_ok ? h->tab.hdr.as<uint4>() : nullptr;
    v.hdr_mask = h->tab.hdr_cap ? h->tab.hdr_cap - 1 : 0;
    v.hdr_shift = h->tab.hdr_shift;
    v.hdr_blk = h->tab.hdr_blk;
    return v;
}
// Sticky {error OR, overflow OR} words of every route / global call since the last
// wq_route_health: the first 8 bytes of the route workspace (route_counters allocates it).
inline uint32_t* route_health(wq_router* h) { return h->rws.buf.as<uint32_t>(); }
// wq_route.hip
int route_config_count();
// 256-message tiles per block of a count or emit pass over `tiles` tiles: one for a short tick, two
// otherwise (the grid strides over the rest) — launch_route's shapes, shared with the sharded passes
uint32_t route_tiles_per_block(uint32_t tiles);
// The tick's counter slots (this call's, the next call's); *cur == nullptr when M == 0 (offsets[0]
// and both slots zeroed, nothing left to launch).
int route_counters(wq_router* h, size_t M, uint32_t* d_offsets, wq_route_counters** cur, wq_route_counters** nxt);
// wq_table.hip
// ops on the host (copied to h->d_ops) or, with on_device, a device array the batch is read from
// (validated on the device: no REMOVE_PEER, no reserved world id).
int table_apply_segment(wq_router* h, const wq_op* ops, size_t n, bool on_device = false);
// keys: sorted unique (world << 32 | peer); world == WQ_WORLD_INVALID removes the peer everywhere.
int table_remove_peers(wq_router* h, const uint64_t* keys_sorted_unique, size_t n);
int table_rebuild_derived(wq_router* h);
// wq_delta.hip. Applies n subscribe / unsubscribe ops (h->cur_ops) to the records and lists in
// place; *applied = false (and nothing changed) when the batch needs the full rebuild.
int table_apply_delta(wq_router* h, size_t n, bool* applied);
// REMOVE_PEER in place: keys sorted unique (world << 32 | peer), world WQ_WORLD_INVALID = every
// world; one pass over every cube's list (wq_delta.hip).
int table_remove_peers_inplace(wq_router* h, const uint64_t* keys, size_t n);
// Folds the device-side entry / live-cube deltas of incremental batches into st.n / tab.n_cubes
// (synchronises the stream).
int table_sync_delta_stats(wq_router* h);
// Folds in the in-flight incremental batch (blocking: waits for it; otherwise only if it has
// finished) and re-applies it through the rebuild if the device could not apply it.
int table_resolve(wq_router* h, bool blocking);
// Regenerates `st` (grouped by cube, peers ascending) from the records, slots and lists.
int table_materialize(wq_router* h);
// Rebuilds the any-keys if incremental updates left them stale.
int table_ensure_any(wq_router* h);
int set_error(wq_router* h, int code, const char* what, hipError_t e = hipSuccess);
// wq_sharded.hip: frees the exchange and its workspace (destroys an RCCL communicator).
void shard_release(wq_router* h);
// wq_multi.hip: the multi-GPU handle's side of the entry points (h->multi != nullptr)
int multi_merge_any(wq_router* h);
int multi_apply_ops(wq_router* h, const wq_op* ops, size_t n);
int multi_apply_ops_device(wq_router* h, const wq_op* d_ops, size_t n);
int multi_remove_peers(wq_router* h, const uint32_t* peers, size_t n);
int multi_route_tick(wq_router* h, const double* pos, const int64_t* keys, const uint32_t* world,
                     const uint32_t* sender, const uint8_t* repl, size_t M, uint32_t* offsets, uint32_t* peers,
                     uint32_t* msgs, size_t capacity, size_t* n_pairs, bool on_device);
int multi_route_slices(wq_router* h, const wq_msg_slice* in, int with_msgs, wq_slice_view* out);
int multi_is_subscribed(wq_router* h, size_t n, const uint32_t* world, const uint32_t* peer, int raw,
                        const void* kp, uint8_t* out);
int multi_stats(wq_router* h, wq_stats* out);
int multi_health(wq_router* h, uint32_t* error_bits, uint32_t* overflow);
int multi_set_positions(wq_router* h, const double* pos, size_t n, bool on_device);
int multi_set_radius(wq_router* h, double radius);
int multi_set_hint(wq_router* h, double pairs_per_message);
void multi_release(wq_router* h);
}  // namespace wq

#define WQ_HIP(h, call)                                                    \
    do {                                                                   \
        hipError_t e_ = (call);                                            \
        if (e_ != hipSuccess) return wq::set_error((h), WQ_E_HIP, #call, e_); \
    } while (0)

#define WQ_ALLOC(h, buf, bytes)                                                     \
    do {                                                                            \
        hipError_t e_ = (buf).ensure(bytes);                                        \
        if (e_ != hipSuccess) return wq::set_error((h), WQ_E_OOM, "hipMalloc " #buf, e_); \
    } while (0)
