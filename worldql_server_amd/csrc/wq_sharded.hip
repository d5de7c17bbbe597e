// wq_sharded.hip — the multi-GPU tick behind the C ABI (include/wq_router.h
// "multi-GPU: sharded ticks").
//
// The reference keeps ONE WorldMap owned by one task (worldql_server/src/processing/thread.rs:
// 113-148). Here G router handles — one per GPU, as threads of one process or one process per
// GPU — each own the (world, cube) buckets with shard_of(world, cube) == rank, and a tick of
// LocalMessages ingested anywhere is
//   1. shard    quantise, owner, group by owner into 40-byte records (wq_shard.hip kernels)
//   2. A2A      per-owner record counts (host read 1), then the records
//   3. route    the single-GPU count / scan / emit on what the owner received (wq_route.hip)
//   4. A2A      per-source pair counts (host read 2: the sizes the next exchange needs)
//   5. A2A      per-record recipient counts and the peers, back to the ingesting GPU (one group)
//   6. unshard  the CSR in the ingesting GPU's own message order: offsets[M+1], peers[P], msgs[P]
// so wq_sharded_route_tick_device returns exactly what wq_route_tick_device returns on one GPU
// holding the whole table (local_message.rs:52-86 per message, on the owner).
//
// Exchanges (all ordered on the handle's stream, segments contiguous in rank order):
//   RCCL      grouped ncclSend / ncclRecv over xGMI; librccl is loaded at run time (the copy a
//             PyTorch process already holds, else the system's), so the library has no link-time
//             RCCL dependency; the self segment is a device copy;
//   hub       G handles of ONE process (a server driving its GPUs from one thread each): a
//             barrier and peer copies (hipMemcpyPeerAsync over xGMI between GPUs);
//   callback  the caller's all-to-all (e.g. gloo in tests).
// Every wait is bounded; a rank whose local step fails still completes the tick's exchanges with
// consistent sizes (so no peer is left waiting) and reports the error at the end.
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <rccl/rccl.h>
#include <rocprim/rocprim.hpp>

#include "route_count.hpp"
#include "route_emit.hpp"
#include "route_gather.hpp"
#include "route_radius.hpp"
#include "route_scan.hpp"

namespace wq {
int launch_shard_messages(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                          const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, wq_msg_rec* d_out,
                          uint32_t* d_counts);
int launch_budget_slots(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                        const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, uint32_t me,
                        const SlotLayout& L, uint32_t* d_slots, uint32_t* d_perm, uint32_t* d_a, int phases,
                        bool hist_ready = false, bool own_too = false, uint32_t* own_slots = nullptr,
                        uint32_t* own_perm = nullptr, uint32_t* zero_e = nullptr, bool row_any = false,
                        uint32_t own_budget = 0xFFFFFFFFu, uint32_t* a_self = nullptr);
uint32_t budget_slot_tile();
int launch_route_records(wq_router* h, const wq_msg_rec* d_recs, size_t M, uint32_t* d_offsets, uint32_t* d_peers,
                         uint32_t* d_msgs, size_t capacity);
int launch_route(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                 const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                 uint32_t* d_peers, uint32_t* d_msgs, size_t capacity);
int launch_op_owner(wq_router* h, const wq_op* d_ops, size_t n, uint32_t G, uint32_t* d_owner);
}  // namespace wq

// ---------------------------------------------------------------------------------------------
// in-process hub
// ---------------------------------------------------------------------------------------------
struct wq_hub {
    uint32_t G = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t arrived = 0;
    uint64_t gen = 0;
    bool broken = false;  // a rank timed out: every later wait fails at once
    struct Post {
        const void* const* send = nullptr;  // per buffer
        const size_t* const* sbytes = nullptr;
        int n = 0;
        int device = 0;
        hipEvent_t ready = nullptr;  // the poster's send buffers are complete once this has fired
        hipEvent_t done = nullptr;   // the poster has finished reading its peers' send buffers
    };
    std::vector<Post> post;
    std::vector<uint32_t> attached;

    // Generation barrier, bounded: false on timeout (then the hub is broken for good).
    bool barrier(double timeout_s) {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == G) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::duration<double>(timeout_s),
                                    [&] { return gen != g || broken; });
        if (!ok || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

namespace wq {

// ---------------------------------------------------------------------------------------------
// RCCL, resolved at run time
// ---------------------------------------------------------------------------------------------
namespace {

struct RcclApi {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
    std::string why;
};

RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* lib = nullptr;
        const char* env = getenv("WQ_RCCL_LIBRARY");
        if (env && *env) lib = dlopen(env, RTLD_NOW | RTLD_LOCAL);
        // the copy a PyTorch-ROCm process has already loaded (one RCCL per process), else the system's
        const char* names[] = {"librccl.so", "librccl.so.1"};
        for (const char* n : names)
            if (!lib) lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
        for (const char* n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
            if (!lib) lib = dlopen(n, RTLD_NOW | RTLD_LOCAL);
        if (!lib) {
            api.why = std::string("librccl not found: ") + (dlerror() ? dlerror() : "");
            return;
        }
        api.GetUniqueId = reinterpret_cast<decltype(api.GetUniqueId)>(dlsym(lib, "ncclGetUniqueId"));
        api.CommInitRank = reinterpret_cast<decltype(api.CommInitRank)>(dlsym(lib, "ncclCommInitRank"));
        api.CommDestroy = reinterpret_cast<decltype(api.CommDestroy)>(dlsym(lib, "ncclCommDestroy"));
        api.Send = reinterpret_cast<decltype(api.Send)>(dlsym(lib, "ncclSend"));
        api.Recv = reinterpret_cast<decltype(api.Recv)>(dlsym(lib, "ncclRecv"));
        api.GroupStart = reinterpret_cast<decltype(api.GroupStart)>(dlsym(lib, "ncclGroupStart"));
        api.GroupEnd = reinterpret_cast<decltype(api.GroupEnd)>(dlsym(lib, "ncclGroupEnd"));
        api.GetErrorString = reinterpret_cast<decltype(api.GetErrorString)>(dlsym(lib, "ncclGetErrorString"));
        api.ok = api.GetUniqueId && api.CommInitRank && api.CommDestroy && api.Send && api.Recv && api.GroupStart &&
                 api.GroupEnd && api.GetErrorString;
        if (!api.ok) api.why = "librccl lacks ncclSend / ncclRecv / group calls";
    });
    return api;
}

constexpr int kXNone = 0, kXHub = 1, kXRccl = 2, kXCallback = 3;
constexpr double kHubTimeoutS = 120.0;
// (the small exchange vectors' layout, kSmall* / kCnt* / kStCodeMask: route_async.hpp)
// Blocks of a sharded count or emit pass over n tiles, shaped as launch_route's (WQ_DEBUG_SHARD_TPB:
// tiles per block, diagnostics)
inline uint32_t pass_blocks(uint32_t n) {
    static const uint32_t env = getenv("WQ_DEBUG_SHARD_TPB") ? (uint32_t)std::max(1, atoi(getenv("WQ_DEBUG_SHARD_TPB"))) : 0u;
    const uint32_t tpb = env ? env : route_tiles_per_block(n);
    return (n + tpb - 1) / tpb;
}

}  // namespace

// Record index bounds of each source shard's segment of the received records (kernel argument).
struct SegBounds {
    uint32_t b[WQ_MAX_SHARDS + 1];
};

// One exchange of n buffers: buffer k sends sbytes[k][d] bytes to rank d (segments contiguous in
// rank order from send[k]) and receives rbytes[k][s] from rank s into recv[k].
struct Xfer {
    const void* send[3];
    const size_t* sbytes[3];
    void* recv[3];
    const size_t* rbytes[3];
    int n;
    // buffer k's self segment is already in place in recv[k] (RCCL and hub exchanges only): not copied
    bool skip_self[3] = {false, false, false};
};

struct ShardCtx {
    uint32_t G = 1, rank = 0;
    int kind = kXNone;
    wq_hub* hub = nullptr;
    ncclComm_t comm = nullptr;
    wq_exchange_fn fn = nullptr;
    void* fn_ctx = nullptr;
    // workspace of the expanded-return tick (radius filter on) and the owner form
    DevBuf recs, recv, cnt2, pc, own_off, own_peers, own_e, ret_e, ret_off, ret_peers, by_msg, tmp, small;
    uint64_t own_cap = 0;
    std::vector<uint32_t> sc, rc;
    std::vector<uint64_t> ps, pr;
    // workspace of the slot tick (compact slots out, row references + cube-list pools back)
    DevBuf slots, perm, rslots, ocnt, hslot, plen, poff, claim, lead, ref_send, ref_recv, pool_send, pool_recv,
        desc_fill, e_msg, info_msg, mtiles, otiles, blk;
    // own slots (the default with G > 1, no radius): this shard's own messages as slots of a segment
    // that is never exchanged, its slot -> message map, and the scratch tile sums of their count
    DevBuf own_slots, own_perm, own_tiles;
    // which form the budgets above were derived from (0 the slot tick, 1 wq_sharded_route_owner_slots)
    int budget_form = 0;
    uint64_t claim_cap = 0;  // claim table entries (power of two); 0 = not allocated
    uint64_t ticks = 0;      // slot ticks run: the claim table's tag
    // exchange budgets of the slot tick, identical on both ends of every pair: slots me -> d and
    // s -> me (whole 256-slot blocks; 0 for this shard itself), pool words me -> s and o -> me. Set
    // from the previous tick's true sizes with headroom; without them (first tick, or after a tick
    // whose sizes outgrew them) the tick runs exact, reading the sizes back twice.
    std::vector<uint32_t> b1_out, b1_in;
    std::vector<uint64_t> b2_out, b2_in;
    bool budgets = false;
    uint64_t n_exact = 0, n_budget = 0;  // slot ticks of each kind (wq_shard_tick_stats)
    void* hsmall = nullptr;              // pinned copy of the small vectors at the end of a tick
    hipStream_t side = nullptr;          // the own-cube count pass, beside the exchanges
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_ready = nullptr, ev_done = nullptr;
    // bytes this shard sent to / received from OTHER shards in its latest tick (xGMI volume)
    uint64_t last_sent = 0, last_recv = 0;
    // the latest tick, kept for wq_sharded_copy_out after WQ_E_CAPACITY
    uint64_t last_M = 0, last_P = 0;
    bool last_ready = false;
    bool last_slots = false;  // the latest tick was a slot tick (copy_out = scan + emit of its rows)
    uint64_t last_gen = 0;    // its table generation: its own-cube rows point into the table
    const uint32_t* last_sender = nullptr;  // its d_sender (OnlySelf rows read the sender)
    const double* last_pos = nullptr;       // radius filter on: its positions and replication codes
    const uint8_t* last_repl = nullptr;     // (the emit re-filters list and pool rows)
    bool last_radius = false;
    // wq_sharded_route_tick_async: pinned snapshots of the small vectors of ticks not read back yet,
    // oldest first (a ring); every call drains them in the same order on every shard, so the budgets
    // derived from them stay identical on both ends of every pair
    // (mapped pinned memory the tick's last kernel writes itself, then a sequence word: no copy
    // launch and no event, each of which costs the stream a ~7 us bubble)
    static constexpr uint32_t kRing = 4;
    void* asnap[kRing] = {};
    uint64_t aseq[kRing] = {};  // the sequence number snapshot k completes with
    uint32_t ahead = 0, acount = 0;
    uint64_t n_async = 0;
    bool small_zeroed = false;  // the last tick's k_async_result left the small vectors zero
};

namespace {

std::vector<size_t> prefix(const size_t* b, uint32_t G) {
    std::vector<size_t> o(G + 1, 0);
    for (uint32_t i = 0; i < G; ++i) o[i + 1] = o[i] + b[i];
    return o;
}

int exchange(wq_router* h, const Xfer& x) {
    ShardCtx& sc = *h->shard;
    const uint32_t G = sc.G, me = sc.rank;
    hipStream_t s = h->stream;
    if (sc.kind == kXCallback) {
        for (int k = 0; k < x.n; ++k) {
            if (x.skip_self[k]) return set_error(h, WQ_E_INVALID, "exchange: the caller's callback copies every segment");
            const int rc = sc.fn(sc.fn_ctx, x.send[k], x.sbytes[k], x.recv[k], x.rbytes[k], (void*)s);
            if (rc) return set_error(h, WQ_E_RCCL, "the caller's exchange callback failed");
        }
        return WQ_OK;
    }
    if (sc.kind == kXRccl) {
        RcclApi& api = rccl();
        for (int k = 0; k < x.n; ++k) {  // the self segment: a device copy
            const auto so = prefix(x.sbytes[k], G), ro = prefix(x.rbytes[k], G);
            if (x.sbytes[k][me] != x.rbytes[k][me]) return set_error(h, WQ_E_INVALID, "self segment size mismatch");
            if (x.sbytes[k][me] && !x.skip_self[k])
                WQ_HIP(h, hipMemcpyAsync(static_cast<char*>(x.recv[k]) + ro[me],
                                         static_cast<const char*>(x.send[k]) + so[me], x.sbytes[k][me],
                                         hipMemcpyDeviceToDevice, s));
        }
        ncclResult_t r = api.GroupStart();
        for (int k = 0; k < x.n && r == ncclSuccess; ++k) {
            const auto so = prefix(x.sbytes[k], G), ro = prefix(x.rbytes[k], G);
            for (uint32_t p = 0; p < G && r == ncclSuccess; ++p) {
                if (p == me) continue;
                if (x.sbytes[k][p])
                    r = api.Send(static_cast<const char*>(x.send[k]) + so[p], x.sbytes[k][p], ncclUint8, (int)p,
                                 sc.comm, s);
                if (r == ncclSuccess && x.rbytes[k][p])
                    r = api.Recv(static_cast<char*>(x.recv[k]) + ro[p], x.rbytes[k][p], ncclUint8, (int)p, sc.comm,
                                 s);
            }
        }
        const ncclResult_t r2 = api.GroupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) {
            h->err = std::string("RCCL exchange: ") + api.GetErrorString(r);
            return WQ_E_RCCL;
        }
        return WQ_OK;
    }
    if (sc.kind == kXHub) {
        // No host wait on the GPU: each rank's send buffers are complete at its `ready` event, which
        // the readers' streams wait on before their peer copies; each reader records `done` after
        // them, and every rank's stream waits on all `done` events before it goes on (and may
        // overwrite a send buffer). The host threads only meet at the two barriers.
        wq_hub& hub = *sc.hub;
        WQ_HIP(h, hipEventRecord(sc.ev_ready, s));
        wq_hub::Post& mine = hub.post[me];
        mine.send = x.send;
        mine.sbytes = x.sbytes;
        mine.n = x.n;
        mine.device = h->device;
        mine.ready = sc.ev_ready;
        if (!hub.barrier(kHubTimeoutS)) return set_error(h, WQ_E_RCCL, "hub exchange: a peer never arrived");
        int rc = WQ_OK;
        for (uint32_t src = 0; src < G && rc == WQ_OK; ++src) {
            const wq_hub::Post& p = hub.post[src];
            if (p.n != x.n) {
                rc = set_error(h, WQ_E_INVALID, "hub exchange: ranks disagree on the buffer count");
                break;
            }
            if (src != me) {
                const hipError_t we = hipStreamWaitEvent(s, p.ready, 0);
                if (we != hipSuccess) {
                    rc = set_error(h, WQ_E_HIP, "hub exchange wait", we);
                    break;
                }
            }
            for (int k = 0; k < x.n; ++k) {
                const size_t bytes = p.sbytes[k][me];
                if (bytes != x.rbytes[k][src]) {
                    rc = set_error(h, WQ_E_INVALID, "hub exchange: send / receive sizes disagree");
                    break;
                }
                if (!bytes || (src == me && x.skip_self[k])) continue;
                size_t soff = 0, roff = 0;
                for (uint32_t d = 0; d < me; ++d) soff += p.sbytes[k][d];
                for (uint32_t q = 0; q < src; ++q) roff += x.rbytes[k][q];
                char* dst = static_cast<char*>(x.recv[k]) + roff;
                const char* from = static_cast<const char*>(p.send[k]) + soff;
                const hipError_t e = p.device == h->device
                                         ? hipMemcpyAsync(dst, from, bytes, hipMemcpyDeviceToDevice, s)
                                         : hipMemcpyPeerAsync(dst, h->device, from, p.device, bytes, s);
                if (e != hipSuccess) {
                    rc = set_error(h, WQ_E_HIP, "hub exchange copy", e);
                    break;
                }
            }
        }
        hipError_t e = hipEventRecord(sc.ev_done, s);  // done reading the peers' buffers ...
        mine.done = sc.ev_done;
        if (!hub.barrier(kHubTimeoutS))                  // ... before any of them reuses one
            return set_error(h, WQ_E_RCCL, "hub exchange: a peer never finished");
        for (uint32_t d = 0; d < G && e == hipSuccess; ++d)
            if (d != me) e = hipStreamWaitEvent(s, hub.post[d].done, 0);
        if (rc) return rc;
        if (e != hipSuccess) return set_error(h, WQ_E_HIP, "hub exchange events", e);
        return WQ_OK;
    }
    return set_error(h, WQ_E_INVALID, "no exchange attached");
}

// per received record: its recipient count; per source segment: {pair count, status}. A route that
// reported an error (counter bits: 4 spin, 2 > 2^32 pairs, 8 stale table) sends no pairs, and its
// status tells every source so, before any pair is exchanged.
__global__ void k_owner_counts(const uint32_t* __restrict__ off, uint32_t R, SegBounds seg, uint32_t G,
                               uint32_t* __restrict__ e, unsigned long long* __restrict__ pc,
                               const wq_route_counters* __restrict__ cnt, const uint32_t* __restrict__ stale) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < R) e[i] = off[i + 1] - off[i];
    if (blockIdx.x == 0 && threadIdx.x < G) {
        uint32_t err = cnt ? cnt->error : 0u;
        if (stale && *stale) err |= kErrStale;
        const uint32_t d = threadIdx.x;
        pc[2 * d] = err ? 0ull : (unsigned long long)(off[seg.b[d + 1]] - off[seg.b[d]]);
        pc[2 * d + 1] = (unsigned long long)err << 32;
    }
}

// counts in message order: by_msg[rec.msg] = e of the record (every message has one record)
__global__ void k_counts_by_msg(const wq_msg_rec* __restrict__ recs, const uint32_t* __restrict__ e, uint32_t M,
                                uint32_t* __restrict__ by_msg) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < M) by_msg[recs[i].msg] = e[i];
}

__global__ void k_set_last(uint32_t* __restrict__ a, uint32_t at, uint32_t v) { a[at] = v; }

// Block b moves the runs of records [256b, 256b + 256) — record i's e[i] peers at ret_off[i] in
// record order — to offsets[msg_i] in message order. Windows of W = R * 256 of the block's outputs:
// each record marks where its run enters the window in a u16 owner map (index + 1), a block-wide
// max-scan carries each owner over its outputs, and thread t moves outputs t, t + 256, ... of the
// window (contiguous reads; each run written contiguously at its message's offset). C3 on one
// shard: 1,059 us (about 5 GB moved: 4.7 TB/s), 1,088 us with an 8-step binary search over the
// run starts per output instead — the move is bandwidth-bound either way.
template <int R>
__global__ __launch_bounds__(kBlock) void k_unshard(const wq_msg_rec* __restrict__ recs, const uint32_t* __restrict__ ret_off,
                                                    const uint32_t* __restrict__ peers_in, uint32_t M, uint32_t P,
                                                    const uint32_t* __restrict__ offsets, uint32_t* __restrict__ peers,
                                                    uint32_t* __restrict__ msgs) {
    static_assert(R % 8 == 0, "map rows of whole 16-byte words");
    constexpr uint32_t W = R * kBlock;
    __shared__ alignas(16) uint16_t map[W];
    __shared__ uint32_t st[kBlock], dst[kBlock], msg[kBlock];
    __shared__ uint32_t wave_max[kWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t i0 = blockIdx.x * kBlock, i = i0 + tid;
    const uint32_t base = ret_off[i0];
    const uint32_t end = i0 + kBlock < M ? ret_off[i0 + kBlock] : P;
    const uint32_t T = end - base;
    uint32_t my_st = 0, my_e = 0;
    if (i < M) {
        const uint32_t m = recs[i].msg;
        const uint32_t a = ret_off[i];
        my_st = a - base;
        my_e = (i + 1 < M ? ret_off[i + 1] : P) - a;
        st[tid] = my_st;
        dst[tid] = offsets[m];
        msg[tid] = m;
    }
    uint4* my_map = reinterpret_cast<uint4*>(map) + tid * (R / 8);
    for (uint32_t w0 = 0; w0 < T; w0 += W) {
#pragma unroll
        for (int q = 0; q < R / 8; ++q) my_map[q] = make_uint4(0, 0, 0, 0);
        lds_barrier();
        if (my_e && my_st + my_e > w0 && my_st < w0 + W) map[(my_st > w0 ? my_st : w0) - w0] = (uint16_t)(tid + 1);
        lds_barrier();
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
        if (lane == 63) wave_max[wave] = incl;
        lds_barrier();
#pragma unroll
        for (int u = 0; u < kWaves; ++u)
            if (u < wave) pre = wave_max[u] > pre ? wave_max[u] : pre;
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
        const uint32_t last = (T - 1 - w0) < W - 1 ? (T - 1 - w0) : W - 1;
        uint32_t pv[R], oo[R], own[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t x = (uint32_t)(u * kBlock + tid) < last ? (uint32_t)(u * kBlock + tid) : last;
            const uint32_t j = (uint32_t)map[x] - 1u;
            const uint32_t r = w0 + x;
            pv[u] = peers_in[base + r];
            oo[u] = dst[j] + (r - st[j]);
            own[u] = j;
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (w0 + u * kBlock + tid < T) {
                peers[oo[u]] = pv[u];
                if (msgs) msgs[oo[u]] = msg[own[u]];
            }
        }
        lds_barrier();  // the next window rewrites the map
    }
}

int scan_excl(wq_router* h, DevBuf& tmp, const uint32_t* in, uint32_t* out, size_t n) {
    if (!n) return WQ_OK;
    // one launch (route_scan.hpp launch_scan_u32) up to 2^32 - 1 elements; WQ_SCAN_MULTI=0: rocPRIM
    static const bool multi = !getenv("WQ_SCAN_MULTI") || atoi(getenv("WQ_SCAN_MULTI")) != 0;
    if (multi && n < 0xFFFFFFFFull) return launch_scan_u32(h, in, out, (uint32_t)n, nullptr);
    size_t bytes = 0;
    WQ_HIP(h, rocprim::exclusive_scan(nullptr, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), h->stream));
    WQ_ALLOC(h, tmp, bytes);
    WQ_HIP(h, rocprim::exclusive_scan(tmp.p, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), h->stream));
    return WQ_OK;
}

// ---------------------------------------------------------------------------------------------
// the slot tick: compact slots to the owners, row references and cube-list pools back
// ---------------------------------------------------------------------------------------------
// What an owner returns per received slot (12 bytes, uint3 {x, y, z}): the message's recipients as
// a row of words — z = kind << 30 | skipped index (kRefSkipNone: none), y = the row's source length
// (OnlySelf: the recipient count, 0 or 1), x = where the source is:
//   POOL    word offset in the pool the owner ships to this source (remote owners only): each cube
//           a source's messages hit is shipped to it ONCE per tick, whatever the number of messages
//   LIST    the cube's list in this handle's table (an owner's own messages: nothing is copied)
//   INLINE  the record slot whose inline peers are the row (ditto)
//   SELF    the sender itself (OnlySelf, when subscribed), or an empty row
// The ingesting GPU turns every reference into a {len, skip, pointer} descriptor in message order
// and gathers the CSR with gather_rows_kernel (route_gather.hpp).
constexpr uint32_t kRefPool = 0, kRefList = 1, kRefInline = 2, kRefSelf = 3;
constexpr uint32_t kRefSkipNone = 0x3FFFFFFFu;
constexpr int kRefClaimTagBits = 26;  // claim words: tag << 38 | source << 32 | cube locator

// Largest s < G with sb.b[s] <= i (segments may be empty).
__device__ __forceinline__ uint32_t seg_find(const SegBounds& sb, uint32_t G, uint32_t i) {
    uint32_t lo = 0, hi = G;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sb.b[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

struct RefOwnerParams {
    const uint32_t* e;     // count pass: filtered recipients per received slot (remote slots)
    const uint2* info;     // count pass: locator per received slot (route_count.hpp finish_message)
    const uint32_t* list;
    const Record* recs;
    SegBounds rrem;        // the remote slots per source shard, in remote index (own segment empty)
    uint32_t G, n_rem;     // remote slots
    uint32_t self_lo, n_self;  // the own segment of the received slots (skipped)
    uint32_t tag;
    unsigned long long* claim;  // (cube, source) claims of this tick, open addressing
    uint32_t* lead;             // claim slot -> the remote slot that claimed it
    uint64_t cmask;
    uint32_t* cnt;         // per remote slot: the cube's peer count (OnlySelf: e)
    uint32_t* hslot;       // per remote slot: its claim slot
    uint32_t* plen;        // per remote slot: words it adds to its source's pool (n_rem + 1 entries)
    const uint32_t* poff;  // exclusive scan of plen
    uint3* ref_send;       // per remote slot: its reference
    uint4* desc_fill;      // pool rows: the claiming slot copies its cube's peers
};

__device__ __forceinline__ uint32_t slot_cnt(const uint2 inf, uint32_t e) {
    if (inf.x & kLocSelf) return e;
    // a list row: e is the count less the sender's entry when the row skips it (finish_message),
    // so no read of the list's count word is needed
    if (inf.x & kLocGlobal) return e + (inf.y != kNone ? 1u : 0u);
    return inf.y == kNone ? 0u : inf.y >> 24;  // inline record, or no subscriber at all
}

// (owner, remote slots) the cube's peer count and the claim of the slot's (source, cube) pair: the
// first claimer ships the cube's peers in that source's pool, the others point at them. The block's
// slots first meet in an LDS table, so each distinct pair of the block claims once in global memory:
// C3's hot cubes put thousands of a source's slots on one claim word, and device-scope atomics on
// one word serialise.
constexpr uint32_t kClaimLds = 2 * kBlock;  // LDS table slots (a block has at most kBlock keys)
constexpr unsigned long long kClaimEmpty = ~0ull;

__global__ __launch_bounds__(kBlock) void k_ref_claim(RefOwnerParams p) {
    __shared__ unsigned long long lkey[kClaimLds];
    __shared__ uint32_t lres[kClaimLds];  // the pair's claim slot | leader bit 31 (set by its representative)
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    for (uint32_t k = threadIdx.x; k < kClaimLds; k += kBlock) lkey[k] = kClaimEmpty;
    if (t == p.n_rem) p.plen[t] = 0;
    const bool live = t < p.n_rem;
    const uint32_t i = t < p.self_lo ? t : t + p.n_self;  // the received slot
    uint2 inf = make_uint2(kLocSelf, kNone);
    uint32_t cnt = 0, s = 0;
    if (live) {
        s = seg_find(p.rrem, p.G, t);
        inf = p.info[i];
        cnt = slot_cnt(inf, p.e[i]);
    }
    const bool claims = live && !(inf.x & kLocSelf) && cnt;
    const unsigned long long pair = ((unsigned long long)s << 32) | inf.x;  // s < G: never kClaimEmpty
    __syncthreads();
    // the block's table: the thread that inserts a pair represents it
    bool rep = false;
    uint32_t lh = 0;
    if (claims) {
        uint64_t hv = pair * 0x9E3779B97F4A7C15ull;
        lh = (uint32_t)(hv >> 40) & (kClaimLds - 1);
        for (;;) {
            const unsigned long long old = atomicCAS(&lkey[lh], kClaimEmpty, pair);
            if (old == kClaimEmpty) {
                rep = true;
                break;
            }
            if (old == pair) break;
            lh = (lh + 1) & (kClaimLds - 1);
        }
    }
    uint64_t hs = 0;
    if (rep) {
        const unsigned long long key = ((unsigned long long)p.tag << 38) | pair;
        uint64_t hv = ((uint64_t)inf.x | ((uint64_t)s << 32)) * 0x9E3779B97F4A7C15ull;
        hv ^= hv >> 29;
        hs = hv & p.cmask;
        bool leader = false;
        for (;;) {
            unsigned long long v = __hip_atomic_load(p.claim + hs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((v >> 38) != p.tag) {  // a previous tick's word: free
                const unsigned long long old = atomicCAS(p.claim + hs, v, key);
                if (old == v) {
                    leader = true;
                    break;
                }
                v = old;
            }
            if (v == key) break;
            if ((v >> 38) == p.tag) hs = (hs + 1) & p.cmask;
        }
        if (leader) p.lead[hs] = t;
        lres[lh] = (uint32_t)hs | (leader ? 0x80000000u : 0u);
    }
    __syncthreads();
    if (!live) return;
    bool leader = false;
    if (claims) {
        const uint32_t r = lres[lh];
        hs = r & 0x7FFFFFFFu;
        leader = rep && (r >> 31);
    }
    p.cnt[t] = cnt;
    p.hslot[t] = (uint32_t)hs;
    p.plen[t] = leader ? cnt : 0u;
}

// The row of a slot from its count-pass locator: kind, source offset (list word / record slot) and
// skipped index (local_message.rs:60-86 as finish_message encoded it).
__device__ __forceinline__ void slot_row(const uint2 inf, uint32_t* kind, uint32_t* off, uint32_t* skip) {
    *kind = kRefSelf;
    *off = 0;
    *skip = kRefSkipNone;
    if (inf.x & kLocSelf) return;
    if (inf.x & kLocGlobal) {
        *kind = kRefList;
        *off = (inf.x & ~kLocGlobal) + 1;
        *skip = inf.y == kNone ? kRefSkipNone : inf.y;
    } else if (inf.y != kNone) {
        *kind = kRefInline;
        *off = inf.x;
        const uint32_t s24 = inf.y & kSkipNone24;
        *skip = s24 == kSkipNone24 ? kRefSkipNone : s24;
    }  // else: no subscriber — an empty SELF row
}

__device__ __forceinline__ const uint32_t* row_src(uint32_t kind, uint32_t off, const uint32_t* list, const Record* recs) {
    return kind == kRefList ? list + off : reinterpret_cast<const uint32_t*>(recs) + ((uint64_t)off * 32 + kInlineWord0);
}

// (owner, remote slots) a remote source's slot becomes its reference into the source's pool and,
// for the claiming slot, the pool row copying its cube's peers.
__global__ __launch_bounds__(kBlock) void k_ref_make(RefOwnerParams p) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= p.n_rem) return;
    const uint32_t i = t < p.self_lo ? t : t + p.n_self;  // the received slot
    const uint32_t s = seg_find(p.rrem, p.G, t);
    uint32_t kind, off, skip;
    slot_row(p.info[i], &kind, &off, &skip);
    const uint32_t cnt = p.cnt[t];
    uint3 ref;
    if (kind == kRefList || kind == kRefInline) {
        const uint32_t j = p.lead[p.hslot[t]];
        ref = make_uint3(p.poff[j] - p.poff[p.rrem.b[s]], cnt, (kRefPool << 30) | skip);
        if (j == t) {
            const uint64_t a = reinterpret_cast<uint64_t>(row_src(kind, off, p.list, p.recs));
            p.desc_fill[t] = make_uint4(cnt, kNone, (uint32_t)a, (uint32_t)(a >> 32));
        }
    } else {
        ref = make_uint3(0, cnt, (kRefSelf << 30) | kRefSkipNone);
    }
    p.ref_send[t] = ref;
}

// (owner) the C vector of the pool-size exchange, per source d: {pool words for d, status}. The
// status carries the owner's device error bits (8: stale table, plus its count pass's bits) and the
// budget bit when this shard knows of ANY budget that was too small — its own slot segments (A
// sent), any source's (A received: every shard receives every A vector), or its own pools here — so
// after the exchange every shard knows the same: redo the tick exactly, or not.
struct CVecParams {
    const uint32_t* a_send;  // 2G words
    const uint32_t* a_recv;  // 2G words
    const uint32_t* poff;    // nullable: no remote slots
    SegBounds rb;            // the receive layout's segments (remote slot index per source)
    uint64_t b2[WQ_MAX_SHARDS];  // pool word budgets me -> d (~0: no budget, the exact pass)
    uint32_t G;
    const uint32_t* stale;
    const wq_route_counters* cnt;  // the owner count pass's counters (nullable)
    uint32_t* c_send;        // out: 2G words
};

__global__ void k_c_vector(CVecParams p) {
    const uint32_t d = threadIdx.x;
    const bool in = d < p.G;
    uint32_t pool = 0;
    bool over = false;
    if (in) {
        pool = p.poff ? p.poff[p.rb.b[d + 1]] - p.poff[p.rb.b[d]] : 0u;
        over = (uint64_t)pool > p.b2[d] || (p.a_send[2 * d + 1] & kStBudget) || (p.a_recv[2 * d + 1] & kStBudget);
    }
    const bool any_over = __any(over);
    uint32_t bits = (p.stale && *p.stale) ? kErrStale : 0u;
    if (p.cnt) bits |= p.cnt->error;
    if (in) {
        p.c_send[2 * d] = pool;
        p.c_send[2 * d + 1] = ((bits & 0xFFFFu) << 8) | (any_over ? kStBudget : 0u);
    }
}

// (owner) per 256-slot block of the receive layout (segments are whole blocks): where its pool rows
// go in the send buffer (the source's budgeted segment) and where that segment ends.
struct PoolBlocksParams {
    const uint32_t* poff;
    SegBounds rb;
    uint64_t pb[WQ_MAX_SHARDS + 1];  // pool segment bases (words) in the send buffer
    uint32_t G, nblk;
    uint64_t* base;
    uint64_t* lim;
};

__global__ void k_pool_blocks(PoolBlocksParams p) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= p.nblk) return;
    const uint32_t i0 = b * kBlock;
    const uint32_t s = seg_find(p.rb, p.G, i0);
    p.base[b] = p.pb[s] + (p.poff[i0] - p.poff[p.rb.b[s]]);
    p.lim[b] = p.pb[s + 1];
}

// (ingesting GPU) the row of every slot it sent, from its owner's reference: e and the locator in
// message order (emit_map_kernel's info: a pool row as kLocPool | word offset into the received
// pools). A reference that does not lie inside its owner's pool segment — an owner that failed, or
// a tick whose budgets were too small (both reported after the tick) — routes to nobody, so no
// kernel ever reads outside the pools.
struct ResolveParams {
    const uint32_t* perm;     // sent slot -> message (kNone: tails, padding)
    const uint3* ref_recv;    // references, in the send layout
    SegBounds sb;             // the send layout's segments (slot index per owner)
    uint32_t G, n;            // n = slots in the send layout
    uint64_t prb[WQ_MAX_SHARDS + 1];  // pool segment bases (words) in the receive buffer
    uint32_t* e_msg;
    uint2* info_msg;
    // RADIUS: the pool rows are filtered here, where the message positions and every peer's position
    // are (the owner has neither the message position nor a reason to need it)
    const uint32_t* pool = nullptr;
    const double* pos = nullptr;
    const uint32_t* sender = nullptr;
    const uint8_t* repl = nullptr;
    TableView tv{};
};

// RADIUS: a pool row keeps its full length (the emit re-filters it, as count_radius_kernel's list
// rows) and e counts the candidates within the radius that replication keeps; an OnlySelf row the
// sender, if subscribed and within the radius of its own message.
template <bool RADIUS>
__global__ __launch_bounds__(kBlock) void k_ref_resolve(ResolveParams p) {
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= p.n) return;
    const uint32_t m = p.perm[k];
    if (m == kNone) return;
    const uint3 ref = p.ref_recv[k];
    const uint32_t kind = ref.z >> 30, sk = ref.z & kRefSkipNone;
    if (kind == kRefSelf) {  // OnlySelf: the sender when subscribed (y = 0 or 1), or an empty row
        uint32_t e = ref.y <= 1u ? ref.y : 0u;
        if (RADIUS && e) {
            const uint32_t me = p.sender[m];
            e = within_radius(p.tv, p.pos[3ull * m], p.pos[3ull * m + 1], p.pos[3ull * m + 2], me) ? 1u : 0u;
        }
        p.e_msg[m] = e;
        p.info_msg[m] = make_uint2(kLocSelf, kNone);
        return;
    }
    const uint32_t o = seg_find(p.sb, p.G, k);
    const uint64_t at = p.prb[o] + ref.x;
    const uint32_t skip = sk == kRefSkipNone ? kNone : sk;
    const bool ok = kind == kRefPool && at + ref.y <= p.prb[o + 1] && ref.y && (skip == kNone || skip < ref.y);
    if (RADIUS) {
        uint32_t e = 0, mask = 0;
        const uint32_t len = ref.y;
        if (ok) {
            const uint32_t me = p.sender[m];
            const uint8_t rp = p.repl[m];
            const double mx = p.pos[3ull * m], my = p.pos[3ull * m + 1], mz = p.pos[3ull * m + 2];
            const uint32_t* row = p.pool + at;
            for (uint32_t i = 0; i < len; ++i) {
                const uint32_t q = row[i];
                const bool keep = repl_keeps(rp, q, me) && within_radius(p.tv, mx, my, mz, q);
                e += keep ? 1u : 0u;
                if (keep && i < (uint32_t)kInline) mask |= 1u << i;
            }
        }
        p.e_msg[m] = e;
        // a short row carries its survivor mask (staged like an inline record's, kPoolShort), a long
        // one its length (re-filtered by the emit)
        p.info_msg[m] = !e ? make_uint2(0, kNone)
                       : len <= (uint32_t)kInline ? make_uint2(kLocPool | (uint32_t)at, kPoolShort | (len << 24) | mask)
                                                  : make_uint2(kLocPool | (uint32_t)at, len);
        return;
    }
    p.e_msg[m] = ok ? ref.y - (skip != kNone ? 1u : 0u) : 0u;
    p.info_msg[m] = ok ? make_uint2(kLocPool | (uint32_t)at, skip) : make_uint2(0, kNone);
}

// (ingesting GPU, G > 1, no radius) the own-cube count and the slot grouping's owner histogram in
// ONE pass over the messages (both quantise every message): block b takes the kHistTiles count
// tiles of histogram tile b (launch_budget_slots' 4 x 256 messages), counts its own cubes' messages
// as count_kernel<OWN> does, and adds every other message's slot weight (2 for an unpacked key) to
// its owner's column, hist[d * nblk + b], as slot_count_kernel would.
constexpr uint32_t kHistTiles = 4;

template <bool RAW>
__global__ __launch_bounds__(kBlock, 8) void own_count_hist_kernel(CountParams p, uint32_t nblk,
                                                                   uint32_t* __restrict__ hist) {
    __shared__ uint64_t wave_F[kWaves];
    __shared__ uint64_t wave_E[kWaves];
    __shared__ uint32_t hcnt[WQ_MAX_SHARDS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t G = p.in.own_G;
    for (uint32_t d = tid; d < G; d += kBlock) hcnt[d] = 0;
    if (blockIdx.x == 0 && tid == 0) {
        p.cnt_next->n_pairs = 0;
        p.cnt_next->n_candidates = 0;
        p.cnt_next->overflow = 0;
        p.cnt_next->error = 0;
    }
    __syncthreads();
    for (uint32_t k = 0; k < kHistTiles; ++k) {
        const uint32_t blk = blockIdx.x * kHistTiles + k;  // block-uniform
        if (blk >= p.n_tiles) break;
        const uint32_t m0 = blk * kBlock, m = m0 + tid;
        uint64_t F_local = 0;
        uint32_t E_local = 0;
        uint32_t e_out[1], own[1];
        uint2 inf_out[1];
        count_rows<RAW, 1, 0, false, false, true>(p.in, p.t, m0, e_out, inf_out, F_local, E_local, nullptr, own);
        if (m < p.in.M) {
            p.e[m] = e_out[0];
            p.info[m] = inf_out[0];
        }
        // the other shards' messages, one LDS add per distinct owner in the wave
        const uint32_t ow = own[0] & 0x7FFFFFFFu;
        const bool rem = m < p.in.M && ow != p.in.own_me;
        const uint64_t wide = __ballot(rem && (own[0] >> 31));
        uint64_t todo = __ballot(rem);
        while (todo) {
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const uint32_t d = __shfl(ow, leader, 64);
            const uint64_t mask = __ballot(rem && ow == d);
            if (lane == leader) atomicAdd(&hcnt[d], (uint32_t)(__popcll(mask) + __popcll(mask & wide)));
            todo &= ~mask;
        }
        const uint64_t Fw = wave_sum_u64(F_local);
        const uint64_t Ew = wave_sum_u64(E_local);
        if (lane == 0) {
            wave_F[wave] = Fw;
            wave_E[wave] = Ew;
        }
        __syncthreads();
        if (tid == 0) {
            uint64_t Fb = 0, Eb = 0;
#pragma unroll
            for (int u = 0; u < kWaves; ++u) {
                Fb += wave_F[u];
                Eb += wave_E[u];
            }
            p.tile_F[blk] = Fb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Fb;
            p.tile_total[blk] = Eb > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Eb;
            if (Eb > 0xFFFFFFFFull) flag_route(p.cnt, p.health, 2u, 0u);
        }
        __syncthreads();  // the next tile rewrites wave_F / wave_E
    }
    for (uint32_t d = tid; d < G; d += kBlock) hist[(uint64_t)d * nblk + blockIdx.x] = hcnt[d];
}

int attach(wq_router* h, uint32_t G, uint32_t rank) {
    if (!h || G == 0 || G > WQ_MAX_SHARDS || rank >= G) return WQ_E_INVALID;
    if (h->shard) return set_error(h, WQ_E_INVALID, "an exchange is already attached (wq_shard_detach first)");
    h->shard = new (std::nothrow) ShardCtx();
    if (!h->shard) return WQ_E_OOM;
    ShardCtx& sc = *h->shard;
    sc.G = G;
    sc.rank = rank;
    // the small exchange vectors live here for the handle's whole attachment: a tick never has to
    // allocate before its first exchange
    bool ok = sc.small.ensure(kSmallBytes) == hipSuccess &&
              hipHostMalloc(&sc.hsmall, kSmallBytes, hipHostMallocDefault) == hipSuccess &&
              hipStreamCreateWithFlags(&sc.side, hipStreamNonBlocking) == hipSuccess;
    // the hub's events order peer copies (system scope); the side stream's fork / join only work on
    // this device: a device-scope release is enough there
    for (hipEvent_t* e : {&sc.ev_ready, &sc.ev_done})
        ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
    for (hipEvent_t* e : {&sc.ev_fork, &sc.ev_join})
        ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventReleaseToDevice) == hipSuccess;
    for (uint32_t k = 0; k < ShardCtx::kRing; ++k) {
        ok = ok && hipHostMalloc(&sc.asnap[k], kSmallBytes + 64, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess;
        if (ok) memset(sc.asnap[k], 0, kSmallBytes + 64);
    }
    if (!ok) {
        shard_release(h);
        return set_error(h, WQ_E_OOM, "shard exchange vectors / stream / events");
    }
    sc.b1_out.assign(G, 0);
    sc.b1_in.assign(G, 0);
    sc.b2_out.assign(G, 0);
    sc.b2_in.assign(G, 0);
    return WQ_OK;
}

// The slot tick's CSR from its rows in message order (e_msg, info_msg; per-256-message totals in
// mtiles): the tile scan (offsets[M] = P, the counters at kCntScan: P, the overflow / error bits),
// then emit_map_kernel — rows of this shard's own cubes read the table, the others the pools
// received (outputs beyond capacity are not written).
int slots_copy_out(wq_router* h, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity,
                   const AsyncResultParams* ar = nullptr, bool* ar_done = nullptr) {
    ShardCtx& sc = *h->shard;
    const uint64_t M = sc.last_M;
    hipStream_t s = h->stream;
    wq_route_counters* cnt = reinterpret_cast<wq_route_counters*>(sc.small.as<char>() + kSmallCnt) + kCntScan;
    if (M == 0) {
        WQ_HIP(h, hipMemsetAsync(cnt, 0, sizeof(*cnt), s));
        WQ_HIP(h, hipMemsetAsync(d_offsets, 0, 4, s));
        return WQ_OK;
    }
    const uint32_t nt = (uint32_t)((M + kBlock - 1) / kBlock);
    uint32_t* tile_total = sc.mtiles.as<uint32_t>();
    uint32_t* tile_prefix = tile_total + nt;
    TileScanParams tp;
    tp.tile_total = tile_total;
    tp.tile_F = tile_total;  // F is reported as P on this path
    tp.tile_prefix = tile_prefix;
    tp.n_tiles = nt;
    tp.offsets = d_offsets;
    tp.M = (uint32_t)M;
    tp.capacity = capacity;
    tp.cnt = cnt;
    tp.health = h->rws.buf.p ? route_health(h) : nullptr;
    tp.stale = h->tab.stale.as<uint32_t>();  // error bit 8: the table still misses a device batch
    if (ar) {  // an asynchronous tick: the scan ends it (if it is the one-block scan)
        tp.ar = *ar;
        tp.async_end = true;
    }
    if (int rc = launch_tile_scan(h, tp, ar_done)) return rc;
    EmitParams ep;
    ep.sender = sc.last_sender;
    ep.pos = sc.last_radius ? sc.last_pos : nullptr;
    ep.repl = sc.last_radius ? sc.last_repl : nullptr;
    ep.M = (uint32_t)M;
    ep.t = table_view(h);
    ep.e = sc.e_msg.as<uint32_t>();
    ep.tile_prefix = tile_prefix;
    ep.count_tile = kBlock;
    ep.offsets = d_offsets;
    ep.info = sc.info_msg.as<uint2>();
    ep.peers = capacity ? d_peers : nullptr;
    ep.msgs = d_msgs;
    ep.capacity = capacity;
    ep.n_blocks = nt;
    ep.pool = sc.G > 1 ? sc.pool_recv.as<uint32_t>() : nullptr;  // pool rows (kLocPool) only at G > 1
    if (sc.last_radius)  // the radius filter's emit: masks of inline rows, list and pool rows re-filtered
        hipLaunchKernelGGL((emit_kernel<4096, 2, true>), dim3(nt), dim3(kBlock), 0, s, ep);
    else
        hipLaunchKernelGGL((emit_map_kernel<16>), dim3(pass_blocks(nt)), dim3(kBlock), 0, s, ep);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

// Unshard the latest tick into the caller's buffers (message order).
int copy_out(wq_router* h, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    ShardCtx& sc = *h->shard;
    sc.small_zeroed = false;  // the scan rewrites the counters in the small vectors
    const uint64_t M = sc.last_M, P = sc.last_P;
    hipStream_t s = h->stream;
    if (sc.last_slots) {
        // the kept rows of this shard's own cubes point into the table: only while it is unchanged
        if (h->table_gen != sc.last_gen)
            return set_error(h, WQ_E_INVALID, "sharded copy-out: the table changed since the tick (route again)");
        if (int rc = slots_copy_out(h, d_offsets, d_peers, d_msgs, capacity)) return rc;
        if (P > capacity) return set_error(h, WQ_E_CAPACITY, "sharded tick: output capacity too small (required size in *n_pairs)");
        return WQ_OK;
    }
    if (M) {
        WQ_ALLOC(h, sc.by_msg, M * 4);
        const unsigned g = (unsigned)((M + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(k_counts_by_msg, dim3(g), dim3(kBlock), 0, s, sc.recs.as<wq_msg_rec>(),
                           sc.ret_e.as<uint32_t>(), (uint32_t)M, sc.by_msg.as<uint32_t>());
        WQ_HIP(h, hipGetLastError());
        int rc = scan_excl(h, sc.tmp, sc.by_msg.as<uint32_t>(), d_offsets, M);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(k_set_last, dim3(1), dim3(1), 0, s, d_offsets, (uint32_t)M, (uint32_t)P);
    WQ_HIP(h, hipGetLastError());
    if (P > capacity) return set_error(h, WQ_E_CAPACITY, "sharded tick: output capacity too small (required size in *n_pairs)");
    if (M && P) {
        const unsigned g = (unsigned)((M + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(k_unshard<16>, dim3(g), dim3(kBlock), 0, s, sc.recs.as<wq_msg_rec>(), sc.ret_off.as<uint32_t>(),
                           sc.ret_peers.as<uint32_t>(), (uint32_t)M, (uint32_t)P, d_offsets, d_peers, d_msgs);
        WQ_HIP(h, hipGetLastError());
    }
    return WQ_OK;
}

}  // namespace

void shard_release(wq_router* h) {
    if (!h->shard) return;
    ShardCtx* sc = h->shard;
    if (sc->kind == kXRccl && sc->comm) (void)rccl().CommDestroy(sc->comm);
    if (sc->side) (void)hipStreamSynchronize(sc->side);
    DevBuf* bufs[] = {&sc->recs,     &sc->recv,      &sc->cnt2,      &sc->pc,        &sc->own_off,  &sc->own_peers,
                      &sc->own_e,    &sc->ret_e,     &sc->ret_off,   &sc->ret_peers, &sc->by_msg,   &sc->tmp,
                      &sc->small,    &sc->slots,     &sc->perm,      &sc->rslots,    &sc->ocnt,     &sc->hslot,
                      &sc->plen,     &sc->poff,      &sc->claim,     &sc->lead,      &sc->ref_send, &sc->ref_recv,
                      &sc->pool_send, &sc->pool_recv, &sc->desc_fill, &sc->e_msg,    &sc->info_msg, &sc->mtiles,
                      &sc->otiles,   &sc->blk,       &sc->own_slots, &sc->own_perm, &sc->own_tiles};
    for (DevBuf* b : bufs) b->release();
    if (sc->hsmall) (void)hipHostFree(sc->hsmall);
    for (uint32_t k = 0; k < ShardCtx::kRing; ++k)
        if (sc->asnap[k]) (void)hipHostFree(sc->asnap[k]);
    if (sc->side) (void)hipStreamDestroy(sc->side);
    for (hipEvent_t e : {sc->ev_fork, sc->ev_join, sc->ev_ready, sc->ev_done})
        if (e) (void)hipEventDestroy(e);
    delete sc;
    h->shard = nullptr;
}

}  // namespace wq

using namespace wq;

extern "C" {

int wq_hub_create(uint32_t n_shards, wq_hub** out) {
    if (!out || n_shards == 0 || n_shards > WQ_MAX_SHARDS) return WQ_E_INVALID;
    wq_hub* hub = new (std::nothrow) wq_hub();
    if (!hub) return WQ_E_OOM;
    hub->G = n_shards;
    hub->post.resize(n_shards);
    *out = hub;
    return WQ_OK;
}

int wq_hub_destroy(wq_hub* hub) {
    if (!hub) return WQ_E_INVALID;
    delete hub;
    return WQ_OK;
}

int wq_shard_attach_hub(wq_router* h, wq_hub* hub, uint32_t rank) {
    if (!h || !hub) return WQ_E_INVALID;
    int rc = attach(h, hub->G, rank);
    if (rc) return rc;
    h->shard->kind = kXHub;
    h->shard->hub = hub;
    return WQ_OK;
}

int wq_shard_attach_exchange(wq_router* h, uint32_t n_shards, uint32_t rank, wq_exchange_fn fn, void* ctx) {
    if (!h || !fn) return WQ_E_INVALID;
    int rc = attach(h, n_shards, rank);
    if (rc) return rc;
    h->shard->kind = kXCallback;
    h->shard->fn = fn;
    h->shard->fn_ctx = ctx;
    return WQ_OK;
}

int wq_rccl_unique_id(uint8_t* id_out) {
    if (!id_out) return WQ_E_INVALID;
    RcclApi& api = rccl();
    if (!api.ok) return WQ_E_RCCL;
    ncclUniqueId id;
    if (api.GetUniqueId(&id) != ncclSuccess) return WQ_E_RCCL;
    static_assert(sizeof(id) == WQ_RCCL_ID_BYTES, "ncclUniqueId is 128 bytes");
    memcpy(id_out, &id, sizeof(id));
    return WQ_OK;
}

int wq_shard_attach_rccl(wq_router* h, uint32_t n_shards, uint32_t rank, const uint8_t* id) {
    if (!h || !id) return WQ_E_INVALID;
    RcclApi& api = rccl();
    if (!api.ok) return set_error(h, WQ_E_RCCL, api.why.c_str());
    WQ_HIP(h, hipSetDevice(h->device));
    int rc = attach(h, n_shards, rank);
    if (rc) return rc;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = api.CommInitRank(&comm, (int)n_shards, uid, (int)rank);
    if (r != ncclSuccess) {
        shard_release(h);
        h->err = std::string("ncclCommInitRank: ") + api.GetErrorString(r);
        return WQ_E_RCCL;
    }
    h->shard->kind = kXRccl;
    h->shard->comm = comm;
    return WQ_OK;
}

int wq_shard_detach(wq_router* h) {
    if (!h) return WQ_E_INVALID;
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    shard_release(h);
    return WQ_OK;
}

int wq_shard_info(wq_router* h, uint32_t* n_shards, uint32_t* rank) {
    if (!h || !n_shards || !rank) return WQ_E_INVALID;
    *n_shards = h->shard ? h->shard->G : 1;
    *rank = h->shard ? h->shard->rank : 0;
    return WQ_OK;
}

int wq_sharded_apply_ops(wq_router* h, const wq_op* ops, size_t n) {
    if (!h || (n && !ops)) return WQ_E_INVALID;
    if (!h->shard || h->shard->G == 1) return wq_apply_ops(h, ops, n);
    if (n >= 0xFFFFFFFFull) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    ShardCtx& sc = *h->shard;
    std::vector<uint32_t> owner(n);
    int rc = wq_shard_ops(h, ops, n, sc.G, owner.data());
    if (rc) return rc;
    std::vector<wq_op> mine;
    mine.reserve(n / sc.G + 16);
    for (size_t i = 0; i < n; ++i)
        if (owner[i] == sc.rank || owner[i] == WQ_SHARD_ALL) mine.push_back(ops[i]);
    return wq_apply_ops(h, mine.data(), mine.size());
}

// A receive buffer could not be allocated after the peers were told what they will send: the
// collective cannot complete. The hub is marked broken (its peers fail at their next wait instead
// of timing out); an RCCL or callback caller has to abandon its communicator.
static int fatal_receive(wq_router* h, const char* what) {
    ShardCtx& sc = *h->shard;
    if (sc.kind == kXHub) {
        std::lock_guard<std::mutex> lk(sc.hub->mu);
        sc.hub->broken = true;
        sc.hub->cv.notify_all();
    }
    return set_error(h, WQ_E_OOM, what);
}

// Status word of a failed local step as the exchanges carry it (the negated WQ_E_* code).
static uint32_t status_of(int rc) { return (uint32_t)(-rc); }

// The error a shard reports for a status word it received (its own or a peer's): counter bits
// << 32 (4 spin, 2 > 2^32 pairs, 8 stale table) or a negated WQ_E_* code.
static int status_error(wq_router* h, uint64_t st, uint32_t from) {
    const uint32_t bits = (uint32_t)(st >> 32), code = (uint32_t)st;
    std::string who = " (shard " + std::to_string(from) + ")";
    if (code) return set_error(h, -(int)code, ("sharded tick: a shard's local step failed" + who).c_str());
    if (bits & kErrStale)
        return set_error(h, WQ_E_INVALID, ("sharded tick: a shard's table is still missing an incremental batch the "
                                           "device could not apply" + who).c_str());
    if (bits & 4u) return set_error(h, WQ_E_TIMEOUT, ("sharded tick: a bounded spin gave up" + who).c_str());
    return set_error(h, WQ_E_CAPACITY, ("sharded tick: more than 2^32-1 pairs in one owner block" + who).c_str());
}

// Steps 1-3 of a sharded tick, shared by the origin and owner forms: shard this rank's messages,
// exchange the counts (host read 1) and the records, route what this shard owns into
// own_off / own_peers. *R_out = records received, *seg = their source segments. A local route
// failure is left in *late_out (the caller keeps the collective going); a return value != WQ_OK is
// an exchange or argument failure.
static int shard_exchange_route(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                                const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs, uint64_t* R_out,
                                SegBounds* seg_out, int* late_out, std::string* late_msg_out) {
    hipStream_t s = h->stream;
    ShardCtx& sc = *h->shard;
    const uint32_t G = sc.G;
    const size_t M = n_msgs;
    sc.last_ready = false;
    sc.last_slots = false;
    sc.small_zeroed = false;  // this form writes the small vectors its own way
    int& late = *late_out;  // a local failure, reported once the tick's exchanges are complete
    std::string& late_msg = *late_msg_out;
    auto fail = [&](int rc) {
        if (rc && !late) {
            late = rc;
            late_msg = h->err;
        }
        return rc;
    };

    const int inject = h->shard_inject;
    h->shard_inject = 0;
    // 1. shard (a failure here: this shard sends nothing, and reports the error after the exchanges)
    uint32_t* cnt_send = reinterpret_cast<uint32_t*>(sc.small.as<char>() + kSmallA);
    uint32_t* cnt_recv = cnt_send + G;
    WQ_HIP(h, hipMemsetAsync(cnt_send, 0, 4 * G, s));
    if (inject == 1) fail(set_error(h, WQ_E_INVALID, "injected failure at step 1 (test hook)"));
    // as the slot tick and the single-GPU tick: the radius filter needs the message positions
    if (h->radius > 0.0 && M && !d_pos && !late)
        fail(set_error(h, WQ_E_INVALID, "the radius filter needs message positions"));
    int rc = late ? late : sc.recs.ensure((M ? M : 1) * sizeof(wq_msg_rec)) == hipSuccess
                 ? WQ_OK
                 : set_error(h, WQ_E_OOM, "hipMalloc of the sharded tick's records");
    if (!fail(rc))
        fail(launch_shard_messages(h, d_pos, d_keys, d_world, d_sender, d_repl, M, G, sc.recs.as<wq_msg_rec>(),
                                   cnt_send));
    if (late) WQ_HIP(h, hipMemsetAsync(cnt_send, 0, 4 * G, s));
    // 2. counts, then the records
    std::vector<size_t> four(G, 4);
    {
        Xfer x{{cnt_send}, {four.data()}, {cnt_recv}, {four.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
    }
    sc.sc.assign(2 * G, 0);
    WQ_HIP(h, hipMemcpyAsync(sc.sc.data(), cnt_send, 2 * G * 4, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));  // host read 1
    sc.rc.assign(sc.sc.begin() + G, sc.sc.end());
    sc.sc.resize(G);
    uint64_t R = 0;
    std::vector<size_t> sb(G), rb(G);
    SegBounds seg;
    seg.b[0] = 0;
    for (uint32_t d = 0; d < G; ++d) {
        sb[d] = (size_t)sc.sc[d] * sizeof(wq_msg_rec);
        rb[d] = (size_t)sc.rc[d] * sizeof(wq_msg_rec);
        R += sc.rc[d];
        seg.b[d + 1] = (uint32_t)R;
    }
    if (R >= 0xFFFFFC00ull) return fatal_receive(h, "more than 2^32 - 1024 records on one owner");
    if (sc.recv.ensure((R ? R : 1) * sizeof(wq_msg_rec)) != hipSuccess)
        return fatal_receive(h, "hipMalloc of the received records");
    {
        Xfer x{{sc.recs.p}, {sb.data()}, {sc.recv.p}, {rb.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
    }
    // 3. route what this shard owns (a failure: empty results here, the error after the exchanges)
    if (!sc.own_cap) {
        sc.own_cap = 16 * R + 4096;
        if (sc.own_cap > 0xFFFFFFFFull) sc.own_cap = 0xFFFFFFFFull;
    }
    const bool bufs = sc.own_off.ensure((R + 1) * 4) == hipSuccess && sc.own_peers.ensure(sc.own_cap * 4) == hipSuccess &&
                      sc.own_e.ensure((R ? R : 1) * 4) == hipSuccess;
    if (!bufs) fail(set_error(h, WQ_E_OOM, "hipMalloc of the owner's route buffers"));
    if (inject == 3) fail(set_error(h, WQ_E_INVALID, "injected failure at step 3 (test hook)"));
    if (!late)
        fail(launch_route_records(h, sc.recv.as<wq_msg_rec>(), R, sc.own_off.as<uint32_t>(), sc.own_peers.as<uint32_t>(),
                                  nullptr, sc.own_cap));
    *R_out = R;
    *seg_out = seg;
    return WQ_OK;
}

// The slot tick (radius filter off) — wq_sharded_route_tick_device's result, built as
//   own     this shard's own cubes: count_kernel<OWN> over the caller's messages, on a side stream
//           beside the exchanges (no slot, nothing crosses a link)
//   X1      {A: slots + status per owner, the slots: 20 B per remote message, budgeted segments}
//   owner   count the received slots (count_kernel<SLOTS>), claim each (source, cube) once
//           (k_ref_claim), a 12-byte reference per slot and per source ONE pool of cube lists
//   X2      {C: pool words + status per source, the references, the pools}
//   ingest  references -> rows (k_ref_resolve), tile scan, emit_map_kernel over own + pool rows
//   end     ONE host read: P, every shard's status, the true sizes (the next tick's budgets)
// so a long list crosses xGMI once per (tick, destination), and the exchanges are enqueued without
// reading anything back: their sizes are the budgets, fixed on the host before the tick (the
// previous tick's true sizes + 1/16 + a block; identical on both ends of every pair, since both saw
// the same sizes). A tick whose sizes outgrow a budget is flagged on the device; the status reaches
// every shard through C, and all of them redo the tick exactly: A and C exchanged alone first and
// read back, as the first tick does. Local failures keep the collective going: a failed step sends
// its status (zero slots / empty pools) and every shard returns the error after X2.
namespace {
inline uint32_t whole_blocks(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock * kBlock); }
inline uint32_t slot_budget(uint64_t n) { return whole_blocks(n + n / 16 + kBlock); }
inline uint64_t pool_budget(uint64_t n) { return n + n / 16 + 1024; }
}  // namespace

static int ensure_health(wq_router* h) {
    RouteWs& rw = h->rws;
    if (!rw.buf.p) {  // as route_counters lays it out: health words first
        WQ_ALLOC(h, rw.buf, 128);
        WQ_HIP(h, hipMemsetAsync(rw.buf.p, 0, 128, h->stream));
        rw.calls = 0;
    }
    return WQ_OK;
}

// The global picture of a finished slot tick from its small vectors (the same on every shard: codes
// and device bits from every shard's A and C), and the next tick's budgets from its true sizes when
// it was clean; a tick whose sizes outgrew a budget leaves the budgets off (the next tick is exact).
struct TickPicture {
    uint32_t code = 0, bits = 0, code_from = 0, bits_from = 0;
    bool over = false;
};
static TickPicture fold_tick(ShardCtx& sc, const char* hs, bool self_seg = false) {
    const uint32_t G = sc.G, me = sc.rank;
    const uint32_t* ha = reinterpret_cast<const uint32_t*>(hs + kSmallA);
    const uint32_t* hc = reinterpret_cast<const uint32_t*>(hs + kSmallC);
    TickPicture t;
    if (self_seg) {  // the owner form on slots: A only, the self segment budgeted like the others
        for (uint32_t d = 0; d < G; ++d) {
            const uint32_t st = ha[2 * G + 2 * d + 1];
            if ((st & kStCodeMask) && !t.code) t.code = st & kStCodeMask, t.code_from = d;
            if (((st >> 8) & 0xFFFFu) && !t.bits) t.bits = (st >> 8) & 0xFFFFu, t.bits_from = d;
            t.over |= (st & kStBudget) != 0;
        }
        if (!t.code && !t.over) {
            for (uint32_t d = 0; d < G; ++d) {
                sc.b1_out[d] = slot_budget(ha[2 * d]);
                sc.b1_in[d] = slot_budget(ha[2 * G + 2 * d]);
            }
            sc.budgets = true;
        }
        if (t.over) sc.budgets = false;
        return t;
    }
    for (uint32_t d = 0; G > 1 && d < G; ++d) {
        for (uint32_t st : {ha[2 * G + 2 * d + 1], hc[2 * G + 2 * d + 1]}) {
            if ((st & kStCodeMask) && !t.code) t.code = st & kStCodeMask, t.code_from = d;
            if (((st >> 8) & 0xFFFFu) && !t.bits) t.bits = (st >> 8) & 0xFFFFu, t.bits_from = d;
            t.over |= (st & kStBudget) != 0;
        }
    }
    if (G > 1 && !t.code && !t.over) {  // next tick's budgets from this tick's true sizes
        for (uint32_t d = 0; d < G; ++d) {
            sc.b1_out[d] = d == me ? 0u : slot_budget(ha[2 * d]);
            sc.b1_in[d] = d == me ? 0u : slot_budget(ha[2 * G + 2 * d]);
            sc.b2_out[d] = d == me ? 0 : pool_budget(hc[2 * d]);
            sc.b2_in[d] = d == me ? 0 : pool_budget(hc[2 * G + 2 * d]);
        }
        sc.budgets = true;
    }
    if (t.over) sc.budgets = false;
    return t;
}

// Folds in the snapshots of asynchronous ticks until at most `keep` are in flight (oldest first,
// waiting for each; every shard makes the same calls, so every shard folds the same ticks).
static int async_drain(wq_router* h, uint32_t keep) {
    ShardCtx& sc = *h->shard;
    while (sc.acount > keep) {
        const uint32_t k = sc.ahead;
        // k_async_result writes the snapshot, then its sequence word (system-scope release)
        const volatile uint64_t* seq =
            reinterpret_cast<const volatile uint64_t*>(static_cast<const char*>(sc.asnap[k]) + kSmallBytes);
        const auto t0 = std::chrono::steady_clock::now();
        while (*seq != sc.aseq[k]) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
                // name everything a post-mortem needs: which tick, which ring slot, what the word holds,
                // and whether the stream still had work (idle + wrong word = the snapshot was never written)
                const hipError_t q = hipStreamQuery(h->stream);
                char msg[320];
                snprintf(msg, sizeof msg,
                         "asynchronous sharded tick: its result never arrived (tick %llu of this handle, ring slot %u "
                         "of %u, %u in flight; sequence word expected %llu, observed %llu; stream %s)",
                         (unsigned long long)sc.aseq[k], k, ShardCtx::kRing, sc.acount, (unsigned long long)sc.aseq[k],
                         (unsigned long long)*seq,
                         q == hipSuccess ? "idle" : q == hipErrorNotReady ? "busy" : hipGetErrorString(q));
                return set_error(h, WQ_E_TIMEOUT, msg);
            }
            std::this_thread::yield();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        const char* snap = static_cast<const char*>(sc.asnap[k]);
        (void)fold_tick(sc, snap, sc.budget_form == 1);  // the ring only ever holds one form's ticks
        if (sc.budget_form == 1) {  // the owner form: a pair buffer that was short grows for the next tick
            const uint64_t P = reinterpret_cast<const wq_route_counters*>(snap + kSmallCnt)[kCntScan].n_pairs;
            if (P > sc.own_cap) sc.own_cap = std::min<uint64_t>(P + P / 4 + 4096, 0xFFFFFFFFull);
        }
        sc.ahead = (k + 1) % ShardCtx::kRing;
        sc.acount--;
    }
    return WQ_OK;
}

// (asynchronous tick) the end-of-tick snapshot kernel, when the tile scan could not take it
// (route_async.hpp async_result_block: a scan over more tiles than one block takes, or no scan)
__global__ __launch_bounds__(256) void k_async_result(AsyncResultParams p) { async_result_block(p); }


static int slot_tick(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                     const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                     uint32_t* d_peers, uint32_t* d_msgs, size_t capacity, size_t* n_pairs, bool exact, int inject,
                     bool* redo, bool async = false, wq_route_counters* d_result = nullptr) {
    hipStream_t s = h->stream;
    ShardCtx& sc = *h->shard;
    const uint32_t G = sc.G, me = sc.rank;
    *redo = false;
    sc.last_ready = false;
    sc.last_slots = true;
    int late = WQ_OK;
    std::string late_msg;
    auto fail = [&](int rc) {
        if (rc && !late) {
            late = rc;
            late_msg = h->err;
        }
        return rc;
    };
    auto alloc = [&](DevBuf& b, size_t bytes) -> int {
        return b.ensure(bytes) == hipSuccess ? WQ_OK : set_error(h, WQ_E_OOM, "hipMalloc (sharded tick workspace)");
    };
    char* small = sc.small.as<char>();
    uint32_t* a_send = reinterpret_cast<uint32_t*>(small + kSmallA);
    uint32_t* a_recv = a_send + 2 * G;
    uint32_t* c_send = reinterpret_cast<uint32_t*>(small + kSmallC);
    uint32_t* c_recv = c_send + 2 * G;
    wq_route_counters* cnts = reinterpret_cast<wq_route_counters*>(small + kSmallCnt);
    const size_t small_used = kSmallCnt + 4 * sizeof(wq_route_counters);
    static_assert(kSmallC + 16 * WQ_MAX_SHARDS <= kSmallCnt, "the C vectors lie inside the zeroed span");
    // A, C (both directions) and the counters (an asynchronous tick's last kernel zeroes them itself)
    if (!sc.small_zeroed) WQ_HIP(h, hipMemsetAsync(small, 0, small_used, s));
    sc.small_zeroed = false;
    if (int rc = ensure_health(h)) return rc;
    if (exact) sc.n_exact++;
    else sc.n_budget++;
    // host sources of status copies: alive until the end-of-tick read has synchronised the stream
    std::vector<uint32_t> st_host(2 * G, 0);
    auto put_status = [&](uint32_t* dst) -> int {
        for (uint32_t d = 0; d < G; ++d) st_host[2 * d + 1] = status_of(late);
        WQ_HIP(h, hipMemcpyAsync(dst, st_host.data(), 8 * G, hipMemcpyHostToDevice, s));
        return WQ_OK;
    };

    if (inject == 1) fail(set_error(h, WQ_E_INVALID, "injected failure at step 1 (test hook)"));
    // the radius filter (C5): own cubes by count_radius_kernel, remote rows filtered where they land
    const bool radius = h->radius > 0.0;
    if (radius && M && !d_pos && !late) fail(set_error(h, WQ_E_INVALID, "the radius filter needs message positions"));
    // fold in a finished incremental batch first (it may rebuild the table the rows point into)
    if (!late) fail(table_resolve(h, false));
    if (!late && G > 1 && h->tab.list.bytes / 4 >= (1ull << 30))
        fail(set_error(h, WQ_E_CAPACITY, "sharded tick: more than 2^30 list words on one shard"));
    const TableView tv = table_view(h);
    const uint32_t nt = (uint32_t)((M + kBlock - 1) / kBlock);
    if (!late && (fail(alloc(sc.e_msg, (M + 1) * 4)) || fail(alloc(sc.info_msg, (M + 1) * 8)) ||
                  fail(alloc(sc.mtiles, ((uint64_t)nt * 3 + 4) * 4)))) {
    }

    // ---- own cubes. G > 1 without the radius filter (own slots): the grouping pass writes this
    // shard's own messages as slots of a segment that is never exchanged, and the side stream counts
    // them once grouped (below), beside the exchanges and the owner's work — the grouping's
    // histogram pass quantises every message, but probes nothing. Otherwise the own-cube count runs
    // over every message on the side stream (count_kernel<OWN>), or (diagnostics,
    // WQ_SHARD_OWN_FUSED) in one pass with the histogram on the tick's stream, as in round 4 ----
    bool forked = false, hist_ready = false;
    static const bool two_pass = getenv("WQ_DEBUG_NO_OWN_HIST") != nullptr;  // diagnostics
    static const bool fused_env = getenv("WQ_SHARD_OWN_FUSED") != nullptr;   // diagnostics
    const bool own_slots = G > 1 && !radius && !two_pass && !fused_env;
    const bool fuse = G > 1 && !radius && budget_slot_tile() == kHistTiles * kBlock && !two_pass && fused_env;
    if (!late && M && own_slots) {
        const uint64_t nto = (2 * M + kBlock - 1) / kBlock;
        if (!fail(alloc(sc.own_slots, (2 * M + 2) * kSlotWords * 4)) && !fail(alloc(sc.own_perm, (2 * M + 2) * 4)) &&
            !fail(alloc(sc.own_tiles, (nto + 1) * 8))) {
            // (a message no step writes a row for — its slot was over budget, the tick is redone —
            // routes to nobody: the histogram pass zeroes every e)
        }
    }
    if (!late && M && fuse) {
        const uint32_t nblk = (uint32_t)((M + kHistTiles * kBlock - 1) / (kHistTiles * kBlock));
        if (!fail(alloc(h->shard_hist, (uint64_t)nblk * G * 4))) {
            CountParams cp{};
            cp.in = RouteIn{d_pos, d_keys, d_world, d_sender, d_repl, (uint32_t)M, (int64_t)h->cube_size};
            cp.in.own_G = G;
            cp.in.own_me = me;
            cp.t = tv;
            cp.e = sc.e_msg.as<uint32_t>();
            cp.info = sc.info_msg.as<uint2>();
            cp.tile_total = sc.mtiles.as<uint32_t>();
            cp.tile_F = cp.tile_total + 2 * (uint64_t)nt;
            cp.cnt = cnts + kCntSelf;
            cp.cnt_next = cnts + kCntScratch;
            cp.health = route_health(h);
            cp.n_tiles = nt;
            if (d_keys)
                hipLaunchKernelGGL(own_count_hist_kernel<true>, dim3(nblk), dim3(kBlock), 0, s, cp, nblk,
                                   h->shard_hist.as<uint32_t>());
            else
                hipLaunchKernelGGL(own_count_hist_kernel<false>, dim3(nblk), dim3(kBlock), 0, s, cp, nblk,
                                   h->shard_hist.as<uint32_t>());
            WQ_HIP(h, hipGetLastError());
            hist_ready = true;
        }
    } else if (!late && M && !own_slots) {
        WQ_HIP(h, hipEventRecord(sc.ev_fork, s));
        WQ_HIP(h, hipStreamWaitEvent(sc.side, sc.ev_fork, 0));
        CountParams cp{};
        cp.in = RouteIn{d_pos, d_keys, d_world, d_sender, d_repl, (uint32_t)M, (int64_t)h->cube_size};
        cp.in.own_G = G;
        cp.in.own_me = me;
        cp.t = tv;
        cp.e = sc.e_msg.as<uint32_t>();
        cp.info = sc.info_msg.as<uint2>();
        cp.tile_total = sc.mtiles.as<uint32_t>();
        cp.tile_F = cp.tile_total + 2 * (uint64_t)nt;
        cp.cnt = cnts + kCntSelf;
        cp.cnt_next = cnts + kCntScratch;
        cp.health = route_health(h);
        cp.n_tiles = nt;
        const dim3 grid(pass_blocks(nt));  // as launch_route
        if (radius && G == 1)
            hipLaunchKernelGGL(count_radius_kernel<false>, dim3(nt), dim3(kBlock), 0, sc.side, cp);
        else if (radius)
            hipLaunchKernelGGL(count_radius_kernel<true>, dim3(nt), dim3(kBlock), 0, sc.side, cp);
        else if (G == 1 && d_keys)
            hipLaunchKernelGGL((count_kernel<true, 1, 8>), grid, dim3(kBlock), 0, sc.side, cp);
        else if (G == 1)
            hipLaunchKernelGGL((count_kernel<false, 1, 8>), grid, dim3(kBlock), 0, sc.side, cp);
        else if (d_keys)
            hipLaunchKernelGGL((count_kernel<true, 1, 8, 0, false, false, true>), grid, dim3(kBlock), 0, sc.side, cp);
        else
            hipLaunchKernelGGL((count_kernel<false, 1, 8, 0, false, false, true>), grid, dim3(kBlock), 0, sc.side, cp);
        WQ_HIP(h, hipGetLastError());
        WQ_HIP(h, hipEventRecord(sc.ev_join, sc.side));
        forked = true;
    }

    // ---- X1: A + the slots ----
    std::vector<size_t> eight(G, 8);
    SlotLayout L{};
    SegBounds sb{}, rb{};
    auto set_layout = [&]() -> int {
        uint64_t so = 0, ro = 0;
        for (uint32_t d = 0; d < G; ++d) {
            L.base[d] = (uint32_t)so;
            L.budget[d] = sc.b1_out[d];
            sb.b[d] = (uint32_t)so;
            rb.b[d] = (uint32_t)ro;
            so += sc.b1_out[d];
            ro += sc.b1_in[d];
        }
        L.base[G] = sb.b[G] = (uint32_t)so;
        rb.b[G] = (uint32_t)ro;
        if (so >= (1ull << 31) || ro >= (1ull << 31)) return fatal_receive(h, "sharded tick: more than 2^31 slots");
        return WQ_OK;
    };
    uint64_t Sb = 0, Rb = 0;
    int rc;
    if (G > 1) {
        if (exact) {  // the true counts first (A alone, read back): budgets = the counts, whole blocks
            SlotLayout inf{};
            for (uint32_t d = 0; d < G; ++d) inf.budget[d] = 0xFFFFFFFFu;
            if (!late)
                fail(launch_budget_slots(h, d_pos, d_keys, d_world, d_sender, d_repl, M, G, me, inf, nullptr, nullptr,
                                         a_send, 1, hist_ready, own_slots, nullptr, nullptr,
                                         own_slots ? sc.e_msg.as<uint32_t>() : nullptr));
            if (late && (rc = put_status(a_send))) return rc;
            Xfer x{{a_send}, {eight.data()}, {a_recv}, {eight.data()}, 1};
            if ((rc = exchange(h, x))) return rc;
            uint32_t* hv = static_cast<uint32_t*>(sc.hsmall);
            WQ_HIP(h, hipMemcpyAsync(hv, a_send, 16 * G, hipMemcpyDeviceToHost, s));
            WQ_HIP(h, hipStreamSynchronize(s));
            for (uint32_t d = 0; d < G; ++d) {
                sc.b1_out[d] = d == me ? 0u : whole_blocks(hv[2 * d]);
                sc.b1_in[d] = d == me ? 0u : whole_blocks(hv[2 * G + 2 * d]);
            }
        }
        if ((rc = set_layout())) return rc;
        Sb = sb.b[G];
        Rb = rb.b[G];
        if (alloc(sc.slots, (Sb + 2) * kSlotWords * 4) || alloc(sc.perm, (Sb + 2) * 4) ||
            alloc(sc.rslots, (Rb + 2) * kSlotWords * 4))
            return fatal_receive(h, "hipMalloc of the sharded tick's slots");
        if (!late)
            fail(launch_budget_slots(h, d_pos, d_keys, d_world, d_sender, d_repl, M, G, me, L, sc.slots.as<uint32_t>(),
                                     sc.perm.as<uint32_t>(), a_send, exact ? 2 : 3, hist_ready, own_slots,
                                     sc.own_slots.as<uint32_t>(), sc.own_perm.as<uint32_t>(),
                                     own_slots && !exact ? sc.e_msg.as<uint32_t>() : nullptr));

        if (late) {  // nothing to send: tail slots everywhere (zero words route to nobody either way)
            WQ_HIP(h, hipMemsetAsync(sc.slots.p, 0, (Sb + 1) * kSlotWords * 4, s));
            WQ_HIP(h, hipMemsetAsync(sc.perm.p, 0xFF, (Sb + 1) * 4, s));
            if (!exact && (rc = put_status(a_send))) return rc;
        }
        std::vector<size_t> sbytes(G), rbytes(G);
        for (uint32_t d = 0; d < G; ++d) {
            sbytes[d] = (size_t)sc.b1_out[d] * kSlotWords * 4;
            rbytes[d] = (size_t)sc.b1_in[d] * kSlotWords * 4;
        }
        if (exact) {
            Xfer x{{sc.slots.p}, {sbytes.data()}, {sc.rslots.p}, {rbytes.data()}, 1};
            if ((rc = exchange(h, x))) return rc;
        } else {
            Xfer x{{a_send, sc.slots.p}, {eight.data(), sbytes.data()}, {a_recv, sc.rslots.p},
                   {eight.data(), rbytes.data()}, 2};
            if ((rc = exchange(h, x))) return rc;
        }
    }

    // ---- the owner: count the received slots (local_message.rs:52-86 per slot), claims, references ----
    if (inject == 3) fail(set_error(h, WQ_E_INVALID, "injected failure at step 3 (test hook)"));
    RefOwnerParams rp{};
    if (G > 1 && (alloc(sc.ref_send, (Rb + 1) * 12) || alloc(sc.plen, (Rb + 1) * 4) || alloc(sc.poff, (Rb + 1) * 4)))
        return fatal_receive(h, "hipMalloc of the owner's references");
    if (G > 1 && Rb && !late) {
        RouteWs& rw = h->rws;
        const uint32_t nto = (uint32_t)(Rb / kBlock);  // whole blocks
        if (!fail(alloc(rw.e, Rb * 4)) && !fail(alloc(rw.info, Rb * 8)) && !fail(alloc(sc.otiles, (uint64_t)nto * 8)) &&
            !fail(alloc(sc.ocnt, Rb * 4)) && !fail(alloc(sc.hslot, Rb * 4)) && !fail(alloc(sc.desc_fill, (Rb + 1) * 16))) {
            CountParams cp{};
            cp.in = RouteIn{nullptr, nullptr, nullptr, nullptr, nullptr, (uint32_t)Rb, (int64_t)h->cube_size};
            cp.in.slots = sc.rslots.as<uint32_t>();
            cp.t = tv;
            cp.e = rw.e.as<uint32_t>();
            cp.info = rw.info.as<uint2>();
            cp.tile_total = sc.otiles.as<uint32_t>();
            cp.tile_F = cp.tile_total + nto;
            cp.cnt = cnts + kCntOwner;
            cp.cnt_next = cnts + kCntScratch;
            cp.health = route_health(h);
            cp.n_tiles = nto;
            hipLaunchKernelGGL((count_kernel<false, 1, 8, 0, false, true>), dim3(pass_blocks(nto)), dim3(kBlock), 0, s, cp);
            if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "count launch (sharded tick)"));
        }
    }
    if (G > 1 && !late && M && own_slots) {
        // after the owner count: beside the claims, references, pool gather and X2 (beside the
        // owner count, the two probe passes only slowed each other down)
        // the own slots (their count: the own column of this tick's histogram, a_send[2 me], known
        // on the device only) counted on the side stream, e / locator straight to message order
        WQ_HIP(h, hipEventRecord(sc.ev_fork, s));
        WQ_HIP(h, hipStreamWaitEvent(sc.side, sc.ev_fork, 0));
        const uint32_t n_max = (uint32_t)(2 * M);
        const uint32_t nto = (n_max + kBlock - 1) / kBlock;
        CountParams cp{};
        cp.in = RouteIn{nullptr, nullptr, nullptr, nullptr, nullptr, n_max, (int64_t)h->cube_size};
        cp.in.slots = sc.own_slots.as<uint32_t>();
        cp.in.m_dev = a_send + 2 * me;
        cp.t = tv;
        cp.e = sc.e_msg.as<uint32_t>();
        cp.info = sc.info_msg.as<uint2>();
        cp.perm = sc.own_perm.as<uint32_t>();
        cp.tile_total = sc.own_tiles.as<uint32_t>();
        cp.tile_F = cp.tile_total + nto;
        cp.cnt = cnts + kCntSelf;
        cp.cnt_next = cnts + kCntScratch;
        cp.health = route_health(h);
        cp.n_tiles = nto;
        hipLaunchKernelGGL((count_kernel<false, 1, 8, 0, false, true>), dim3(std::min<uint32_t>(nto, 4096u)),
                           dim3(kBlock), 0, sc.side, cp);
        WQ_HIP(h, hipGetLastError());
        WQ_HIP(h, hipEventRecord(sc.ev_join, sc.side));
        forked = true;
    }
    if (G > 1 && Rb && !late) {
        RouteWs& rw = h->rws;
        uint64_t C = 1024;  // claim table: load <= 1/2
        while (C < 2 * Rb) C <<= 1;
        if (!late && C > sc.claim_cap) {
            if (!fail(alloc(sc.claim, C * 8)) && !fail(alloc(sc.lead, C * 4))) {
                if (hipMemsetAsync(sc.claim.p, 0, C * 8, s) != hipSuccess) fail(set_error(h, WQ_E_HIP, "memset"));
                sc.claim_cap = C;
            }
        }
        C = sc.claim_cap;
        if (!late) {
            const uint64_t period = (1ull << kRefClaimTagBits) - 1;
            if (sc.ticks && sc.ticks % period == 0 && hipMemsetAsync(sc.claim.p, 0, sc.claim_cap * 8, s) != hipSuccess)
                fail(set_error(h, WQ_E_HIP, "memset"));  // the tags wrap: forget them all
            rp.e = rw.e.as<uint32_t>();
            rp.info = rw.info.as<uint2>();
            rp.list = tv.list;
            rp.recs = tv.recs;
            rp.rrem = rb;
            rp.G = G;
            rp.n_rem = (uint32_t)Rb;
            rp.self_lo = (uint32_t)Rb;  // no own segment: received slot t is remote slot t
            rp.n_self = 0;
            rp.tag = (uint32_t)(sc.ticks % period) + 1u;
            rp.claim = sc.claim.as<unsigned long long>();
            rp.lead = sc.lead.as<uint32_t>();
            rp.cmask = C - 1;
            rp.cnt = sc.ocnt.as<uint32_t>();
            rp.hslot = sc.hslot.as<uint32_t>();
            rp.plen = sc.plen.as<uint32_t>();
            rp.poff = sc.poff.as<uint32_t>();
            rp.ref_send = sc.ref_send.as<uint3>();
            rp.desc_fill = sc.desc_fill.as<uint4>();
            sc.ticks++;
            hipLaunchKernelGGL(k_ref_claim, dim3((unsigned)((Rb + kBlock) / kBlock)), dim3(kBlock), 0, s, rp);
            if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "claim launch (sharded tick)"));
            if (!late) fail(scan_excl(h, sc.tmp, sc.plen.as<uint32_t>(), sc.poff.as<uint32_t>(), Rb + 1));
            if (!late) {
                hipLaunchKernelGGL(k_ref_make, dim3((unsigned)(Rb / kBlock)), dim3(kBlock), 0, s, rp);
                if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "reference launch (sharded tick)"));
            }
        }
    }

    // ---- X2: C + the references and pools ----
    std::vector<uint64_t> pb(G + 1, 0), prb(G + 1, 0);
    uint64_t sent = 0, recvd = 0;
    if (G > 1) {
        const bool owner_ok = Rb && !late;
        if (!late) {
            CVecParams cv{};
            cv.a_send = a_send;
            cv.a_recv = a_recv;
            cv.poff = owner_ok ? sc.poff.as<uint32_t>() : nullptr;
            cv.rb = rb;
            for (uint32_t d = 0; d < G; ++d) cv.b2[d] = exact ? ~0ull : sc.b2_out[d];
            cv.G = G;
            cv.stale = tv.stale;
            cv.cnt = owner_ok ? cnts + kCntOwner : nullptr;
            cv.c_send = c_send;
            hipLaunchKernelGGL(k_c_vector, dim3(1), dim3(64), 0, s, cv);
            if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "size launch (sharded tick)"));
        }
        if (late) {
            if ((rc = put_status(c_send))) return rc;
            WQ_HIP(h, hipMemsetAsync(sc.ref_send.p, 0, (Rb + 1) * 12, s));  // references that route to nobody
        }
        if (exact) {  // the true pool sizes first (C alone, read back)
            Xfer x{{c_send}, {eight.data()}, {c_recv}, {eight.data()}, 1};
            if ((rc = exchange(h, x))) return rc;
            uint32_t* hv = static_cast<uint32_t*>(sc.hsmall);
            WQ_HIP(h, hipMemcpyAsync(hv, c_send, 16 * G, hipMemcpyDeviceToHost, s));
            WQ_HIP(h, hipStreamSynchronize(s));
            for (uint32_t d = 0; d < G; ++d) {
                sc.b2_out[d] = d == me ? 0 : hv[2 * d];
                sc.b2_in[d] = d == me ? 0 : hv[2 * G + 2 * d];
            }
        }
        for (uint32_t d = 0; d < G; ++d) {
            pb[d + 1] = pb[d] + sc.b2_out[d];
            prb[d + 1] = prb[d] + sc.b2_in[d];
        }
        if (prb[G] >= (1ull << 30)) return fatal_receive(h, "sharded tick: more than 2^30 pool words to receive");
        if (alloc(sc.pool_send, (pb[G] + 1) * 4) || alloc(sc.pool_recv, (prb[G] + 1) * 4) ||
            alloc(sc.ref_recv, (Sb + 1) * 12))
            return fatal_receive(h, "hipMalloc of the references / pools");
        if (owner_ok && !late && pb[G]) {
            const uint32_t nbo = (uint32_t)(Rb / kBlock);
            if (alloc(sc.blk, (uint64_t)nbo * 16 + 16)) return fatal_receive(h, "hipMalloc of the pool blocks");
            PoolBlocksParams bp{};
            bp.poff = sc.poff.as<uint32_t>();
            bp.rb = rb;
            for (uint32_t d = 0; d <= G; ++d) bp.pb[d] = pb[d];
            bp.G = G;
            bp.nblk = nbo;
            bp.base = sc.blk.as<uint64_t>();
            bp.lim = bp.base + nbo;
            hipLaunchKernelGGL(k_pool_blocks, dim3((nbo + kBlock - 1) / kBlock), dim3(kBlock), 0, s, bp);
            GatherParams gp{sc.poff.as<uint32_t>(), sc.desc_fill.as<uint4>(), (uint32_t)Rb, sc.pool_send.as<uint32_t>(),
                            nullptr, pb[G]};
            gp.blk_base = bp.base;
            gp.blk_lim = bp.lim;
            hipLaunchKernelGGL((gather_rows_kernel<16, false>), dim3(nbo), dim3(kBlock), 0, s, gp);
            if (hipGetLastError() != hipSuccess) return fatal_receive(h, "pool gather launch");
        }
        std::vector<size_t> rs(G), rr(G), ps(G), pr(G);
        for (uint32_t d = 0; d < G; ++d) {
            rs[d] = (size_t)sc.b1_in[d] * 12;   // references for the slots d sent here
            rr[d] = (size_t)sc.b1_out[d] * 12;  // references for the slots sent to d
            ps[d] = (size_t)sc.b2_out[d] * 4;
            pr[d] = (size_t)sc.b2_in[d] * 4;
            if (d != me) {
                sent += 16 + (uint64_t)sc.b1_out[d] * kSlotWords * 4 + rs[d] + ps[d];
                recvd += 16 + (uint64_t)sc.b1_in[d] * kSlotWords * 4 + rr[d] + pr[d];
            }
        }
        if (exact) {
            Xfer x{{sc.ref_send.p, sc.pool_send.p}, {rs.data(), ps.data()}, {sc.ref_recv.p, sc.pool_recv.p},
                   {rr.data(), pr.data()}, 2};
            if ((rc = exchange(h, x))) return rc;
        } else {
            Xfer x{{c_send, sc.ref_send.p, sc.pool_send.p}, {eight.data(), rs.data(), ps.data()},
                   {c_recv, sc.ref_recv.p, sc.pool_recv.p}, {eight.data(), rr.data(), pr.data()}, 3};
            if ((rc = exchange(h, x))) return rc;
        }
    }
    sc.last_sent = sent;
    sc.last_recv = recvd;

    // ---- the ingesting side: rows in message order, then the CSR ----
    if (forked && !own_slots) WQ_HIP(h, hipStreamWaitEvent(s, sc.ev_join, 0));  // own rows written (remote: e = 0)
    if (!late && G > 1 && Sb) {
        ResolveParams rv{};
        rv.perm = sc.perm.as<uint32_t>();
        rv.ref_recv = sc.ref_recv.as<uint3>();
        rv.sb = sb;
        rv.G = G;
        rv.n = (uint32_t)Sb;
        for (uint32_t d = 0; d <= G; ++d) rv.prb[d] = prb[d];
        rv.e_msg = sc.e_msg.as<uint32_t>();
        rv.info_msg = sc.info_msg.as<uint2>();
        const dim3 rg((unsigned)((Sb + kBlock - 1) / kBlock));
        if (radius) {
            rv.pool = sc.pool_recv.as<uint32_t>();
            rv.pos = d_pos;
            rv.sender = d_sender;
            rv.repl = d_repl;
            rv.tv = tv;
            hipLaunchKernelGGL(k_ref_resolve<true>, rg, dim3(kBlock), 0, s, rv);
        } else {
            hipLaunchKernelGGL(k_ref_resolve<false>, rg, dim3(kBlock), 0, s, rv);
        }
        WQ_HIP(h, hipGetLastError());
    }
    if (forked && own_slots) WQ_HIP(h, hipStreamWaitEvent(s, sc.ev_join, 0));  // own rows written
    // the per-tile totals of every row (a count pass's held its own rows only)
    if (!late && G > 1 && M && (Sb || own_slots)) {
        hipLaunchKernelGGL(row_tile_sums_kernel, dim3(nt), dim3(kBlock), 0, s, sc.e_msg.as<uint32_t>(), (uint32_t)M,
                           sc.mtiles.as<uint32_t>());
        WQ_HIP(h, hipGetLastError());
    }
    if (!late) {
        sc.last_M = M;
        sc.last_sender = d_sender;
        sc.last_pos = d_pos;
        sc.last_repl = d_repl;
        sc.last_radius = radius;
        sc.last_gen = h->table_gen;
    }
    // ---- asynchronous end (wq_sharded_route_tick_async, a budgeted tick): no host read; the small
    // vectors go to a pinned snapshot the next calls fold in (budgets), P and the statuses to the
    // caller's counters and the health words — at the end of the tile scan when one block runs it,
    // else by k_async_result. A shard whose local step failed takes this end too (and then returns its
    // error): whether a tick is queued in the snapshot ring must be decided by state every shard
    // shares, or the shards would fold different ticks and size their next exchanges differently ----
    const bool async_end = async && !exact;
    AsyncResultParams ar{};
    const uint32_t ak = (sc.ahead + sc.acount) % ShardCtx::kRing;  // async_drain left a free slot
    if (async_end) {
        ar.a_recv = a_recv;
        ar.c_recv = c_recv;
        ar.G = G;
        ar.statuses = G > 1 ? 1u : 0u;
        ar.cnt = cnts;
        ar.has_msgs = M ? 1u : 0u;
        ar.capacity = capacity;
        ar.out = d_result;
        ar.health = route_health(h);
        ar.small = reinterpret_cast<const uint32_t*>(small);
        ar.snap = static_cast<uint32_t*>(sc.asnap[ak]);
        ar.seq = sc.n_async + 1;
        ar.zero = reinterpret_cast<uint32_t*>(small);
    }
    bool ar_done = false;
    if (!late && (rc = slots_copy_out(h, d_offsets, d_peers, d_msgs, capacity, async_end ? &ar : nullptr, &ar_done)))
        return rc;
    if (async_end) {
        if (!ar_done) {
            hipLaunchKernelGGL(k_async_result, dim3(1), dim3(256), 0, s, ar);
            WQ_HIP(h, hipGetLastError());
        }
        sc.acount++;
        sc.n_async++;
        sc.aseq[ak] = sc.n_async;
        sc.small_zeroed = true;
        sc.last_ready = false;  // no copy-out of an unread tick (its P is on the device)
        *n_pairs = 0;
        if (late) {  // st_host (the status copies' source) lives on this frame: let them finish first
            WQ_HIP(h, hipStreamSynchronize(s));
            h->err = late_msg;
            return late;
        }
        return WQ_OK;
    }

    // ---- the one host read: P, the statuses, the true sizes ----
    WQ_HIP(h, hipMemcpyAsync(sc.hsmall, small, small_used, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));
    const char* hs = static_cast<const char*>(sc.hsmall);
    const wq_route_counters* hcnt = reinterpret_cast<const wq_route_counters*>(hs + kSmallCnt);
    const TickPicture tp = fold_tick(sc, hs);
    if (late) {
        h->err = late_msg;
        return late;
    }
    if (tp.code) return status_error(h, tp.code, tp.code_from);
    if (tp.over) {  // every shard saw it: all of them redo the tick exactly
        *redo = true;
        return WQ_OK;
    }
    if (tp.bits) return status_error(h, (uint64_t)tp.bits << 32, tp.bits_from);
    const uint32_t err = hcnt[kCntScan].error | hcnt[kCntSelf].error | hcnt[kCntOwner].error;
    const uint64_t P = M ? hcnt[kCntScan].n_pairs : 0;
    sc.last_P = P;
    sc.last_ready = true;
    *n_pairs = P;
    if (err) return status_error(h, (uint64_t)err << 32, me);
    if (P > capacity) return set_error(h, WQ_E_CAPACITY, "sharded tick: output capacity too small (required size in *n_pairs)");
    return WQ_OK;
}

// ---- the owner form on budgeted slots (wq_sharded_route_owner_slots) ----
// Every message becomes a 20-byte slot of its owner's budgeted segment — this shard's own messages
// included (the self segment is a device copy) — and X1 {A, the slots} is the tick's only exchange:
// each owner routes what it received where it is (count_kernel<SLOTS>, the tile scan and
// emit_map_kernel over the received slots) and the pairs stay there (first
// option; area_map.rs:52-60 per slot). No claims, references, pools or second exchange. The budgets
// work as in the slot tick (the previous tick's true sizes + headroom, the first tick exact); a short
// budget anywhere reaches every shard through X1 (ShardIn::a_or) and all of them redo the tick
// exactly. One host read at the end: P, the statuses, the true sizes.
static int owner_emit(wq_router* h, uint64_t Rb, const TableView& tv, const AsyncResultParams* ar = nullptr,
                      bool* ar_done = nullptr) {
    ShardCtx& sc = *h->shard;
    RouteWs& rw = h->rws;
    hipStream_t s = h->stream;
    const uint32_t nto = (uint32_t)(Rb / kBlock);
    uint32_t* tiles = sc.otiles.as<uint32_t>();
    TileScanParams tp;
    tp.tile_total = tiles;
    tp.tile_F = tiles + nto;
    tp.tile_prefix = tiles + 2 * (uint64_t)nto;
    tp.n_tiles = nto;
    tp.offsets = sc.own_off.as<uint32_t>();
    tp.M = (uint32_t)Rb;
    tp.capacity = sc.own_cap;
    tp.cnt = reinterpret_cast<wq_route_counters*>(sc.small.as<char>() + kSmallCnt) + kCntScan;
    tp.health = nullptr;  // a short pair buffer is grown and emitted again, not an overflow
    tp.stale = tv.stale;
    if (ar) {  // an asynchronous tick: the scan ends it (if it is the one-block scan)
        tp.ar = *ar;
        tp.async_end = true;
    }
    if (int rc = launch_tile_scan(h, tp, ar_done)) return rc;
    EmitParams ep;
    ep.sender = sc.rslots.as<uint32_t>() + 3;  // OnlySelf rows: the slot's sender word
    ep.sender_stride = kSlotWords;
    ep.pos = nullptr;
    ep.repl = nullptr;
    ep.M = (uint32_t)Rb;
    ep.t = tv;
    ep.e = rw.e.as<uint32_t>();
    ep.tile_prefix = tp.tile_prefix;
    ep.count_tile = kBlock;
    ep.offsets = tp.offsets;
    ep.info = rw.info.as<uint2>();
    ep.peers = sc.own_peers.as<uint32_t>();
    ep.msgs = nullptr;  // the CSR over the received slots says whose each pair is
    ep.capacity = sc.own_cap;
    ep.n_blocks = nto;
    hipLaunchKernelGGL((emit_map_kernel<16>), dim3(pass_blocks(nto)), dim3(kBlock), 0, s, ep);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

static int owner_slot_tick(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                           const uint32_t* d_sender, const uint8_t* d_repl, size_t M, bool exact, int inject,
                           bool* redo, wq_owner_slot_view* out, bool async = false,
                           wq_route_counters* d_result = nullptr) {
    hipStream_t s = h->stream;
    ShardCtx& sc = *h->shard;
    const uint32_t G = sc.G, me = sc.rank;
    *redo = false;
    sc.last_ready = false;
    sc.last_slots = false;
    int late = WQ_OK;
    std::string late_msg;
    auto fail = [&](int rc) {
        if (rc && !late) {
            late = rc;
            late_msg = h->err;
        }
        return rc;
    };
    auto alloc = [&](DevBuf& b, size_t bytes) -> int {
        return b.ensure(bytes) == hipSuccess ? WQ_OK : set_error(h, WQ_E_OOM, "hipMalloc (sharded tick workspace)");
    };
    char* small = sc.small.as<char>();
    uint32_t* a_send = reinterpret_cast<uint32_t*>(small + kSmallA);
    uint32_t* a_recv = a_send + 2 * G;
    wq_route_counters* cnts = reinterpret_cast<wq_route_counters*>(small + kSmallCnt);
    const size_t small_used = kSmallCnt + 4 * sizeof(wq_route_counters);
    if (!sc.small_zeroed) WQ_HIP(h, hipMemsetAsync(small, 0, small_used, s));
    sc.small_zeroed = false;
    if (int rc = ensure_health(h)) return rc;
    if (exact) sc.n_exact++;
    else sc.n_budget++;
    std::vector<uint32_t> st_host(2 * G, 0);  // alive until the end-of-tick read
    auto put_status = [&](uint32_t* dst) -> int {
        for (uint32_t d = 0; d < G; ++d) st_host[2 * d + 1] = status_of(late);
        WQ_HIP(h, hipMemcpyAsync(dst, st_host.data(), 8 * G, hipMemcpyHostToDevice, s));
        return WQ_OK;
    };
    if (inject == 1) fail(set_error(h, WQ_E_INVALID, "injected failure at step 1 (test hook)"));
    if (h->radius > 0.0 && !late)
        fail(set_error(h, WQ_E_INVALID, "the owner form on slots has no radius filter (wq_sharded_route_owner_device has)"));
    if (!late) fail(table_resolve(h, false));
    const TableView tv = table_view(h);

    // ---- X1: A + the slots (every owner's segment budgeted, this shard's own included) ----
    std::vector<size_t> eight(G, 8);
    SlotLayout L{};
    SegBounds sb{}, rb{};
    int rc;
    if (exact) {  // the true counts first (A alone, read back): budgets = the counts, whole blocks
        SlotLayout inf{};
        for (uint32_t d = 0; d < G; ++d) inf.budget[d] = 0xFFFFFFFFu;
        if (!late)
            fail(launch_budget_slots(h, d_pos, d_keys, d_world, d_sender, d_repl, M, G, G, inf, nullptr, nullptr,
                                     a_send, 1, false, true));
        if (late && (rc = put_status(a_send))) return rc;
        Xfer x{{a_send}, {eight.data()}, {a_recv}, {eight.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
        uint32_t* hv = static_cast<uint32_t*>(sc.hsmall);
        WQ_HIP(h, hipMemcpyAsync(hv, a_send, 16 * G, hipMemcpyDeviceToHost, s));
        WQ_HIP(h, hipStreamSynchronize(s));
        for (uint32_t d = 0; d < G; ++d) {
            sc.b1_out[d] = whole_blocks(hv[2 * d]);
            sc.b1_in[d] = whole_blocks(hv[2 * G + 2 * d]);
        }
    }
    uint64_t so = 0, ro = 0;
    for (uint32_t d = 0; d < G; ++d) {
        L.base[d] = (uint32_t)so;
        L.budget[d] = sc.b1_out[d];
        sb.b[d] = (uint32_t)so;
        rb.b[d] = (uint32_t)ro;
        so += sc.b1_out[d];
        ro += sc.b1_in[d];
    }
    if (so >= (1ull << 31) || ro >= (1ull << 31)) return fatal_receive(h, "sharded tick: more than 2^31 slots");
    L.base[G] = sb.b[G] = (uint32_t)so;
    rb.b[G] = (uint32_t)ro;
    const uint64_t Sb = so, Rb = ro;
    if (alloc(sc.slots, (Sb + 2) * kSlotWords * 4) || alloc(sc.perm, (Sb + 2) * 4) ||
        alloc(sc.rslots, (Rb + 2) * kSlotWords * 4))
        return fatal_receive(h, "hipMalloc of the sharded tick's slots");
    // the self segment straight into the receive buffer (not through the exchange's self copy), except
    // with the caller's callback, which copies every segment itself
    const bool in_place = sc.kind != kXCallback;
    // ... and its A entry too, on a budgeted tick (the one-pass grouping's last block writes it)
    const bool a_in_place = in_place && !exact && M && !late && !getenv("WQ_DEBUG_SLOT_3PASS");
    uint32_t* a_self = a_in_place ? a_recv + 2 * me : nullptr;
    if (!late)
        fail(launch_budget_slots(h, d_pos, d_keys, d_world, d_sender, d_repl, M, G, in_place ? me : G, L,
                                 sc.slots.as<uint32_t>(), sc.perm.as<uint32_t>(), a_send, exact ? 2 : 3, false, true,
                                 in_place ? sc.rslots.as<uint32_t>() + (uint64_t)kSlotWords * rb.b[me] : nullptr,
                                 in_place ? sc.perm.as<uint32_t>() + L.base[me] : nullptr, nullptr, !exact,
                                 in_place ? L.budget[me] : 0xFFFFFFFFu, a_self));
    if (late) {  // nothing to send: tail slots everywhere
        WQ_HIP(h, hipMemsetAsync(sc.slots.p, 0, (Sb + 1) * kSlotWords * 4, s));
        WQ_HIP(h, hipMemsetAsync(sc.perm.p, 0xFF, (Sb + 1) * 4, s));
        if (!exact && (rc = put_status(a_send))) return rc;
    }
    std::vector<size_t> sbytes(G), rbytes(G);
    uint64_t sent = 0, recvd = 0;
    for (uint32_t d = 0; d < G; ++d) {
        sbytes[d] = (size_t)sc.b1_out[d] * kSlotWords * 4;
        rbytes[d] = (size_t)sc.b1_in[d] * kSlotWords * 4;
        if (d != me) {
            sent += 8 + sbytes[d];
            recvd += 8 + rbytes[d];
        }
    }
    if (exact) {
        Xfer x{{sc.slots.p}, {sbytes.data()}, {sc.rslots.p}, {rbytes.data()}, 1};
        x.skip_self[0] = in_place && !late;
        if ((rc = exchange(h, x))) return rc;
    } else {
        Xfer x{{a_send, sc.slots.p}, {eight.data(), sbytes.data()}, {a_recv, sc.rslots.p},
               {eight.data(), rbytes.data()}, 2};
        x.skip_self[0] = a_in_place && !late;
        x.skip_self[1] = in_place && !late;
        if ((rc = exchange(h, x))) return rc;
    }
    sc.last_sent = sent;
    sc.last_recv = recvd;

    // ---- the owner: count the received slots, the tile scan, the emit; the pairs stay here ----
    if (inject == 3) fail(set_error(h, WQ_E_INVALID, "injected failure at step 3 (test hook)"));
    RouteWs& rw = h->rws;
    const uint32_t nto = (uint32_t)(Rb / kBlock);  // whole blocks
    if (!sc.own_cap) sc.own_cap = std::min<uint64_t>(8 * Rb + 4096, 0xFFFFFFFFull);
    if (!late && (fail(alloc(rw.e, (Rb + 1) * 4)) || fail(alloc(rw.info, (Rb + 1) * 8)) ||
                  fail(alloc(sc.otiles, ((uint64_t)nto * 3 + 4) * 4)) || fail(alloc(sc.own_off, (Rb + 1) * 4)) ||
                  fail(alloc(sc.own_peers, sc.own_cap * 4)))) {
    }
    // the asynchronous end's snapshot (below), taken by the tile scan when one block runs it
    const bool async_end = async && !exact;
    AsyncResultParams ar{};
    const uint32_t ak = (sc.ahead + sc.acount) % ShardCtx::kRing;  // async_drain left a free slot
    if (async_end) {
        ar.a_recv = a_recv;
        ar.c_recv = reinterpret_cast<const uint32_t*>(small + kSmallC) + 2 * G;  // zero: no second exchange
        ar.G = G;
        ar.statuses = 1u;  // every segment budgeted, this shard's own included: G = 1 too
        ar.cnt = cnts;
        ar.has_msgs = Rb ? 1u : 0u;
        ar.capacity = sc.own_cap;
        ar.out = d_result;
        ar.health = route_health(h);
        ar.small = reinterpret_cast<const uint32_t*>(small);
        ar.snap = static_cast<uint32_t*>(sc.asnap[ak]);
        ar.seq = sc.n_async + 1;
        ar.zero = reinterpret_cast<uint32_t*>(small);
    }
    bool ar_done = false;
    if (!late && Rb) {
        CountParams cp{};
        cp.in = RouteIn{nullptr, nullptr, nullptr, nullptr, nullptr, (uint32_t)Rb, (int64_t)h->cube_size};
        cp.in.slots = sc.rslots.as<uint32_t>();
        cp.t = tv;
        cp.e = rw.e.as<uint32_t>();
        cp.info = rw.info.as<uint2>();
        cp.tile_total = sc.otiles.as<uint32_t>();
        cp.tile_F = cp.tile_total + nto;
        cp.cnt = cnts + kCntOwner;
        cp.cnt_next = cnts + kCntScratch;
        cp.health = route_health(h);
        cp.n_tiles = nto;
        hipLaunchKernelGGL((count_kernel<false, 1, 8, 0, false, true>), dim3(pass_blocks(nto)), dim3(kBlock), 0, s, cp);
        if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "count launch (owner form)"));
        if (!late) fail(owner_emit(h, Rb, tv, async_end && !late ? &ar : nullptr, &ar_done));
    }

    auto fill_view = [&](uint64_t P) {
        out->slots = sc.rslots.as<uint32_t>();
        out->offsets = sc.own_off.as<uint32_t>();
        out->peers = sc.own_peers.as<uint32_t>();
        out->send_perm = sc.perm.as<uint32_t>();
        out->n_slots = Rb;
        out->n_pairs = P;
        for (uint32_t d = 0; d <= G; ++d) {
            out->seg[d] = rb.b[d];
            out->send_seg[d] = sb.b[d];
        }
    };
    // ---- asynchronous end (a budgeted tick): as the slot tick's — the small vectors to a pinned
    // snapshot folded in two calls later, P and the statuses to the caller's counters and the health
    // words; a pair buffer that was short shows as overflow. A shard whose local step failed takes
    // it too, then returns its error (every shard queues the same ticks: ADVICE r5) ----
    if (async_end) {
        if (!Rb && !late) WQ_HIP(h, hipMemsetAsync(sc.own_off.p, 0, 4, s));
        if (!ar_done) {
            hipLaunchKernelGGL(k_async_result, dim3(1), dim3(256), 0, s, ar);
            WQ_HIP(h, hipGetLastError());
        }
        sc.acount++;
        sc.n_async++;
        sc.aseq[ak] = sc.n_async;
        sc.small_zeroed = true;
        if (late) {  // st_host (the status copies' source) lives on this frame: let them finish first
            WQ_HIP(h, hipStreamSynchronize(s));
            h->err = late_msg;
            return late;
        }
        fill_view(~0ull);  // P: in the caller's counters
        return WQ_OK;
    }

    // ---- the one host read ----
    WQ_HIP(h, hipMemcpyAsync(sc.hsmall, small, small_used, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));
    const char* hs = static_cast<const char*>(sc.hsmall);
    const wq_route_counters* hcnt = reinterpret_cast<const wq_route_counters*>(hs + kSmallCnt);
    const TickPicture tp = fold_tick(sc, hs, true);
    if (late) {
        h->err = late_msg;
        return late;
    }
    if (tp.code) return status_error(h, tp.code, tp.code_from);
    if (tp.over) {  // every shard saw it: all of them redo the tick exactly
        *redo = true;
        return WQ_OK;
    }
    if (tp.bits) return status_error(h, (uint64_t)tp.bits << 32, tp.bits_from);
    const uint32_t err = Rb ? (hcnt[kCntScan].error | hcnt[kCntOwner].error) : 0u;
    if (err) return status_error(h, (uint64_t)err << 32, me);
    const uint64_t P = Rb ? hcnt[kCntScan].n_pairs : 0;
    if (P > sc.own_cap) {  // the pair buffers were short: grow them and emit again (the rows are kept)
        sc.own_cap = std::min<uint64_t>(P + P / 4 + 4096, 0xFFFFFFFFull);
        if (alloc(sc.own_peers, sc.own_cap * 4)) return WQ_E_OOM;
        if ((rc = owner_emit(h, Rb, tv))) return rc;
        WQ_HIP(h, hipStreamSynchronize(s));
    }
    if (!Rb) WQ_HIP(h, hipMemsetAsync(sc.own_off.p, 0, 4, s));
    fill_view(P);
    return WQ_OK;
}

static int sharded_tick_slots(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                              const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                              uint32_t* d_peers, uint32_t* d_msgs, size_t capacity, size_t* n_pairs, bool async = false,
                              wq_route_counters* d_result = nullptr) {
    ShardCtx& sc = *h->shard;
    // earlier asynchronous ticks first: a synchronous tick folds them all in; an asynchronous one
    // keeps the latest in flight (its budgets come from the tick before), unless it must run exact
    if (sc.budget_form != 0) {  // the owner form's budgets include the self segment: run exact
        if (int rc = async_drain(h, 0)) return rc;
        sc.budgets = false;
        sc.budget_form = 0;
    } else if (int rc = async_drain(h, async && sc.budgets ? 1u : 0u)) {
        return rc;
    }
    const int inject = h->shard_inject;
    h->shard_inject = 0;
    bool redo = false;
    int rc = slot_tick(h, d_pos, d_keys, d_world, d_sender, d_repl, M, d_offsets, d_peers, d_msgs, capacity, n_pairs,
                       sc.G > 1 && !sc.budgets, inject, &redo, async, d_result);
    if (rc == WQ_OK && redo)
        rc = slot_tick(h, d_pos, d_keys, d_world, d_sender, d_repl, M, d_offsets, d_peers, d_msgs, capacity, n_pairs,
                       true, 0, &redo);
    // an asynchronous call that ran synchronously (exact, or a local failure) leaves its result in the
    // caller's counters all the same
    if (async && d_result && (rc == WQ_OK || rc == WQ_E_CAPACITY) && sc.last_ready) {
        wq_route_counters c{};
        c.n_pairs = *n_pairs;
        c.overflow = *n_pairs > capacity ? 1u : 0u;
        WQ_HIP(h, hipMemcpyAsync(d_result, &c, sizeof(c), hipMemcpyHostToDevice, h->stream));
        WQ_HIP(h, hipStreamSynchronize(h->stream));  // c lives on this stack frame
    }
    return rc;
}

int wq_sharded_route_tick_device(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                                 const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs, uint32_t* d_offsets,
                                 uint32_t* d_peers, uint32_t* d_msgs, size_t capacity, size_t* n_pairs) {
    if (!h || !d_offsets || !n_pairs || (n_msgs && (!d_world || !d_sender || !d_repl || (!d_pos && !d_keys))) ||
        (capacity && !d_peers))
        return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    WQ_HIP(h, hipSetDevice(h->device));
    if (capacity > 0xFFFFFFFFull) capacity = 0xFFFFFFFFull;
    hipStream_t s = h->stream;
    *n_pairs = 0;
    if (h->shard && !h->shard_expanded)
        return sharded_tick_slots(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, d_offsets, d_peers, d_msgs,
                                  capacity, n_pairs);
    if (!h->shard) {  // G = 1 without an exchange: the single-GPU tick, P read back
        int rc = launch_route(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, d_offsets, d_peers, d_msgs, capacity);
        if (rc) return rc;
        wq_route_counters c;
        WQ_HIP(h, hipMemcpyAsync(&c, h->rws.last, sizeof(c), hipMemcpyDeviceToHost, s));
        WQ_HIP(h, hipStreamSynchronize(s));
        *n_pairs = n_msgs ? c.n_pairs : 0;
        if (c.error & 4u) return set_error(h, WQ_E_TIMEOUT, "route look-back spin gave up");
        if (c.error) return set_error(h, WQ_E_CAPACITY, "more than 2^32-1 pairs in one tick");
        if (n_msgs && c.n_pairs > capacity) return set_error(h, WQ_E_CAPACITY, "output capacity too small");
        return WQ_OK;
    }
    ShardCtx& sc = *h->shard;
    const uint32_t G = sc.G, me = sc.rank;
    const size_t M = n_msgs;
    int late = WQ_OK;  // a local failure, reported once the tick's exchanges are complete
    std::string late_msg;
    auto fail = [&](int code) {
        if (code && !late) {
            late = code;
            late_msg = h->err;
        }
        return code;
    };
    uint64_t R = 0;
    SegBounds seg;
    int rc = shard_exchange_route(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, &R, &seg, &late, &late_msg);
    if (rc) return rc;
    std::vector<size_t> sixteen(G, 16);
    // 4. per-record counts; per source {pair count, status}, exchanged before any pair moves
    unsigned long long* pc_send = reinterpret_cast<unsigned long long*>(sc.small.as<char>() + kSmallC);
    unsigned long long* pc_recv = pc_send + 2 * G;
    if (!late) {
        hipLaunchKernelGGL(k_owner_counts, dim3((unsigned)((R + kBlock - 1) / kBlock) + 1), dim3(kBlock), 0, s,
                           sc.own_off.as<uint32_t>(), (uint32_t)R, seg, G, sc.own_e.as<uint32_t>(), pc_send,
                           R ? h->rws.last : nullptr, h->tab.stale.as<uint32_t>());
        if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "owner counts launch"));
    }
    std::vector<unsigned long long> pc_status(2 * G, 0);  // lives until host read 2 below
    if (late) {
        for (uint32_t d = 0; d < G; ++d) pc_status[2 * d + 1] = status_of(late);
        WQ_HIP(h, hipMemcpyAsync(pc_send, pc_status.data(), 16 * G, hipMemcpyHostToDevice, s));
    }
    {
        Xfer x{{pc_send}, {sixteen.data()}, {pc_recv}, {sixteen.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
    }
    std::vector<unsigned long long> hp(4 * G);
    WQ_HIP(h, hipMemcpyAsync(hp.data(), pc_send, 32 * G, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));  // host read 2
    uint64_t peer_status = 0, P_own = 0;
    uint32_t peer_from = 0;
    for (uint32_t d = 0; d < G; ++d) {
        P_own += hp[2 * d];
        const uint64_t st = hp[2 * G + 2 * d + 1];
        if (st && !peer_status) {
            peer_status = st;
            peer_from = d;
        }
    }
    if (!late && P_own > sc.own_cap) {  // the pair buffer was short: offsets are right, route again
        sc.own_cap = P_own + P_own / 4 + 4096;
        if (sc.own_cap > 0xFFFFFFFFull) sc.own_cap = 0xFFFFFFFFull;
        // the sizes are promised: a shard that cannot keep the promise breaks the collective
        if (sc.own_peers.ensure(sc.own_cap * 4) != hipSuccess) return fatal_receive(h, "hipMalloc of the owner's pairs");
        if ((rc = launch_route_records(h, sc.recv.as<wq_msg_rec>(), R, sc.own_off.as<uint32_t>(),
                                       sc.own_peers.as<uint32_t>(), nullptr, sc.own_cap)))
            return fatal_receive(h, "owner re-route");
    }
    // 5. recipient counts and peers back to the ingesting shards (one exchange group); a shard whose
    // local step failed sends none of either, as its status said
    std::vector<size_t> eb_s(G), eb_r(G), pb_s(G), pb_r(G);
    uint64_t P = 0;
    for (uint32_t d = 0; d < G; ++d) {
        const bool d_failed = (uint32_t)hp[2 * G + 2 * d + 1] != 0;
        eb_s[d] = late ? 0 : (size_t)sc.rc[d] * 4;      // to source d: e of the records it sent here
        eb_r[d] = d_failed ? 0 : (size_t)sc.sc[d] * 4;  // from owner d: e of the records sent there
        pb_s[d] = (size_t)hp[2 * d] * 4;
        pb_r[d] = (size_t)hp[2 * G + 2 * d] * 4;
        P += hp[2 * G + 2 * d];
    }
    if (sc.ret_e.ensure((M ? M : 1) * 4) != hipSuccess || sc.ret_peers.ensure((P ? P : 1) * 4) != hipSuccess)
        return fatal_receive(h, "hipMalloc of the returned pairs");
    sc.last_sent = sc.last_recv = 0;
    for (uint32_t d = 0; d < G; ++d)
        if (d != me) {
            sc.last_sent += 4 + (uint64_t)sc.sc[d] * sizeof(wq_msg_rec) + 16 + eb_s[d] + pb_s[d];
            sc.last_recv += 4 + (uint64_t)sc.rc[d] * sizeof(wq_msg_rec) + 16 + eb_r[d] + pb_r[d];
        }
    {
        Xfer x{{sc.own_e.p, sc.own_peers.p}, {eb_s.data(), pb_s.data()}, {sc.ret_e.p, sc.ret_peers.p},
               {eb_r.data(), pb_r.data()}, 2};
        if ((rc = exchange(h, x))) return rc;
    }
    (void)me;
    if (late) {
        h->err = late_msg;
        return late;
    }
    if (peer_status) return status_error(h, peer_status, peer_from);
    *n_pairs = P;
    if (P > 0xFFFFFFFFull) return set_error(h, WQ_E_CAPACITY, "more than 2^32-1 pairs in one tick");
    // 6. unshard into the caller's CSR, message order
    WQ_ALLOC(h, sc.ret_off, (M ? M : 1) * 4);
    if ((rc = scan_excl(h, sc.tmp, sc.ret_e.as<uint32_t>(), sc.ret_off.as<uint32_t>(), M))) return rc;
    sc.last_M = M;
    sc.last_P = P;
    sc.last_ready = true;
    return copy_out(h, d_offsets, d_peers, d_msgs, capacity);
}

int wq_sharded_route_tick_async(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                                const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs, uint32_t* d_offsets,
                                uint32_t* d_peers, uint32_t* d_msgs, size_t capacity, wq_route_counters* d_counters) {
    if (!h || !d_offsets || (n_msgs && (!d_world || !d_sender || !d_repl || (!d_pos && !d_keys))) ||
        (capacity && !d_peers))
        return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    if (!h->shard || h->shard_expanded)
        return set_error(h, WQ_E_INVALID, "wq_sharded_route_tick_async: no exchange attached, or the expanded form");
    WQ_HIP(h, hipSetDevice(h->device));
    if (capacity > 0xFFFFFFFFull) capacity = 0xFFFFFFFFull;
    size_t P = 0;
    return sharded_tick_slots(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, d_offsets, d_peers, d_msgs, capacity,
                              &P, true, d_counters);
}

int wq_sharded_route_owner_device(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                                  const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs, wq_owner_view* out) {
    if (!h || !out || (n_msgs && (!d_world || !d_sender || !d_repl || (!d_pos && !d_keys)))) return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    WQ_HIP(h, hipSetDevice(h->device));
    if (!h->shard) return set_error(h, WQ_E_INVALID, "no exchange attached (wq_shard_attach_*)");
    memset(out, 0, sizeof(*out));
    hipStream_t s = h->stream;
    ShardCtx& sc = *h->shard;
    int late = WQ_OK;
    std::string late_msg;
    uint64_t R = 0;
    SegBounds seg;
    int rc = shard_exchange_route(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, &R, &seg, &late, &late_msg);
    if (rc) return rc;
    if (late) {  // nothing else is exchanged in this form: report it now
        h->err = late_msg;
        return late;
    }
    // the pairs stay here (first option): only this shard's counters are read
    wq_route_counters c{};
    if (R) {
        WQ_HIP(h, hipMemcpyAsync(&c, h->rws.last, sizeof(c), hipMemcpyDeviceToHost, s));
        WQ_HIP(h, hipStreamSynchronize(s));
        if (c.error & 4u) return set_error(h, WQ_E_TIMEOUT, "owner route: look-back spin gave up");
        if (c.error) return set_error(h, WQ_E_CAPACITY, "owner route: more than 2^32-1 pairs");
        if (c.n_pairs > sc.own_cap) {  // the pair buffer was short: offsets are right, route again
            sc.own_cap = c.n_pairs + c.n_pairs / 4 + 4096;
            if (sc.own_cap > 0xFFFFFFFFull) sc.own_cap = 0xFFFFFFFFull;
            WQ_ALLOC(h, sc.own_peers, sc.own_cap * 4);
            if ((rc = launch_route_records(h, sc.recv.as<wq_msg_rec>(), R, sc.own_off.as<uint32_t>(),
                                           sc.own_peers.as<uint32_t>(), nullptr, sc.own_cap)))
                return rc;
        }
    }
    out->recs = sc.recv.as<wq_msg_rec>();
    out->offsets = sc.own_off.as<uint32_t>();
    out->peers = sc.own_peers.as<uint32_t>();
    out->n_recs = R;
    out->n_pairs = R ? c.n_pairs : 0;
    for (uint32_t d = 0; d <= sc.G; ++d) out->seg[d] = seg.b[d];
    return WQ_OK;
}

// Folds in earlier asynchronous ticks (all of them when the budgets' form changes: the ring then
// holds only one form's ticks), then one tick, redone exactly when a budget was short.
static int owner_slots_call(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                            const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs, wq_owner_slot_view* out,
                            bool async, wq_route_counters* d_result) {
    ShardCtx& sc = *h->shard;
    if (sc.budget_form != 1) {  // budgets of the slot tick leave out the self segment: run exact
        if (int rc = async_drain(h, 0)) return rc;
        sc.budgets = false;
        sc.budget_form = 1;
    } else if (int rc = async_drain(h, async && sc.budgets ? 1u : 0u)) {
        return rc;
    }
    const int inject = h->shard_inject;
    h->shard_inject = 0;
    bool redo = false;
    int rc = owner_slot_tick(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, !sc.budgets, inject, &redo, out,
                             async, d_result);
    if (rc == WQ_OK && redo)
        rc = owner_slot_tick(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, true, 0, &redo, out);
    // an asynchronous call that ran synchronously (exact, or redone) leaves its result in the
    // caller's counters all the same
    if (async && d_result && rc == WQ_OK && out->n_pairs != ~0ull) {
        wq_route_counters c{};
        c.n_pairs = out->n_pairs;
        WQ_HIP(h, hipMemcpyAsync(d_result, &c, sizeof(c), hipMemcpyHostToDevice, h->stream));
        WQ_HIP(h, hipStreamSynchronize(h->stream));  // c lives on this stack frame
    }
    return rc;
}

int wq_sharded_route_owner_slots(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                                 const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs,
                                 wq_owner_slot_view* out) {
    if (!h || !out || (n_msgs && (!d_world || !d_sender || !d_repl || (!d_pos && !d_keys)))) return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    WQ_HIP(h, hipSetDevice(h->device));
    if (!h->shard) return set_error(h, WQ_E_INVALID, "no exchange attached (wq_shard_attach_*)");
    memset(out, 0, sizeof(*out));
    return owner_slots_call(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, out, false, nullptr);
}

int wq_sharded_route_owner_slots_async(wq_router* h, const double* d_pos, const int64_t* d_keys,
                                       const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                                       size_t n_msgs, wq_route_counters* d_counters, wq_owner_slot_view* out) {
    if (!h || !out || (n_msgs && (!d_world || !d_sender || !d_repl || (!d_pos && !d_keys)))) return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    WQ_HIP(h, hipSetDevice(h->device));
    if (!h->shard) return set_error(h, WQ_E_INVALID, "no exchange attached (wq_shard_attach_*)");
    memset(out, 0, sizeof(*out));
    return owner_slots_call(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, out, true, d_counters);
}

int wq_sharded_copy_out(wq_router* h, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    if (!h || !d_offsets || (capacity && !d_peers)) return WQ_E_INVALID;
    if (!h->shard || !h->shard->last_ready) return set_error(h, WQ_E_INVALID, "no sharded tick to copy out");
    WQ_HIP(h, hipSetDevice(h->device));
    return copy_out(h, d_offsets, d_peers, d_msgs, capacity > 0xFFFFFFFFull ? 0xFFFFFFFFull : capacity);
}

int wq_shard_last_bytes(wq_router* h, uint64_t* sent, uint64_t* received) {
    if (!h || !sent || !received) return WQ_E_INVALID;
    *sent = h->shard ? h->shard->last_sent : 0;
    *received = h->shard ? h->shard->last_recv : 0;
    return WQ_OK;
}

int wq_shard_tick_stats(wq_router* h, uint64_t* exact, uint64_t* budgeted) {
    if (!h || !exact || !budgeted) return WQ_E_INVALID;
    *exact = h->shard ? h->shard->n_exact : 0;
    *budgeted = h->shard ? h->shard->n_budget : 0;
    return WQ_OK;
}

int wq_debug_inject_shard_failure(wq_router* h, int step) {
    if (!h || step < 0 || step > 3) return WQ_E_INVALID;
    h->shard_inject = step;
    return WQ_OK;
}

int wq_debug_set_shard_form(wq_router* h, int expanded) {
    if (!h) return WQ_E_INVALID;
    h->shard_expanded = expanded != 0;
    return WQ_OK;
}

}  // extern "C"
