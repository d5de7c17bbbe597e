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

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <rccl/rccl.h>
#include <rocprim/rocprim.hpp>

#include "route_count.hpp"
#include "route_gather.hpp"
#include "route_scan.hpp"

namespace wq {
int launch_shard_messages(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                          const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, wq_msg_rec* d_out,
                          uint32_t* d_counts);
int launch_shard_slots(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                       const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, uint32_t* d_slots,
                       uint32_t* d_perm, uint32_t* d_counts, uint32_t stride);
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
// The small exchange vectors (ShardCtx::small, allocated at attach): the slot counts exchange
// {slots, status} u32 x 2 per shard (send at kSmallA, receive after it), the pool-size exchange
// {pool words, 0, status, 0} u64 x 4 per shard (send at kSmallC, receive after it), and the
// message-side counters of a slot tick (kSmallCnt: P and the error bits, from its tile scan).
constexpr size_t kSmallA = 0, kSmallC = 1024, kSmallCnt = 5120, kSmallBytes = 8192;
static_assert(kSmallA + 4 * WQ_MAX_SHARDS * 4 <= kSmallC && kSmallC + 8 * WQ_MAX_SHARDS * 8 <= kSmallCnt &&
                  kSmallCnt + sizeof(wq_route_counters) <= kSmallBytes,
              "small exchange vector layout");

}  // namespace

// Record index bounds of each source shard's segment of the received records (kernel argument).
struct SegBounds {
    uint32_t b[WQ_MAX_SHARDS + 1];
};

// One exchange of n buffers: buffer k sends sbytes[k][d] bytes to rank d (segments contiguous in
// rank order from send[k]) and receives rbytes[k][s] from rank s into recv[k].
struct Xfer {
    const void* send[2];
    const size_t* sbytes[2];
    void* recv[2];
    const size_t* rbytes[2];
    int n;
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
    DevBuf slots, perm, rslots, ocnt, hslot, plen, poff, claim, lead, self_ref, ref_send, ref_recv, pool_send,
        pool_recv, desc_fill, desc_msg, e_msg, self_w, mtiles;
    uint64_t claim_cap = 0;  // claim table entries (power of two); 0 = not allocated
    uint64_t ticks = 0;      // slot ticks run: the claim table's tag
    // bytes this shard sent to / received from OTHER shards in its latest tick (xGMI volume)
    uint64_t last_sent = 0, last_recv = 0;
    // the latest tick, kept for wq_sharded_copy_out after WQ_E_CAPACITY
    uint64_t last_M = 0, last_P = 0;
    bool last_ready = false;
    bool last_slots = false;  // the latest tick was a slot tick (copy_out = scan + gather of desc_msg)
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
            if (x.sbytes[k][me])
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
        wq_hub& hub = *sc.hub;
        WQ_HIP(h, hipStreamSynchronize(s));  // this rank's send buffers are complete
        wq_hub::Post& mine = hub.post[me];
        mine.send = x.send;
        mine.sbytes = x.sbytes;
        mine.n = x.n;
        mine.device = h->device;
        if (!hub.barrier(kHubTimeoutS)) return set_error(h, WQ_E_RCCL, "hub exchange: a peer never arrived");
        int rc = WQ_OK;
        for (uint32_t src = 0; src < G && rc == WQ_OK; ++src) {
            const wq_hub::Post& p = hub.post[src];
            if (p.n != x.n) {
                rc = set_error(h, WQ_E_INVALID, "hub exchange: ranks disagree on the buffer count");
                break;
            }
            for (int k = 0; k < x.n; ++k) {
                const size_t bytes = p.sbytes[k][me];
                if (bytes != x.rbytes[k][src]) {
                    rc = set_error(h, WQ_E_INVALID, "hub exchange: send / receive sizes disagree");
                    break;
                }
                if (!bytes) continue;
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
        const hipError_t e = hipStreamSynchronize(s);  // done reading the peers' buffers ...
        if (!hub.barrier(kHubTimeoutS))                // ... before any of them reuses one
            return set_error(h, WQ_E_RCCL, "hub exchange: a peer never finished");
        if (rc) return rc;
        if (e != hipSuccess) return set_error(h, WQ_E_HIP, "hub exchange sync", e);
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

__device__ __forceinline__ uint32_t slot_cnt(const uint2 inf, uint32_t e, const uint32_t* list) {
    if (inf.x & kLocSelf) return e;
    if (inf.x & kLocGlobal) return list[inf.x & ~kLocGlobal];
    return inf.y == kNone ? 0u : inf.y >> 24;  // inline record, or no subscriber at all
}

// (owner, remote slots) the cube's peer count and the claim of the slot's (source, cube) pair: the
// first claimer ships the cube's peers in that source's pool, the others point at them.
__global__ __launch_bounds__(kBlock) void k_ref_claim(RefOwnerParams p) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t == p.n_rem) p.plen[t] = 0;
    if (t >= p.n_rem) return;
    const uint32_t i = t < p.self_lo ? t : t + p.n_self;  // the received slot
    const uint32_t s = seg_find(p.rrem, p.G, t);
    const uint2 inf = p.info[i];
    const uint32_t cnt = slot_cnt(inf, p.e[i], p.list);
    bool leader = false;
    uint64_t hs = 0;
    if (!(inf.x & kLocSelf) && cnt) {
        const unsigned long long key = ((unsigned long long)p.tag << 38) | ((unsigned long long)s << 32) | inf.x;
        uint64_t hv = ((uint64_t)inf.x | ((uint64_t)s << 32)) * 0x9E3779B97F4A7C15ull;
        hv ^= hv >> 29;
        hs = hv & p.cmask;
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

__device__ __forceinline__ void put_desc(uint4* desc_msg, uint32_t* e_msg, uint32_t m, uint32_t e, uint32_t skip,
                                         const uint32_t* src) {
    const uint64_t a = reinterpret_cast<uint64_t>(src);
    desc_msg[m] = make_uint4(e, skip, (uint32_t)a, (uint32_t)(a >> 32));
    e_msg[m] = e;
}

// (owner) the count pass over the received slots (route_count.hpp count_rows, one slot per lane).
// This shard's own slots — all of them at G = 1 — resolve right here into their messages'
// descriptors (pointers into the table): the ingesting side is this GPU, so nothing is staged and
// the record lines the count just read are still in the caches when the gather follows. A remote
// source's slot leaves its count and locator for the claim / reference kernels.
struct SlotCountParams {
    CountParams c;
    uint32_t self_lo, self_hi;  // this shard's own segment of the received slots
    const uint32_t* perm;       // sent slot -> message
    uint32_t self_sent;         // first sent slot of the own segment
    const uint32_t* sender;
    uint4* desc_msg;
    uint32_t* e_msg;
    uint32_t* self_w;
};

__global__ __launch_bounds__(kBlock, 8) void k_count_slots(SlotCountParams p) {
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && tid == 0) {
        p.c.cnt_next->n_pairs = 0;
        p.c.cnt_next->n_candidates = 0;
        p.c.cnt_next->overflow = 0;
        p.c.cnt_next->error = 0;
    }
    const uint32_t m0 = blockIdx.x * kBlock;
    uint64_t F_local = 0;
    uint32_t E_local = 0;
    uint32_t e_out[1];
    uint2 inf_out[1];
    count_rows<true, 1, 0, false, true>(p.c.in, p.c.t, m0, e_out, inf_out, F_local, E_local);
    const uint32_t i = m0 + tid;
    if (i >= p.c.in.M) return;
    if (i >= p.self_lo && i < p.self_hi) {
        const uint32_t m = p.perm[p.self_sent + (i - p.self_lo)];
        if (m == kNone) return;  // a tail slot
        uint32_t kind, off, skip;
        slot_row(inf_out[0], &kind, &off, &skip);
        const uint32_t e = e_out[0];
        if (kind == kRefSelf) {
            if (e) p.self_w[m] = p.sender[m];
            put_desc(p.desc_msg, p.e_msg, m, e, kNone, p.self_w + m);
        } else {
            put_desc(p.desc_msg, p.e_msg, m, e, skip == kRefSkipNone ? kNone : skip,
                     row_src(kind, off, p.c.t.list, p.c.t.recs));
        }
        return;
    }
    p.c.e[i] = e_out[0];
    p.c.info[i] = inf_out[0];
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

// (owner, G > 1) the per-destination words of the pool-size exchange: {pool words, 0, status, 0}.
// status = error bits of the count pass (8: stale table) << 32.
__global__ void k_ref_sizes(const uint32_t* __restrict__ poff, SegBounds rrem, uint32_t G,
                            const uint32_t* __restrict__ stale, unsigned long long* __restrict__ out) {
    const uint32_t d = threadIdx.x;
    if (d >= G) return;
    const uint32_t err = (stale && *stale) ? kErrStale : 0u;
    out[4 * d] = poff ? (unsigned long long)(poff[rrem.b[d + 1]] - poff[rrem.b[d]]) : 0ull;
    out[4 * d + 1] = 0;
    out[4 * d + 2] = (unsigned long long)err << 32;
    out[4 * d + 3] = 0;
}

struct ResolveParams {
    const uint32_t* perm;     // sent slot -> message (kNone: a tail slot)
    const uint32_t* sender;   // the caller's d_sender
    const uint3* ref_recv;    // references from the remote owners, in sent-slot order (own segment left out)
    uint32_t self_a, self_b;  // this shard's own segment of the sent slots
    SegBounds sseg;           // sent slots per owner
    uint32_t G, n;            // n = remote slots
    const uint32_t* pool;     // the pools received, owner after owner
    uint64_t pbase[WQ_MAX_SHARDS + 1];
    uint4* desc_msg;          // per message: {recipients, skip, pointer}
    uint32_t* e_msg;          // per message: recipients
    uint32_t* self_w;         // per message: the sender, for OnlySelf rows
};

// (ingesting GPU) per slot sent to a remote owner: the message's row descriptor, in message order.
__global__ __launch_bounds__(kBlock) void k_ref_resolve(ResolveParams p) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= p.n) return;
    const uint32_t k = t < p.self_a ? t : t + (p.self_b - p.self_a);  // the sent slot
    const uint32_t m = p.perm[k];
    if (m == kNone) return;  // the tail of a two-slot message
    const uint3 ref = p.ref_recv[t];
    const uint32_t kind = ref.z >> 30, sk = ref.z & kRefSkipNone;
    if (kind == kRefSelf) {
        if (ref.y) p.self_w[m] = p.sender[m];
        put_desc(p.desc_msg, p.e_msg, m, ref.y, kNone, p.self_w + m);
        return;
    }
    const uint32_t skip = sk == kRefSkipNone ? kNone : sk;
    const uint32_t e = ref.y - (skip != kNone ? 1u : 0u);
    put_desc(p.desc_msg, p.e_msg, m, e, skip, p.pool + p.pbase[seg_find(p.sseg, p.G, k)] + ref.x);
}

int attach(wq_router* h, uint32_t G, uint32_t rank) {
    if (!h || G == 0 || G > WQ_MAX_SHARDS || rank >= G) return WQ_E_INVALID;
    if (h->shard) return set_error(h, WQ_E_INVALID, "an exchange is already attached (wq_shard_detach first)");
    h->shard = new (std::nothrow) ShardCtx();
    if (!h->shard) return WQ_E_OOM;
    h->shard->G = G;
    h->shard->rank = rank;
    // the small exchange vectors live here for the handle's whole attachment: a tick never has to
    // allocate before its first exchange
    if (h->shard->small.ensure(kSmallBytes) != hipSuccess) {
        delete h->shard;
        h->shard = nullptr;
        return set_error(h, WQ_E_OOM, "hipMalloc of the shard exchange vectors");
    }
    return WQ_OK;
}

// The slot tick's CSR from its message-order descriptors (e_msg, desc_msg): per-256-message
// totals, the tile scan (offsets[M] = P, the counters at kSmallCnt: P, the overflow / error bits),
// then the rows gathered with their offsets (outputs beyond capacity are not written).
int slots_copy_out(wq_router* h, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    ShardCtx& sc = *h->shard;
    const uint64_t M = sc.last_M;
    hipStream_t s = h->stream;
    wq_route_counters* cnt = reinterpret_cast<wq_route_counters*>(sc.small.as<char>() + kSmallCnt);
    WQ_HIP(h, hipMemsetAsync(cnt, 0, sizeof(*cnt), s));
    if (M == 0) {
        WQ_HIP(h, hipMemsetAsync(d_offsets, 0, 4, s));
        return WQ_OK;
    }
    const uint32_t nt = (uint32_t)((M + kBlock - 1) / kBlock);
    WQ_ALLOC(h, sc.mtiles, (uint64_t)nt * 8);
    uint32_t* tile_total = sc.mtiles.as<uint32_t>();
    uint32_t* tile_prefix = tile_total + nt;
    hipLaunchKernelGGL(row_tile_sums_kernel, dim3(nt), dim3(kBlock), 0, s, sc.e_msg.as<uint32_t>(), (uint32_t)M,
                       tile_total);
    WQ_HIP(h, hipGetLastError());
    TileScanParams tp;
    tp.tile_total = tile_total;
    tp.tile_F = tile_total;  // no candidate count on this path: F is reported as P
    tp.tile_prefix = tile_prefix;
    tp.n_tiles = nt;
    tp.offsets = d_offsets;
    tp.M = (uint32_t)M;
    tp.capacity = capacity;
    tp.cnt = cnt;
    tp.health = h->rws.buf.p ? route_health(h) : nullptr;
    tp.stale = h->tab.stale.as<uint32_t>();  // error bit 8: the table still misses a device batch
    if (int rc = launch_tile_scan(h, tp)) return rc;
    GatherParams gp{nullptr, sc.desc_msg.as<uint4>(), (uint32_t)M, capacity ? d_peers : nullptr, d_msgs, capacity};
    gp.e = sc.e_msg.as<uint32_t>();
    gp.tile_prefix = tile_prefix;
    gp.offsets = d_offsets;
    hipLaunchKernelGGL((gather_rows_kernel<16, true>), dim3(nt), dim3(kBlock), 0, s, gp);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

// Unshard the latest tick into the caller's buffers (message order).
int copy_out(wq_router* h, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    ShardCtx& sc = *h->shard;
    const uint64_t M = sc.last_M, P = sc.last_P;
    hipStream_t s = h->stream;
    if (sc.last_slots) {
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
    DevBuf* bufs[] = {&sc->recs,     &sc->recv,      &sc->cnt2,     &sc->pc,        &sc->own_off,  &sc->own_peers,
                      &sc->own_e,    &sc->ret_e,     &sc->ret_off,  &sc->ret_peers, &sc->by_msg,   &sc->tmp,
                      &sc->small,    &sc->slots,     &sc->perm,     &sc->rslots,    &sc->ocnt,     &sc->hslot,
                      &sc->plen,     &sc->poff,      &sc->claim,    &sc->lead,      &sc->self_ref, &sc->ref_send,
                      &sc->ref_recv, &sc->pool_send, &sc->pool_recv, &sc->desc_fill, &sc->desc_msg, &sc->e_msg,
                      &sc->self_w,   &sc->mtiles};
    for (DevBuf* b : bufs) b->release();
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

// The slot tick (radius filter off): wq_sharded_route_tick_device's result with
//   A   {slots, status} per owner                                        (host read 1)
//   B   the compact slots (20 B per regular message)
//   C   {pool words, recipients, status} per source                     (host read 2)
//   D   per slot a 12-byte row reference, and per source ONE copy of every cube its messages hit
// so a long list crosses xGMI once per (tick, destination) instead of once per message; the
// ingesting GPU gathers the CSR itself. G = 1 skips the exchanges and reads P back at the end.
// Local failures keep the collective going: a failed shard step sends zero-sized segments with its
// status, every shard sees every status and all of them return the error after exchange D.
static int sharded_tick_slots(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                              const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                              uint32_t* d_peers, uint32_t* d_msgs, size_t capacity, size_t* n_pairs) {
    hipStream_t s = h->stream;
    ShardCtx& sc = *h->shard;
    const uint32_t G = sc.G, me = sc.rank;
    sc.last_ready = false;
    sc.last_slots = true;
    const int inject = h->shard_inject;
    h->shard_inject = 0;
    int late = WQ_OK;
    std::string late_msg;
    auto fail = [&](int rc) {
        if (rc && !late) {
            late = rc;
            late_msg = h->err;
        }
        return rc;
    };
    char* small = sc.small.as<char>();
    uint32_t* a_send = reinterpret_cast<uint32_t*>(small + kSmallA);
    uint32_t* a_recv = a_send + 2 * G;
    unsigned long long* c_send = reinterpret_cast<unsigned long long*>(small + kSmallC);
    unsigned long long* c_recv = c_send + 4 * G;
    auto alloc = [&](DevBuf& b, size_t bytes) -> int {
        return b.ensure(bytes) == hipSuccess ? WQ_OK : set_error(h, WQ_E_OOM, "hipMalloc (sharded tick workspace)");
    };

    // ---- 1. the M-sized buffers, then the slots grouped by owner ----
    const uint64_t slot_cap = 2 * (uint64_t)M + 1;
    WQ_HIP(h, hipMemsetAsync(small, 0, kSmallCnt, s));  // counts and statuses
    if (inject == 1) fail(set_error(h, WQ_E_INVALID, "injected failure at step 1 (test hook)"));
    if (!late && !fail(alloc(sc.slots, slot_cap * kSlotWords * 4)) && !fail(alloc(sc.perm, slot_cap * 4)) &&
        !fail(alloc(sc.desc_msg, (M + 1) * 16)) && !fail(alloc(sc.e_msg, (M + 1) * 4)) &&
        !fail(alloc(sc.self_w, (M + 1) * 4)))
        fail(launch_shard_slots(h, d_pos, d_keys, d_world, d_sender, d_repl, M, G, sc.slots.as<uint32_t>(),
                                sc.perm.as<uint32_t>(), a_send, 2));
    // host sources of status copies live until the call's host reads have synchronised the stream
    std::vector<uint32_t> a_status(2 * G, 0);
    std::vector<unsigned long long> c_status(4 * G, 0);
    if (late) {  // nothing to send: zero slots everywhere, and the status
        for (uint32_t d = 0; d < G; ++d) a_status[2 * d + 1] = status_of(late);
        WQ_HIP(h, hipMemcpyAsync(a_send, a_status.data(), 8 * G, hipMemcpyHostToDevice, s));
    }
    std::vector<size_t> eight(G, 8), thirty2(G, 32);
    int rc;
    if (G > 1) {
        Xfer x{{a_send}, {eight.data()}, {a_recv}, {eight.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
    }
    std::vector<uint32_t> av(4 * G);
    WQ_HIP(h, hipMemcpyAsync(av.data(), a_send, (G > 1 ? 16 : 8) * G, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));  // host read 1
    if (G == 1) av[2] = av[0], av[3] = av[1];
    std::vector<uint64_t> n_out(G), n_in(G);
    uint64_t peer_status = 0;
    uint32_t peer_from = 0;
    SegBounds sseg, rseg, rrem;
    sseg.b[0] = rseg.b[0] = rrem.b[0] = 0;
    uint64_t R = 0, S = 0, Rr = 0;
    for (uint32_t d = 0; d < G; ++d) {
        n_out[d] = av[2 * d];
        n_in[d] = av[2 * G + 2 * d];
        if (av[2 * G + 2 * d + 1] && !peer_status) {
            peer_status = av[2 * G + 2 * d + 1];
            peer_from = d;
        }
        S += n_out[d];
        R += n_in[d];
        if (d != me) Rr += n_in[d];
        sseg.b[d + 1] = (uint32_t)S;
        rseg.b[d + 1] = (uint32_t)R;
        rrem.b[d + 1] = (uint32_t)Rr;  // the remote slots, own segment left out
    }
    if (R >= 0xFFFFFC00ull) return fatal_receive(h, "more than 2^32 - 1024 slots on one owner");
    const uint64_t n_self = n_in[me], R_remote = R - n_self, S_remote = S - n_out[me];

    // ---- 2. the slots ----
    const uint32_t* rslots = sc.slots.as<uint32_t>();
    if (G > 1) {
        if (alloc(sc.rslots, (R ? R : 1) * kSlotWords * 4)) return fatal_receive(h, "hipMalloc of the received slots");
        std::vector<size_t> sb(G), rb(G);
        for (uint32_t d = 0; d < G; ++d) {
            sb[d] = n_out[d] * kSlotWords * 4;
            rb[d] = n_in[d] * kSlotWords * 4;
        }
        Xfer x{{sc.slots.p}, {sb.data()}, {sc.rslots.p}, {rb.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
        rslots = sc.rslots.as<uint32_t>();
    }

    // ---- 3. the owner: count (local_message.rs:52-86 per slot; own slots resolved in place),
    //         then the remote slots' claims, pools and references ----
    if (inject == 3) fail(set_error(h, WQ_E_INVALID, "injected failure at step 3 (test hook)"));
    // fold in a finished incremental batch first (it may rebuild the table the view points into)
    if (!late) fail(table_resolve(h, false));
    const TableView tv = table_view(h);
    wq_route_counters *cur = nullptr, *nxt = nullptr;
    if (!late && R) fail(route_counters(h, R, nullptr, &cur, &nxt));
    if (!late && R) {
        RouteWs& rw = h->rws;
        if (!fail(alloc(rw.e, R * 4)) && !fail(alloc(rw.info, R * 8)) &&
            (!R_remote || (!fail(alloc(sc.ocnt, R_remote * 4)) && !fail(alloc(sc.hslot, R_remote * 4)) &&
                           !fail(alloc(sc.plen, (R_remote + 1) * 4)) && !fail(alloc(sc.poff, (R_remote + 1) * 4)) &&
                           !fail(alloc(sc.desc_fill, (R_remote + 1) * 16)) &&
                           !fail(alloc(sc.ref_send, (R_remote + 1) * 12))))) {
            SlotCountParams cp{};
            cp.c.in = RouteIn{nullptr, nullptr, nullptr, nullptr, nullptr, (uint32_t)R, (int64_t)h->cube_size};
            cp.c.in.slots = rslots;
            cp.c.t = tv;
            cp.c.e = rw.e.as<uint32_t>();
            cp.c.info = rw.info.as<uint2>();
            cp.c.cnt = cur;
            cp.c.cnt_next = nxt;
            cp.c.health = route_health(h);
            cp.self_lo = rseg.b[me];
            cp.self_hi = rseg.b[me + 1];
            cp.perm = sc.perm.as<uint32_t>();
            cp.self_sent = sseg.b[me];
            cp.sender = d_sender;
            cp.desc_msg = sc.desc_msg.as<uint4>();
            cp.e_msg = sc.e_msg.as<uint32_t>();
            cp.self_w = sc.self_w.as<uint32_t>();
            hipLaunchKernelGGL(k_count_slots, dim3((unsigned)((R + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, cp);
            if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "count launch (sharded tick)"));
        }
        uint64_t C = 0;
        if (!late && R_remote) {  // claim table: load <= 1/2
            C = 1024;
            while (C < 2 * R_remote) C <<= 1;
            if (C > sc.claim_cap) {
                if (!fail(alloc(sc.claim, C * 8)) && !fail(alloc(sc.lead, C * 4))) {
                    if (hipMemsetAsync(sc.claim.p, 0, C * 8, s) != hipSuccess) fail(set_error(h, WQ_E_HIP, "memset"));
                    sc.claim_cap = C;
                }
            } else {
                C = sc.claim_cap;
            }
        }
        if (!late && R_remote) {
            const uint64_t period = (1ull << kRefClaimTagBits) - 1;
            if (sc.ticks && sc.ticks % period == 0 && hipMemsetAsync(sc.claim.p, 0, sc.claim_cap * 8, s) != hipSuccess)
                fail(set_error(h, WQ_E_HIP, "memset"));  // the tags wrap: forget them all
            RefOwnerParams rp{};
            rp.e = rw.e.as<uint32_t>();
            rp.info = rw.info.as<uint2>();
            rp.list = tv.list;
            rp.recs = tv.recs;
            rp.rrem = rrem;
            rp.G = G;
            rp.n_rem = (uint32_t)R_remote;
            rp.self_lo = rseg.b[me];
            rp.n_self = (uint32_t)n_self;
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
            hipLaunchKernelGGL(k_ref_claim, dim3((unsigned)((R_remote + kBlock) / kBlock)), dim3(kBlock), 0, s, rp);
            if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "claim launch (sharded tick)"));
            if (!late) fail(scan_excl(h, sc.tmp, sc.plen.as<uint32_t>(), sc.poff.as<uint32_t>(), R_remote + 1));
            if (!late) {
                hipLaunchKernelGGL(k_ref_make, dim3((unsigned)((R_remote + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rp);
                if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "reference launch (sharded tick)"));
            }
        }
    }

    // ---- 4. pool sizes, then the references and pools (G > 1) ----
    std::vector<unsigned long long> cv(8 * G, 0);
    std::vector<uint64_t> pbase(G + 1, 0);
    uint64_t sent = 0, recvd = 0;
    if (G > 1) {
        if (!late) {
            hipLaunchKernelGGL(k_ref_sizes, dim3(1), dim3(64), 0, s, R_remote ? sc.poff.as<uint32_t>() : nullptr, rrem,
                               G, tv.stale, c_send);
            if (hipGetLastError() != hipSuccess) fail(set_error(h, WQ_E_HIP, "size launch (sharded tick)"));
        }
        if (late) {  // nothing routed here: zero sizes and the status
            for (uint32_t d = 0; d < G; ++d) c_status[4 * d + 2] = status_of(late);
            WQ_HIP(h, hipMemcpyAsync(c_send, c_status.data(), 32 * G, hipMemcpyHostToDevice, s));
        }
        {
            Xfer x{{c_send}, {thirty2.data()}, {c_recv}, {thirty2.data()}, 1};
            if ((rc = exchange(h, x))) return rc;
        }
        WQ_HIP(h, hipMemcpyAsync(cv.data(), c_send, 64 * G, hipMemcpyDeviceToHost, s));
        WQ_HIP(h, hipStreamSynchronize(s));  // host read 2
        std::vector<uint64_t> pool_out(G), pool_in(G);
        uint64_t pool_out_total = 0, pool_in_total = 0;
        for (uint32_t d = 0; d < G; ++d) {
            pool_out[d] = cv[4 * d];
            pool_in[d] = cv[4 * G + 4 * d];
            const uint64_t st = cv[4 * G + 4 * d + 2];
            if (st && !peer_status) {
                peer_status = st;
                peer_from = d;
            }
            pool_out_total += pool_out[d];
            pbase[d] = pool_in_total;
            pool_in_total += pool_in[d];
        }
        pbase[G] = pool_in_total;
        if (alloc(sc.pool_send, (pool_out_total + 1) * 4)) return fatal_receive(h, "hipMalloc of the pools to send");
        if (alloc(sc.pool_recv, (pool_in_total + 1) * 4) || alloc(sc.ref_recv, (S_remote + 1) * 12))
            return fatal_receive(h, "hipMalloc of the references / pools to receive");
        if (!late && R_remote && pool_out_total) {
            GatherParams gp{sc.poff.as<uint32_t>(), sc.desc_fill.as<uint4>(), (uint32_t)R_remote,
                            sc.pool_send.as<uint32_t>(), nullptr, pool_out_total};
            hipLaunchKernelGGL((gather_rows_kernel<16, false>), dim3((unsigned)((R_remote + kBlock - 1) / kBlock)),
                               dim3(kBlock), 0, s, gp);
            if (hipGetLastError() != hipSuccess) return fatal_receive(h, "pool gather launch");
        }
        std::vector<size_t> rs(G), rr(G), ps(G), pr(G);
        for (uint32_t d = 0; d < G; ++d) {
            rs[d] = d == me || late ? 0 : n_in[d] * 12;  // references for the slots d sent here
            // a shard whose local step failed (a WQ_E_* code in its status) sends no references
            rr[d] = d == me || (uint32_t)cv[4 * G + 4 * d + 2] != 0 ? 0 : n_out[d] * 12;
            ps[d] = late ? 0 : pool_out[d] * 4;
            pr[d] = pool_in[d] * 4;
            if (d != me) {
                sent += 8 + n_out[d] * kSlotWords * 4 + 32 + rs[d] + ps[d];
                recvd += 8 + n_in[d] * kSlotWords * 4 + 32 + rr[d] + pr[d];
            }
        }
        Xfer x{{sc.ref_send.p, sc.pool_send.p}, {rs.data(), ps.data()}, {sc.ref_recv.p, sc.pool_recv.p},
               {rr.data(), pr.data()}, 2};
        if ((rc = exchange(h, x))) return rc;
    }
    sc.last_sent = sent;
    sc.last_recv = recvd;
    if (late) {
        h->err = late_msg;
        return late;
    }
    if (peer_status) return status_error(h, peer_status, peer_from);

    // ---- 5. the ingesting side: remote references -> descriptors, then the CSR ----
    if (S_remote) {
        ResolveParams rp{};
        rp.perm = sc.perm.as<uint32_t>();
        rp.sender = d_sender;
        rp.ref_recv = sc.ref_recv.as<uint3>();
        rp.self_a = sseg.b[me];
        rp.self_b = sseg.b[me + 1];
        rp.sseg = sseg;
        rp.G = G;
        rp.n = (uint32_t)S_remote;
        rp.pool = sc.pool_recv.as<uint32_t>();
        for (uint32_t d = 0; d <= G; ++d) rp.pbase[d] = pbase[d];
        rp.desc_msg = sc.desc_msg.as<uint4>();
        rp.e_msg = sc.e_msg.as<uint32_t>();
        rp.self_w = sc.self_w.as<uint32_t>();
        hipLaunchKernelGGL(k_ref_resolve, dim3((unsigned)((S_remote + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rp);
        WQ_HIP(h, hipGetLastError());
    }
    sc.last_M = M;
    sc.last_ready = true;
    if ((rc = slots_copy_out(h, d_offsets, d_peers, d_msgs, capacity))) return rc;
    // P and the error bits: the message-side tile scan's counters and the count pass's, read once
    // the tick has run (the one host wait after the exchanges)
    wq_route_counters c[2];
    WQ_HIP(h, hipMemcpyAsync(&c[0], small + kSmallCnt, sizeof(c[0]), hipMemcpyDeviceToHost, s));
    if (cur) WQ_HIP(h, hipMemcpyAsync(&c[1], cur, sizeof(c[1]), hipMemcpyDeviceToHost, s));
    else c[1] = wq_route_counters{};
    WQ_HIP(h, hipStreamSynchronize(s));
    const uint32_t err = c[0].error | c[1].error;
    const uint64_t P = M ? c[0].n_pairs : 0;
    sc.last_P = P;
    *n_pairs = P;
    if (err) return status_error(h, (uint64_t)err << 32, me);
    if (P > capacity) return set_error(h, WQ_E_CAPACITY, "sharded tick: output capacity too small (required size in *n_pairs)");
    return WQ_OK;
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
    if (h->shard && !(h->radius > 0.0) && !h->shard_expanded)
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
