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

#include "route_common.hpp"

namespace wq {
int launch_shard_messages(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                          const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, wq_msg_rec* d_out,
                          uint32_t* d_counts);
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
    // workspace
    DevBuf recs, recv, cnt2, pc, own_off, own_peers, own_e, ret_e, ret_off, ret_peers, by_msg, tmp, small;
    uint64_t own_cap = 0;
    std::vector<uint32_t> sc, rc;
    std::vector<uint64_t> ps, pr;
    // the latest tick, kept for wq_sharded_copy_out after WQ_E_CAPACITY
    uint64_t last_M = 0, last_P = 0;
    bool last_ready = false;
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

// per received record: its recipient count; per source segment: its pair count
__global__ void k_owner_counts(const uint32_t* __restrict__ off, uint32_t R, SegBounds seg, uint32_t G,
                               uint32_t* __restrict__ e, uint64_t* __restrict__ pc) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < R) e[i] = off[i + 1] - off[i];
    if (blockIdx.x == 0 && threadIdx.x < G) pc[threadIdx.x] = (uint64_t)off[seg.b[threadIdx.x + 1]] - off[seg.b[threadIdx.x]];
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

int attach(wq_router* h, uint32_t G, uint32_t rank) {
    if (!h || G == 0 || G > WQ_MAX_SHARDS || rank >= G) return WQ_E_INVALID;
    if (h->shard) return set_error(h, WQ_E_INVALID, "an exchange is already attached (wq_shard_detach first)");
    h->shard = new (std::nothrow) ShardCtx();
    if (!h->shard) return WQ_E_OOM;
    h->shard->G = G;
    h->shard->rank = rank;
    return WQ_OK;
}

// Unshard the latest tick into the caller's buffers (message order).
int copy_out(wq_router* h, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    ShardCtx& sc = *h->shard;
    const uint64_t M = sc.last_M, P = sc.last_P;
    hipStream_t s = h->stream;
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
    DevBuf* bufs[] = {&sc->recs, &sc->recv, &sc->cnt2, &sc->pc, &sc->own_off, &sc->own_peers, &sc->own_e,
                      &sc->ret_e, &sc->ret_off, &sc->ret_peers, &sc->by_msg, &sc->tmp, &sc->small};
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
    int& late = *late_out;  // a local failure, reported once the tick's exchanges are complete
    std::string& late_msg = *late_msg_out;

    // 1. shard
    WQ_ALLOC(h, sc.recs, (M ? M : 1) * sizeof(wq_msg_rec));
    WQ_ALLOC(h, sc.cnt2, 2 * G * 4);
    uint32_t* cnt_send = sc.cnt2.as<uint32_t>();
    uint32_t* cnt_recv = cnt_send + G;
    int rc = launch_shard_messages(h, d_pos, d_keys, d_world, d_sender, d_repl, M, G, sc.recs.as<wq_msg_rec>(),
                                   cnt_send);
    if (rc) return rc;  // nothing exchanged yet: every rank's failure here is local and symmetric-safe
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
    if (R >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "more than 2^32 - 1024 records on one owner");
    WQ_ALLOC(h, sc.recv, (R ? R : 1) * sizeof(wq_msg_rec));
    {
        Xfer x{{sc.recs.p}, {sb.data()}, {sc.recv.p}, {rb.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
    }
    // 3. route what this shard owns
    WQ_ALLOC(h, sc.own_off, (R + 1) * 4);
    if (!sc.own_cap) {
        sc.own_cap = 16 * R + 4096;
        if (sc.own_cap > 0xFFFFFFFFull) sc.own_cap = 0xFFFFFFFFull;
    }
    WQ_ALLOC(h, sc.own_peers, sc.own_cap * 4);
    rc = launch_route_records(h, sc.recv.as<wq_msg_rec>(), R, sc.own_off.as<uint32_t>(), sc.own_peers.as<uint32_t>(),
                              nullptr, sc.own_cap);
    if (rc) {  // keep the collective going with empty results
        late = rc;
        late_msg = h->err;
        WQ_HIP(h, hipMemsetAsync(sc.own_off.p, 0, (R + 1) * 4, s));
    }
    *R_out = R;
    *seg_out = seg;
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
    uint64_t R = 0;
    SegBounds seg;
    int rc = shard_exchange_route(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, &R, &seg, &late, &late_msg);
    if (rc) return rc;
    std::vector<size_t> eight(G, 8);
    // 4. per-record counts, per-source pair counts, exchanged
    WQ_ALLOC(h, sc.own_e, (R ? R : 1) * 4);
    WQ_ALLOC(h, sc.pc, 2 * G * 8 + sizeof(wq_route_counters));
    uint64_t* pc_send = sc.pc.as<uint64_t>();
    uint64_t* pc_recv = pc_send + G;
    wq_route_counters* cnt_copy = reinterpret_cast<wq_route_counters*>(pc_recv + G);
    hipLaunchKernelGGL(k_owner_counts, dim3((unsigned)((R + kBlock - 1) / kBlock) + 1), dim3(kBlock), 0, s,
                       sc.own_off.as<uint32_t>(), (uint32_t)R, seg, G, sc.own_e.as<uint32_t>(), pc_send);
    WQ_HIP(h, hipGetLastError());
    if (!late && R) WQ_HIP(h, hipMemcpyAsync(cnt_copy, h->rws.last, sizeof(wq_route_counters), hipMemcpyDeviceToDevice, s));
    else WQ_HIP(h, hipMemsetAsync(cnt_copy, 0, sizeof(wq_route_counters), s));
    {
        Xfer x{{pc_send}, {eight.data()}, {pc_recv}, {eight.data()}, 1};
        if ((rc = exchange(h, x))) return rc;
    }
    std::vector<uint64_t> hp(2 * G + 3);
    WQ_HIP(h, hipMemcpyAsync(hp.data(), pc_send, 2 * G * 8 + sizeof(wq_route_counters), hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));  // host read 2
    wq_route_counters oc;
    memcpy(&oc, hp.data() + 2 * G, sizeof(oc));
    if (!late && oc.error) {
        late = (oc.error & 4u) ? WQ_E_TIMEOUT : WQ_E_CAPACITY;
        late_msg = (oc.error & 4u) ? "owner route: look-back spin gave up" : "owner route: more than 2^32-1 pairs";
    }
    const uint64_t P_own = R ? oc.n_pairs : 0;
    if (!late && P_own > sc.own_cap) {  // the pair buffer was short: offsets are right, route again
        sc.own_cap = P_own + P_own / 4 + 4096;
        if (sc.own_cap > 0xFFFFFFFFull) sc.own_cap = 0xFFFFFFFFull;
        WQ_ALLOC(h, sc.own_peers, sc.own_cap * 4);
        rc = launch_route_records(h, sc.recv.as<wq_msg_rec>(), R, sc.own_off.as<uint32_t>(),
                                  sc.own_peers.as<uint32_t>(), nullptr, sc.own_cap);
        if (rc) {
            late = rc;
            late_msg = h->err;
        }
    }
    // 5. recipient counts and peers back to the ingesting shards (one exchange group)
    std::vector<size_t> eb_s(G), eb_r(G), pb_s(G), pb_r(G);
    uint64_t P = 0;
    for (uint32_t d = 0; d < G; ++d) {
        eb_s[d] = (size_t)sc.rc[d] * 4;  // to source d: e of the records it sent here
        eb_r[d] = (size_t)sc.sc[d] * 4;  // from owner d: e of the records sent there
        pb_s[d] = (size_t)hp[d] * 4;
        pb_r[d] = (size_t)hp[G + d] * 4;
        P += hp[G + d];
    }
    WQ_ALLOC(h, sc.ret_e, (M ? M : 1) * 4);
    WQ_ALLOC(h, sc.ret_peers, (P ? P : 1) * 4);
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

}  // extern "C"
