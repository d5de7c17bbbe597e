// wq_multi.hip — ONE handle over G GPUs (wq_router_create(cube_size, n_gpus,
// devices, ...)), the reference's one-owner model kept at the boundary.
//
// The reference owns one WorldMap in one task (worldql_server/src/processing/thread.rs:119, driven
// by the select! loop at :122-146). wq_router_create_multi gives that task one handle again: inside,
// G shard handles (one per device, cube-hash owners, wq_sharded.hip) attached to an in-process hub,
// and G worker threads — one per shard, since a sharded tick is collective — that the calling thread
// hands each call to and waits for. What a call does on the multi handle:
//   wq_apply_ops / _device, wq_remove_peers   every shard gets the whole op stream and keeps what it
//                                             owns (+ every REMOVE_PEER): wq_sharded_apply_ops
//   wq_route_tick / _device                   the messages split in G contiguous slices, one per
//                                             shard, routed by the sharded tick (owners anywhere),
//                                             the G CSRs concatenated into the caller's in message
//                                             order: exactly the one-table result
//   wq_is_subscribed                          every shard answers, OR (only the owner can hold it)
//   wq_is_subscribed_any, wq_world_peers,     the shards' any-keys (world << 32 | peer) merged
//   wq_route_global[_device], wq_get_stats    (sort + unique) into the handle's own any-keys on
//                                             devices[0], then the single-GPU kernels on them
//   radius filter / peer positions / hint     forwarded to every shard
// Device-pointer calls take their arrays on devices[0] and are synchronous on return.
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "wq_internal.hpp"

namespace wq {

struct MultiCtx {
    uint32_t G = 0;
    std::vector<int> dev;
    std::vector<wq_router*> sub;
    wq_hub* hub = nullptr;
    // per shard, on its device: staged inputs and outputs of a tick
    std::vector<DevBuf> in, out;
    std::vector<uint64_t> cap, P;
    bool any_dirty = true;  // the merged any-keys need rebuilding (an op was applied since)
    DevBuf tmp, cnt;        // merge scratch (devices[0])
    // worker pool: worker g runs task(g) on device dev[g]
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable go, done;
    std::function<int(uint32_t)> task;
    uint64_t gen = 0;
    uint32_t busy = 0;
    bool stop = false;
    std::vector<int> rc;
};

namespace {

constexpr size_t kAlign = 256;
size_t al(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

void worker(MultiCtx* m, uint32_t g) {
    (void)hipSetDevice(m->dev[g]);
    uint64_t seen = 0;
    for (;;) {
        std::function<int(uint32_t)> f;
        {
            std::unique_lock<std::mutex> lk(m->mu);
            m->go.wait(lk, [&] { return m->stop || m->gen != seen; });
            if (m->stop) return;
            seen = m->gen;
            f = m->task;
        }
        (void)hipSetDevice(m->dev[g]);
        const int r = f(g);
        std::lock_guard<std::mutex> lk(m->mu);
        m->rc[g] = r;
        if (--m->busy == 0) m->done.notify_all();
    }
}

// f(g) on every shard's worker at once; the first failing shard's status and message.
int run_all(wq_router* h, const std::function<int(uint32_t)>& f) {
    MultiCtx& m = *h->multi;
    {
        std::unique_lock<std::mutex> lk(m.mu);
        m.task = f;
        m.busy = m.G;
        std::fill(m.rc.begin(), m.rc.end(), 0);
        ++m.gen;
        m.go.notify_all();
        m.done.wait(lk, [&] { return m.busy == 0; });
    }
    for (uint32_t g = 0; g < m.G; ++g)
        if (m.rc[g]) {
            h->err = "shard " + std::to_string(g) + ": " + m.sub[g]->err;
            return m.rc[g];
        }
    (void)hipSetDevice(h->device);
    return WQ_OK;
}

__global__ void k_add_u32(uint32_t* __restrict__ a, uint64_t n, uint32_t c) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] += c;
}

int add_u32(wq_router* s, uint32_t* a, uint64_t n, uint32_t c) {
    if (!n || !c) return WQ_OK;
    hipLaunchKernelGGL(k_add_u32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->stream, a, n, c);
    WQ_HIP(s, hipGetLastError());
    return WQ_OK;
}

// Slice g of M messages.
void slice(uint64_t M, uint32_t G, uint32_t g, uint64_t* lo, uint64_t* hi) {
    *lo = M * g / G;
    *hi = M * (g + 1) / G;
}

// One shard's part of a tick: its slice's inputs staged at `din` (device g) — pos or keys, world,
// sender, repl at the offsets below — routed by the sharded tick into the shard's output staging
// (offsets, peers, msgs), grown and re-copied when the pairs outgrow it. m.P[g] = its pairs.
int shard_tick(wq_router* h, uint32_t g, const char* din, uint64_t Mg, bool keys, bool msgs) {
    MultiCtx& m = *h->multi;
    wq_router* s = m.sub[g];
    const size_t o_w = al(Mg * 24), o_s = al(o_w + Mg * 4), o_r = al(o_s + Mg * 4);
    for (int attempt = 0; attempt < 2; ++attempt) {
        const uint64_t cap = m.cap[g];
        const size_t op = al((Mg + 1) * 4), om = al(op + cap * 4);
        WQ_ALLOC(s, m.out[g], om + (msgs ? cap * 4 : 0) + kAlign);
        char* dout = m.out[g].as<char>();
        size_t P = 0;
        int rc = wq_sharded_route_tick_device(
            s, keys ? nullptr : reinterpret_cast<const double*>(din), keys ? reinterpret_cast<const int64_t*>(din) : nullptr,
            reinterpret_cast<const uint32_t*>(din + o_w), reinterpret_cast<const uint32_t*>(din + o_s),
            reinterpret_cast<const uint8_t*>(din + o_r), Mg, reinterpret_cast<uint32_t*>(dout),
            reinterpret_cast<uint32_t*>(dout + op), msgs ? reinterpret_cast<uint32_t*>(dout + om) : nullptr, cap, &P);
        m.P[g] = P;
        if (rc == WQ_E_CAPACITY && P > cap && P <= 0xFFFFFFFFull) {
            // the shard's staging was short: grow it and copy the kept result out again (no re-exchange)
            m.cap[g] = P + P / 4 + 1024;
            const uint64_t c2 = m.cap[g];
            const size_t op2 = al((Mg + 1) * 4), om2 = al(op2 + c2 * 4);
            WQ_ALLOC(s, m.out[g], om2 + (msgs ? c2 * 4 : 0) + kAlign);
            char* d2 = m.out[g].as<char>();
            return wq_sharded_copy_out(s, reinterpret_cast<uint32_t*>(d2), reinterpret_cast<uint32_t*>(d2 + op2),
                                       msgs ? reinterpret_cast<uint32_t*>(d2 + om2) : nullptr, c2);
        }
        return rc;
    }
    return WQ_OK;
}

// Per shard: the CSR slice, rebased (offsets + base, msgs + lo), into the caller's arrays —
// host arrays (kind D2H) or devices[0] arrays (peer copies).
int shard_copy_back(wq_router* h, uint32_t g, uint64_t lo, uint64_t Mg, uint64_t base, uint32_t* offsets,
                    uint32_t* peers, uint32_t* msgs, size_t capacity, bool to_host) {
    MultiCtx& m = *h->multi;
    wq_router* s = m.sub[g];
    const uint64_t cap = m.cap[g];
    const size_t op = al((Mg + 1) * 4), om = al(op + cap * 4);
    char* dout = m.out[g].as<char>();
    uint32_t* d_off = reinterpret_cast<uint32_t*>(dout);
    uint32_t* d_msgs = reinterpret_cast<uint32_t*>(dout + om);
    const uint64_t Pg = m.P[g];
    if (int rc = add_u32(s, d_off, Mg, (uint32_t)base)) return rc;
    if (msgs && Pg) {
        if (int rc = add_u32(s, d_msgs, Pg, (uint32_t)lo)) return rc;
    }
    const uint64_t keep = base >= capacity ? 0 : std::min<uint64_t>(Pg, capacity - base);
    auto copy = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        if (to_host) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s->stream);
        return m.dev[g] == h->device ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s->stream)
                                     : hipMemcpyPeerAsync(dst, h->device, src, m.dev[g], bytes, s->stream);
    };
    WQ_HIP(s, copy(offsets + lo, d_off, Mg * 4));
    if (keep) {
        WQ_HIP(s, copy(peers + base, dout + op, keep * 4));
        if (msgs) WQ_HIP(s, copy(msgs + base, d_msgs, keep * 4));
    }
    WQ_HIP(s, hipStreamSynchronize(s->stream));
    return WQ_OK;
}

}  // namespace

// The shards' any-keys, merged into the multi handle's own (devices[0]) when an op changed them.
int multi_merge_any(wq_router* h) {
    MultiCtx& m = *h->multi;
    if (!m.any_dirty) return WQ_OK;
    if (int rc = run_all(h, [&](uint32_t g) { return table_ensure_any(m.sub[g]); })) return rc;
    uint64_t total = 0;
    for (wq_router* s : m.sub) total += s->tab.n_any;
    hipStream_t st = h->stream;
    WQ_ALLOC(h, h->tab.any, (total ? total : 1) * 8);
    WQ_ALLOC(h, h->key64_a, (total ? total : 1) * 8);
    uint64_t at = 0;
    for (uint32_t g = 0; g < m.G; ++g) {
        wq_router* s = m.sub[g];
        const uint64_t n = s->tab.n_any;
        if (!n) continue;
        WQ_HIP(h, hipStreamSynchronize(s->stream));
        uint64_t* dst = h->key64_a.as<uint64_t>() + at;
        if (m.dev[g] == h->device)
            WQ_HIP(h, hipMemcpyAsync(dst, s->tab.any.p, n * 8, hipMemcpyDeviceToDevice, st));
        else
            WQ_HIP(h, hipMemcpyPeerAsync(dst, h->device, s->tab.any.p, m.dev[g], n * 8, st));
        at += n;
    }
    uint64_t uniq = 0;
    if (total) {
        // sort (world << 32 | peer), then drop duplicates: a peer with cubes on several shards
        size_t b1 = 0, b2 = 0;
        uint64_t* keys = h->key64_a.as<uint64_t>();
        uint64_t* sorted = h->tab.any.as<uint64_t>();
        WQ_HIP(h, rocprim::radix_sort_keys(nullptr, b1, keys, sorted, (size_t)total, 0, 64, st));
        WQ_ALLOC(h, h->key64_b, (total ? total : 1) * 8);
        WQ_HIP(h, rocprim::unique(nullptr, b2, sorted, h->key64_b.as<uint64_t>(), (uint64_t*)nullptr, (size_t)total,
                                  rocprim::equal_to<uint64_t>(), st));
        WQ_ALLOC(h, m.tmp, std::max(b1, b2));
        WQ_ALLOC(m.sub[0], m.cnt, 64);
        WQ_HIP(h, rocprim::radix_sort_keys(m.tmp.p, b1, keys, sorted, (size_t)total, 0, 64, st));
        WQ_HIP(h, rocprim::unique(m.tmp.p, b2, sorted, h->key64_b.as<uint64_t>(), m.cnt.as<uint64_t>(), (size_t)total,
                                  rocprim::equal_to<uint64_t>(), st));
        WQ_HIP(h, hipMemcpyAsync(&uniq, m.cnt.p, 8, hipMemcpyDeviceToHost, st));
        WQ_HIP(h, hipStreamSynchronize(st));
        WQ_HIP(h, hipMemcpyAsync(h->tab.any.p, h->key64_b.p, uniq * 8, hipMemcpyDeviceToDevice, st));
        WQ_HIP(h, hipStreamSynchronize(st));
    }
    h->tab.n_any = uniq;
    h->any_stale = false;
    m.any_dirty = false;
    return WQ_OK;
}

int multi_apply_ops(wq_router* h, const wq_op* ops, size_t n) {
    h->multi->any_dirty = true;
    return run_all(h, [&](uint32_t g) { return wq_sharded_apply_ops(h->multi->sub[g], ops, n); });
}

int multi_apply_ops_device(wq_router* h, const wq_op* d_ops, size_t n) {
    std::vector<wq_op> ops(n);
    if (n) {
        WQ_HIP(h, hipStreamSynchronize(h->stream));
        WQ_HIP(h, hipMemcpy(ops.data(), d_ops, n * sizeof(wq_op), hipMemcpyDeviceToHost));
    }
    for (const wq_op& o : ops)  // the device-batch contract: subscribe / unsubscribe only
        if (o.kind > WQ_OP_UNSUBSCRIBE || o.world == WQ_WORLD_INVALID)
            return set_error(h, WQ_E_INVALID, "device op batch: REMOVE_PEER or the reserved world id");
    return multi_apply_ops(h, ops.data(), n);
}

int multi_remove_peers(wq_router* h, const uint32_t* peers, size_t n) {
    h->multi->any_dirty = true;
    return run_all(h, [&](uint32_t g) { return wq_remove_peers(h->multi->sub[g], peers, n); });
}

int multi_route_tick(wq_router* h, const double* pos, const int64_t* keys, const uint32_t* world,
                     const uint32_t* sender, const uint8_t* repl, size_t M, uint32_t* offsets, uint32_t* peers,
                     uint32_t* msgs, size_t capacity, size_t* n_pairs, bool on_device) {
    MultiCtx& m = *h->multi;
    const uint32_t G = m.G;
    const bool use_keys = keys != nullptr;
    hipEvent_t ready = nullptr;
    if (on_device) {  // the caller's arrays (devices[0]) are complete once its stream gets here
        WQ_HIP(h, hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        WQ_HIP(h, hipEventRecord(ready, h->stream));
    }
    int rc = run_all(h, [&](uint32_t g) -> int {
        wq_router* s = m.sub[g];
        uint64_t lo, hi;
        slice(M, G, g, &lo, &hi);
        const uint64_t Mg = hi - lo;
        if (!m.cap[g]) m.cap[g] = 16 * Mg + 1024;
        const size_t o_w = al(Mg * 24), o_s = al(o_w + Mg * 4), o_r = al(o_s + Mg * 4), n_in = al(o_r + Mg + 1);
        WQ_ALLOC(s, m.in[g], n_in);
        char* din = m.in[g].as<char>();
        const void* src_k = use_keys ? (const void*)(keys + 3 * lo) : (const void*)(pos ? pos + 3 * lo : nullptr);
        if (on_device) WQ_HIP(s, hipStreamWaitEvent(s->stream, ready, 0));
        auto put = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
            if (!bytes) return hipSuccess;
            if (!on_device) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s->stream);
            return m.dev[g] == h->device ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s->stream)
                                         : hipMemcpyPeerAsync(dst, m.dev[g], src, h->device, bytes, s->stream);
        };
        if (src_k) WQ_HIP(s, put(din, src_k, Mg * 24));
        WQ_HIP(s, put(din + o_w, world + lo, Mg * 4));
        WQ_HIP(s, put(din + o_s, sender + lo, Mg * 4));
        WQ_HIP(s, put(din + o_r, repl + lo, Mg));
        return shard_tick(h, g, din, Mg, use_keys, msgs != nullptr);
    });
    if (ready) (void)hipEventDestroy(ready);
    if (rc) return rc;
    std::vector<uint64_t> base(G + 1, 0);
    for (uint32_t g = 0; g < G; ++g) base[g + 1] = base[g] + m.P[g];
    const uint64_t P = base[G];
    *n_pairs = P;
    if (P > 0xFFFFFFFFull) return set_error(h, WQ_E_CAPACITY, "more than 2^32-1 pairs in one tick");
    rc = run_all(h, [&](uint32_t g) -> int {
        uint64_t lo, hi;
        slice(M, G, g, &lo, &hi);
        return shard_copy_back(h, g, lo, hi - lo, base[g], offsets, peers, msgs, capacity, !on_device);
    });
    if (rc) return rc;
    const uint32_t last = (uint32_t)P;
    if (on_device) {
        WQ_HIP(h, hipMemcpyAsync(offsets + M, &last, 4, hipMemcpyHostToDevice, h->stream));
        WQ_HIP(h, hipStreamSynchronize(h->stream));
    } else {
        offsets[M] = last;
    }
    if (P > capacity) return set_error(h, WQ_E_CAPACITY, "output capacity too small (required size in *n_pairs)");
    return WQ_OK;
}

int multi_is_subscribed(wq_router* h, size_t n, const uint32_t* world, const uint32_t* peer, int raw,
                        const void* kp, uint8_t* out) {
    MultiCtx& m = *h->multi;
    std::vector<std::vector<uint8_t>> part(m.G, std::vector<uint8_t>(n));
    if (int rc = run_all(h, [&](uint32_t g) { return wq_is_subscribed(m.sub[g], n, world, peer, raw, kp, part[g].data()); }))
        return rc;
    for (size_t i = 0; i < n; ++i) {
        uint8_t v = 0;
        for (uint32_t g = 0; g < m.G; ++g) v |= part[g][i];
        out[i] = v ? 1 : 0;
    }
    return WQ_OK;
}

int multi_set_positions(wq_router* h, const double* pos, size_t n, bool on_device) {
    MultiCtx& m = *h->multi;
    if (!on_device)
        return run_all(h, [&](uint32_t g) { return wq_set_peer_positions(m.sub[g], pos, n); });
    // device positions live on devices[0]: every shard takes its own copy (peer reads)
    WQ_HIP(h, hipStreamSynchronize(h->stream));
    return run_all(h, [&](uint32_t g) -> int {
        wq_router* s = m.sub[g];
        if (m.dev[g] == h->device) return wq_set_peer_positions_device(s, pos, n);
        WQ_ALLOC(s, m.in[g], n * 24 + kAlign);
        WQ_HIP(s, hipMemcpyPeerAsync(m.in[g].p, m.dev[g], pos, h->device, n * 24, s->stream));
        return wq_set_peer_positions_device(s, m.in[g].as<double>(), n);
    });
}

int multi_set_radius(wq_router* h, double radius) {
    return run_all(h, [&](uint32_t g) { return wq_set_radius(h->multi->sub[g], radius); });
}

int multi_set_hint(wq_router* h, double pairs_per_message) {
    return run_all(h, [&](uint32_t g) { return wq_set_fanout_hint(h->multi->sub[g], pairs_per_message); });
}

int multi_stats(wq_router* h, wq_stats* out) {
    MultiCtx& m = *h->multi;
    std::vector<wq_stats> st(m.G);
    if (int rc = run_all(h, [&](uint32_t g) { return wq_get_stats(m.sub[g], &st[g]); })) return rc;
    if (int rc = multi_merge_any(h)) return rc;
    memset(out, 0, sizeof(*out));
    for (const wq_stats& s : st) {
        out->n_entries += s.n_entries;
        out->n_cubes += s.n_cubes;
        out->table_slots += s.table_slots;
        out->hash_fallbacks += s.hash_fallbacks;
    }
    out->n_any = h->tab.n_any;
    out->cube_size = h->cube_size;
    out->device = h->device;
    return WQ_OK;
}

int multi_health(wq_router* h, uint32_t* error_bits, uint32_t* overflow) {
    MultiCtx& m = *h->multi;
    std::vector<uint32_t> e(m.G, 0), o(m.G, 0);
    if (int rc = run_all(h, [&](uint32_t g) { return wq_route_health(m.sub[g], &e[g], &o[g]); })) return rc;
    for (uint32_t g = 0; g < m.G; ++g) {
        *error_bits |= e[g];
        *overflow |= o[g];
    }
    return WQ_OK;
}

void multi_release(wq_router* h) {
    MultiCtx* m = h->multi;
    if (!m) return;
    {
        std::lock_guard<std::mutex> lk(m->mu);
        m->stop = true;
        m->go.notify_all();
    }
    for (std::thread& t : m->th)
        if (t.joinable()) t.join();
    for (uint32_t g = 0; g < m->sub.size(); ++g) {
        (void)hipSetDevice(m->dev[g]);
        m->in[g].release();
        m->out[g].release();
        if (m->sub[g]) wq_router_destroy(m->sub[g]);
    }
    (void)hipSetDevice(h->device);
    m->tmp.release();
    m->cnt.release();
    if (m->hub) wq_hub_destroy(m->hub);
    delete m;
    h->multi = nullptr;
}

}  // namespace wq

using namespace wq;

extern "C" int wq_router_create_multi(uint16_t cube_size, int n_gpus, const int* devices, wq_router** out) {
    if (!out || cube_size == 0 || n_gpus < 1 || n_gpus > WQ_MAX_SHARDS || !devices) return WQ_E_INVALID;
    *out = nullptr;
    wq_router* h = nullptr;
    int rc = wq_router_create(cube_size, devices[0], &h);  // the handle itself: devices[0], the merged any-keys
    if (rc) return rc;
    MultiCtx* m = new (std::nothrow) MultiCtx();
    if (!m) {
        wq_router_destroy(h);
        return WQ_E_OOM;
    }
    h->multi = m;
    const uint32_t G = (uint32_t)n_gpus;
    m->G = G;
    m->dev.assign(devices, devices + G);
    m->sub.assign(G, nullptr);
    m->in.resize(G);
    m->out.resize(G);
    m->cap.assign(G, 0);
    m->P.assign(G, 0);
    m->rc.assign(G, 0);
    rc = wq_hub_create(G, &m->hub);
    for (uint32_t g = 0; g < G && rc == WQ_OK; ++g) {
        rc = wq_router_create(cube_size, devices[g], &m->sub[g]);
        if (rc == WQ_OK) rc = wq_shard_attach_hub(m->sub[g], m->hub, g);
        if (rc) h->err = std::string("shard ") + std::to_string(g) + ": " + wq_last_error(m->sub[g]);
    }
    if (rc == WQ_OK) {
        try {
            for (uint32_t g = 0; g < G; ++g) m->th.emplace_back(worker, m, g);
        } catch (...) {
            rc = WQ_E_OOM;
        }
    }
    (void)hipSetDevice(devices[0]);
    if (rc) {
        wq_router_destroy(h);
        return rc;
    }
    *out = h;
    return WQ_OK;
}

extern "C" int wq_multi_info(wq_router* h, uint32_t* n_gpus) {
    if (!h || !n_gpus) return WQ_E_INVALID;
    *n_gpus = h->multi ? h->multi->G : 1;
    return WQ_OK;
}
