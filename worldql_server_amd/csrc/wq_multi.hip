// wq_multi.hip — ONE handle over G GPUs (wq_router_create(cube_size, n_gpus,
// devices, ...)), the reference's one-owner model kept at the boundary.
//
// The reference owns one WorldMap in one task (worldql_server/src/processing/thread.rs:119, driven
// by the select! loop at :122-146). wq_router_create_multi[_mode] gives that task one handle again:
// inside, G sub-handles (one per device) and G worker threads — one per sub-handle, since a sharded
// tick is collective — that the calling thread hands each call to and waits for. Two layouts:
//   WQ_MULTI_CUBE_HASH  every (world, cube) bucket lives on one shard (cube-hash owner, wq_sharded.hip);
//                       the sub-handles share an in-process hub and a tick is the sharded tick
//   WQ_MULTI_REPLICATE  every device holds the whole table (288 GB of HBM holds C3's ~10 GB many
//                       times over) and routes its own slice of the messages with the single-GPU
//                       tick: no exchange at all; every op is applied on every device
// What a call does on the multi handle:
//   wq_apply_ops, wq_remove_peers     cube hash: every shard gets the whole stream and keeps what it
//                                     owns (+ every REMOVE_PEER); replicate: every replica applies all
//   wq_apply_ops_device               cube hash: ops validated and partitioned by owner on devices[0]
//                                     (one read-back of G counts), each shard's part applied on its
//                                     device; replicate: the batch to every replica, asynchronous
//   wq_route_tick / _device           the messages in G contiguous slices, one per sub-handle, the G
//                                     CSRs concatenated into the caller's in message order: exactly
//                                     the one-table result (all pairs cross to devices[0])
//   wq_route_tick_slices_device       each device's own messages routed where they are, each CSR left
//                                     on its device (views): the scaling form
//   wq_is_subscribed[_any], wq_world_peers, wq_route_global[_device], wq_get_stats
//                                     cube hash: shard answers combined (any-keys merged on
//                                     devices[0]); replicate: replica 0 answers
//   radius filter / peer positions / hint   forwarded to every sub-handle
// Device-pointer calls take their arrays on devices[0] (the slice form: on each slice's device).
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
    int mode = WQ_MULTI_CUBE_HASH;
    std::vector<int> dev;
    std::vector<wq_router*> sub;
    wq_hub* hub = nullptr;
    // per sub-handle, on its device: staged inputs and outputs of a tick, device op batches
    // (two, alternating: a sub-handle may re-apply its previous batch at its next call)
    std::vector<DevBuf> in, out, ops0, ops1;
    std::vector<uint64_t> cap, P;
    // wq_route_tick_slices_device's outputs: their own staging, so the views it returns survive every
    // other call on the handle (routes, queries, op batches) until the next slices call
    std::vector<DevBuf> vout;
    std::vector<uint64_t> vcap, vP;
    std::vector<uint32_t> flip;
    // per sub-handle, recorded on its stream after it copied a device op batch out of m.part: the
    // next write of m.part (on the handle's stream) waits for every one of them
    std::vector<hipEvent_t> copied;
    bool any_dirty = true;  // the merged any-keys need rebuilding (an op was applied since)
    DevBuf tmp, cnt, part;  // devices[0] scratch: the any-key merge, the device op partition
    hipEvent_t ready = nullptr;
    uint32_t err_sticky = 0, ovf_sticky = 0;  // the handle's own health bits (wq_route_health)
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

// f(g) on every sub-handle's worker at once; the first failing one's status and message.
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
            h->err = "device " + std::to_string(g) + ": " + m.sub[g]->err;
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

// A device op batch on devices[0] -> its owner shard per op (G = an invalid op: REMOVE_PEER or
// the reserved world id, which the device-batch contract rejects) and the count per owner.
__global__ void k_multi_op_owner(const wq_op* __restrict__ ops, uint32_t n, double sf, int64_t si, uint32_t G,
                                 uint32_t* __restrict__ owner, uint32_t* __restrict__ counts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const wq_op op = ops[i];
    uint32_t o = G;
    if (op.kind <= WQ_OP_UNSUBSCRIBE && op.world != WQ_WORLD_INVALID) {
        int64_t x, y, z;
        if (op.key_is_raw) {
            x = op.u.key[0];
            y = op.u.key[1];
            z = op.u.key[2];
        } else {
            x = coord_clamp_dev(op.u.pos[0], sf, si);
            y = coord_clamp_dev(op.u.pos[1], sf, si);
            z = coord_clamp_dev(op.u.pos[2], sf, si);
        }
        o = shard_of(op.world, x, y, z, G);
    }
    owner[i] = o;
    atomicAdd(counts + o, 1u);
}

__global__ void k_multi_iota(uint32_t* __restrict__ a, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = i;
}

__global__ void k_multi_gather_ops(const wq_op* __restrict__ ops, const uint32_t* __restrict__ order, uint32_t n,
                                   wq_op* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = ops[order[i]];
}

// Slice g of M messages.
void slice(uint64_t M, uint32_t G, uint32_t g, uint64_t* lo, uint64_t* hi) {
    *lo = M * g / G;
    *hi = M * (g + 1) / G;
}

// One sub-handle's messages (device pointers on its device).
struct SliceIn {
    const double* pos;
    const int64_t* keys;
    const uint32_t* world;
    const uint32_t* sender;
    const uint8_t* repl;
    uint64_t M;
};

// Output staging of sub-handle g: offsets, peers, msgs at these offsets of m.out[g].
void out_layout(uint64_t M, uint64_t cap, size_t* op, size_t* om) {
    *op = al((M + 1) * 4);
    *om = al(*op + cap * 4);
}

// The sub-handle's health words hold an overflow bit for every staging attempt that came up short
// (the handle grows its staging and routes / copies again): not the caller's overflow. Cleared.
int clear_staging_overflow(wq_router* s) {
    if (!s->rws.buf.p) return WQ_OK;
    WQ_HIP(s, hipMemsetAsync(route_health(s) + 1, 0, 4, s->stream));
    return WQ_OK;
}

// One sub-handle's part of a tick: its messages routed into its output staging (offsets, peers,
// msgs), grown when the pairs outgrow it. m.P[g] = its pairs. Cube hash: the sharded tick (every
// sub-handle takes part: it is collective); replicate: the single-GPU tick on the replica.
int tick_into(wq_router* h, uint32_t g, const SliceIn& x, bool msgs, bool view) {
    MultiCtx& m = *h->multi;
    wq_router* s = m.sub[g];
    DevBuf& ob = view ? m.vout[g] : m.out[g];
    uint64_t& capr = view ? m.vcap[g] : m.cap[g];
    uint64_t& Pr = view ? m.vP[g] : m.P[g];
    if (!capr) capr = 16 * x.M + 1024;
    for (int attempt = 0; attempt < 3; ++attempt) {
        const uint64_t cap = capr;
        size_t op, om;
        out_layout(x.M, cap, &op, &om);
        WQ_ALLOC(s, ob, om + (msgs ? cap * 4 : 0) + kAlign);
        char* dout = ob.as<char>();
        uint32_t* d_off = reinterpret_cast<uint32_t*>(dout);
        uint32_t* d_peers = reinterpret_cast<uint32_t*>(dout + op);
        uint32_t* d_msgs = msgs ? reinterpret_cast<uint32_t*>(dout + om) : nullptr;
        if (m.mode == WQ_MULTI_CUBE_HASH) {
            size_t P = 0;
            int rc = wq_sharded_route_tick_device(s, x.pos, x.keys, x.world, x.sender, x.repl, x.M, d_off, d_peers,
                                                  d_msgs, cap, &P);
            Pr = P;
            if (rc == WQ_E_CAPACITY && P > cap && P <= 0xFFFFFFFFull) {
                // the staging was short: grow it and copy the kept result out again (no re-exchange)
                capr = P + P / 4 + 1024;
                const uint64_t c2 = capr;
                size_t op2, om2;
                out_layout(x.M, c2, &op2, &om2);
                WQ_ALLOC(s, ob, om2 + (msgs ? c2 * 4 : 0) + kAlign);
                char* d2 = ob.as<char>();
                rc = wq_sharded_copy_out(s, reinterpret_cast<uint32_t*>(d2), reinterpret_cast<uint32_t*>(d2 + op2),
                                         msgs ? reinterpret_cast<uint32_t*>(d2 + om2) : nullptr, c2);
                if (rc == WQ_OK) rc = clear_staging_overflow(s);
                // the copy-out is enqueued, not finished: the slices' views are read as soon as the
                // call returns (wq_route_tick_slices_device is synchronous), so wait for it here
                if (rc == WQ_OK && hipStreamSynchronize(s->stream) != hipSuccess)
                    rc = set_error(s, WQ_E_HIP, "sharded copy-out");
            }
            return rc;
        }
        // replicate: the single-GPU tick, P read back
        int rc = wq_route_tick_device(s, x.pos, x.keys, x.world, x.sender, x.repl, x.M, d_off, d_peers, d_msgs, cap,
                                      nullptr);
        if (rc) return rc;
        wq_route_counters c{};
        WQ_HIP(s, hipMemcpyAsync(&c, s->rws.last, sizeof(c), hipMemcpyDeviceToHost, s->stream));
        WQ_HIP(s, hipStreamSynchronize(s->stream));
        if (x.M == 0) c.n_pairs = 0;
        if (c.error & 4u) return set_error(s, WQ_E_TIMEOUT, "route look-back spin gave up");
        if (c.error & 8u) return set_error(s, WQ_E_INVALID, "a replica's table still misses a device batch");
        if (c.error) return set_error(s, WQ_E_CAPACITY, "more than 2^32-1 pairs in one tick");
        Pr = c.n_pairs;
        // the next tick's shape from this one's fan-out, as the host-array tick does (a replica's
        // device ticks are read back here anyway)
        if (s->fanout_auto && x.M >= 256) s->heavy_fanout = (double)c.n_pairs >= WQ_HEAVY_FANOUT * (double)x.M;
        if (c.n_pairs <= cap) return WQ_OK;
        if (c.n_pairs > 0xFFFFFFFFull) return set_error(s, WQ_E_CAPACITY, "more than 2^32-1 pairs in one tick");
        capr = c.n_pairs + c.n_pairs / 4 + 1024;  // short: grow the staging and route again
        if (int r2 = clear_staging_overflow(s)) return r2;
    }
    return set_error(s, WQ_E_CAPACITY, "replica staging kept growing");
}

// Per sub-handle: the CSR slice, rebased (offsets + base, msgs + lo), into the caller's arrays —
// host arrays (kind D2H) or devices[0] arrays (peer copies).
int shard_copy_back(wq_router* h, uint32_t g, uint64_t lo, uint64_t Mg, uint64_t base, uint32_t* offsets,
                    uint32_t* peers, uint32_t* msgs, size_t capacity, bool to_host) {
    MultiCtx& m = *h->multi;
    wq_router* s = m.sub[g];
    size_t op, om;
    out_layout(Mg, m.cap[g], &op, &om);
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

// A device op batch (m.part on devices[0]) to sub-handle g: copied to its alternating staging
// buffer on its own stream after the handle's stream has produced it, then applied (asynchronously).
int apply_staged(wq_router* h, uint32_t g, const wq_op* src, size_t n) {
    MultiCtx& m = *h->multi;
    wq_router* s = m.sub[g];
    if (!n) return WQ_OK;
    DevBuf& st = (m.flip[g] ^= 1u) ? m.ops1[g] : m.ops0[g];
    WQ_ALLOC(s, st, n * sizeof(wq_op));
    WQ_HIP(s, hipStreamWaitEvent(s->stream, m.ready, 0));
    if (m.dev[g] == h->device)
        WQ_HIP(s, hipMemcpyAsync(st.p, src, n * sizeof(wq_op), hipMemcpyDeviceToDevice, s->stream));
    else
        WQ_HIP(s, hipMemcpyPeerAsync(st.p, m.dev[g], src, h->device, n * sizeof(wq_op), s->stream));
    WQ_HIP(s, hipEventRecord(m.copied[g], s->stream));  // src (m.part) may be rewritten after this
    return wq_apply_ops_device(s, st.as<wq_op>(), n);
}

}  // namespace

// The any-keys behind the handle's queries, in its own (devices[0]) table when an op changed them:
// the shards' merged (cube hash), or replica 0's (replicate).
int multi_merge_any(wq_router* h) {
    MultiCtx& m = *h->multi;
    if (!m.any_dirty) return WQ_OK;
    hipStream_t st = h->stream;
    if (m.mode == WQ_MULTI_REPLICATE) {
        wq_router* s = m.sub[0];
        (void)hipSetDevice(s->device);
        if (int rc = table_ensure_any(s)) return rc;
        WQ_HIP(s, hipStreamSynchronize(s->stream));
        (void)hipSetDevice(h->device);
        const uint64_t n = s->tab.n_any;
        WQ_ALLOC(h, h->tab.any, (n ? n : 1) * 8);
        if (n) {
            if (m.dev[0] == h->device)
                WQ_HIP(h, hipMemcpyAsync(h->tab.any.p, s->tab.any.p, n * 8, hipMemcpyDeviceToDevice, st));
            else
                WQ_HIP(h, hipMemcpyPeerAsync(h->tab.any.p, h->device, s->tab.any.p, m.dev[0], n * 8, st));
            WQ_HIP(h, hipStreamSynchronize(st));
        }
        h->tab.n_any = n;
        h->any_stale = false;
        m.any_dirty = false;
        return WQ_OK;
    }
    if (int rc = run_all(h, [&](uint32_t g) { return table_ensure_any(m.sub[g]); })) return rc;
    uint64_t total = 0;
    for (wq_router* s : m.sub) total += s->tab.n_any;
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
        WQ_ALLOC(h, m.cnt, 64);
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
    MultiCtx& m = *h->multi;
    m.any_dirty = true;
    if (m.mode == WQ_MULTI_REPLICATE) return run_all(h, [&](uint32_t g) { return wq_apply_ops(m.sub[g], ops, n); });
    return run_all(h, [&](uint32_t g) { return wq_sharded_apply_ops(m.sub[g], ops, n); });
}

// The device-batch contract of the single-GPU handle on G devices: an invalid op (REMOVE_PEER, the
// reserved world id) rejects the whole batch, reported as error bit 16 of wq_route_health and in
// wq_last_error while the call itself returns WQ_OK. Replicate: every replica takes the batch
// asynchronously (each rejects an invalid one itself). Cube hash: the ops are validated and
// partitioned by owner on devices[0] — one read-back of G + 1 counts, not of the batch — and each
// shard's part is applied on its own device.
int multi_apply_ops_device(wq_router* h, const wq_op* d_ops, size_t n) {
    MultiCtx& m = *h->multi;
    const uint32_t G = m.G;
    if (n == 0) return WQ_OK;
    if (n >= 0xFFFFFFFFull) return set_error(h, WQ_E_INVALID, "device op batch larger than 2^32 - 1 ops");
    m.any_dirty = true;
    hipStream_t st = h->stream;
    // m.part is read by the sub-handles' copies of the previous batch: order this batch's writes of it
    // after them (and wait for them on the host before the buffer may be reallocated)
    const bool grow = n * sizeof(wq_op) > m.part.bytes;
    for (uint32_t g = 0; g < G; ++g) {
        if (grow) WQ_HIP(h, hipEventSynchronize(m.copied[g]));
        WQ_HIP(h, hipStreamWaitEvent(st, m.copied[g], 0));
    }
    WQ_ALLOC(h, m.part, n * sizeof(wq_op));
    if (m.mode == WQ_MULTI_REPLICATE) {
        // the caller's batch is read once, on the caller's stream; the replicas copy the handle's
        // staging (so the caller may reuse d_ops as soon as its stream has passed this call)
        WQ_HIP(h, hipMemcpyAsync(m.part.p, d_ops, n * sizeof(wq_op), hipMemcpyDeviceToDevice, st));
        WQ_HIP(h, hipEventRecord(m.ready, st));
        return run_all(h, [&](uint32_t g) { return apply_staged(h, g, m.part.as<wq_op>(), n); });
    }
    WQ_ALLOC(h, h->key32_a, n * 4);
    WQ_ALLOC(h, h->key32_b, n * 4);
    WQ_ALLOC(h, h->idx_a, n * 4);
    WQ_ALLOC(h, h->idx_b, n * 4);
    WQ_ALLOC(h, m.cnt, 4 * (WQ_MAX_SHARDS + 1));
    uint32_t* owner = h->key32_a.as<uint32_t>();
    uint32_t* cnt = m.cnt.as<uint32_t>();
    WQ_HIP(h, hipMemsetAsync(cnt, 0, 4 * (G + 1), st));
    const unsigned gr = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_multi_op_owner, dim3(gr), dim3(256), 0, st, d_ops, (uint32_t)n, (double)h->cube_size,
                       (int64_t)h->cube_size, G, owner, cnt);
    hipLaunchKernelGGL(k_multi_iota, dim3(gr), dim3(256), 0, st, h->idx_a.as<uint32_t>(), (uint32_t)n);
    WQ_HIP(h, hipGetLastError());
    std::vector<uint32_t> c(G + 1);
    WQ_HIP(h, hipMemcpyAsync(c.data(), cnt, 4 * (G + 1), hipMemcpyDeviceToHost, st));
    WQ_HIP(h, hipStreamSynchronize(st));
    if (c[G]) {  // rejected whole, as a single-GPU handle rejects it
        m.err_sticky |= kErrBadBatch;
        h->err = "bad op (kind or reserved world id) in a device batch: that batch was not applied";
        return WQ_OK;
    }
    // stable partition by owner: a radix sort of (owner, op index) over the owner's bits
    int bits = 1;
    while ((1u << bits) <= G) ++bits;
    size_t tb = 0;
    WQ_HIP(h, rocprim::radix_sort_pairs(nullptr, tb, owner, h->key32_b.as<uint32_t>(), h->idx_a.as<uint32_t>(),
                                        h->idx_b.as<uint32_t>(), n, 0, bits, st));
    WQ_ALLOC(h, m.tmp, tb);
    WQ_HIP(h, rocprim::radix_sort_pairs(m.tmp.p, tb, owner, h->key32_b.as<uint32_t>(), h->idx_a.as<uint32_t>(),
                                        h->idx_b.as<uint32_t>(), n, 0, bits, st));
    hipLaunchKernelGGL(k_multi_gather_ops, dim3(gr), dim3(256), 0, st, d_ops, h->idx_b.as<uint32_t>(), (uint32_t)n,
                       m.part.as<wq_op>());
    WQ_HIP(h, hipGetLastError());
    WQ_HIP(h, hipEventRecord(m.ready, st));
    std::vector<size_t> off(G + 1, 0);
    for (uint32_t g = 0; g < G; ++g) off[g + 1] = off[g] + c[g];
    return run_all(h, [&](uint32_t g) { return apply_staged(h, g, m.part.as<wq_op>() + off[g], c[g]); });
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
    if (on_device) WQ_HIP(h, hipEventRecord(m.ready, h->stream));  // the caller's arrays are complete here
    int rc = run_all(h, [&](uint32_t g) -> int {
        wq_router* s = m.sub[g];
        uint64_t lo, hi;
        slice(M, G, g, &lo, &hi);
        const uint64_t Mg = hi - lo;
        const size_t o_w = al(Mg * 24), o_s = al(o_w + Mg * 4), o_r = al(o_s + Mg * 4), n_in = al(o_r + Mg + 1);
        WQ_ALLOC(s, m.in[g], n_in);
        char* din = m.in[g].as<char>();
        const void* src_k = use_keys ? (const void*)(keys + 3 * lo) : (const void*)(pos ? pos + 3 * lo : nullptr);
        if (on_device) WQ_HIP(s, hipStreamWaitEvent(s->stream, m.ready, 0));
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
        SliceIn x{use_keys ? nullptr : reinterpret_cast<const double*>(din),
                  use_keys ? reinterpret_cast<const int64_t*>(din) : nullptr,
                  reinterpret_cast<const uint32_t*>(din + o_w), reinterpret_cast<const uint32_t*>(din + o_s),
                  reinterpret_cast<const uint8_t*>(din + o_r), Mg};
        return tick_into(h, g, x, msgs != nullptr, false);
    });
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
    if (P > capacity) {
        m.ovf_sticky = 1;  // as a single-GPU tick's sticky overflow word
        return set_error(h, WQ_E_CAPACITY, "output capacity too small (required size in *n_pairs)");
    }
    return WQ_OK;
}

int multi_route_slices(wq_router* h, const wq_msg_slice* in, int with_msgs, wq_slice_view* out) {
    MultiCtx& m = *h->multi;
    for (uint32_t g = 0; g < m.G; ++g) {
        const wq_msg_slice& x = in[g];
        if (x.n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per slice");
        if (x.n_msgs && (!x.d_world || !x.d_sender || !x.d_repl || (!x.d_pos && !x.d_keys)))
            return set_error(h, WQ_E_INVALID, "a slice with messages but without its arrays");
    }
    int rc = run_all(h, [&](uint32_t g) -> int {
        const wq_msg_slice& x = in[g];
        SliceIn si{x.d_keys ? nullptr : x.d_pos, x.d_keys, x.d_world, x.d_sender, x.d_repl, x.n_msgs};
        return tick_into(h, g, si, with_msgs != 0, true);
    });
    if (rc) return rc;
    for (uint32_t g = 0; g < m.G; ++g) {
        size_t op, om;
        out_layout(in[g].n_msgs, m.vcap[g], &op, &om);
        const char* d = m.vout[g].as<char>();
        wq_slice_view& v = out[g];
        v.device = m.dev[g];
        v.pad_ = 0;
        v.n_msgs = in[g].n_msgs;
        v.n_pairs = m.vP[g];
        v.offsets = reinterpret_cast<const uint32_t*>(d);
        v.peers = reinterpret_cast<const uint32_t*>(d + op);
        v.msgs = with_msgs ? reinterpret_cast<const uint32_t*>(d + om) : nullptr;
    }
    return WQ_OK;
}

int multi_is_subscribed(wq_router* h, size_t n, const uint32_t* world, const uint32_t* peer, int raw,
                        const void* kp, uint8_t* out) {
    MultiCtx& m = *h->multi;
    if (m.mode == WQ_MULTI_REPLICATE) return wq_is_subscribed(m.sub[0], n, world, peer, raw, kp, out);
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
    // device positions live on devices[0]: every sub-handle takes its own copy (peer reads)
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
    if (m.mode == WQ_MULTI_REPLICATE) {
        *out = st[0];
    } else {
        for (const wq_stats& s : st) {
            out->n_entries += s.n_entries;
            out->n_cubes += s.n_cubes;
            out->table_slots += s.table_slots;
            out->hash_fallbacks += s.hash_fallbacks;
        }
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
    *error_bits |= m.err_sticky;
    *overflow |= m.ovf_sticky;
    m.err_sticky = m.ovf_sticky = 0;
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
        if (m->sub[g]) (void)hipStreamSynchronize(m->sub[g]->stream);
        m->in[g].release();
        m->out[g].release();
        m->vout[g].release();
        if (m->copied[g]) (void)hipEventDestroy(m->copied[g]);
        m->ops0[g].release();
        m->ops1[g].release();
        if (m->sub[g]) wq_router_destroy(m->sub[g]);
    }
    (void)hipSetDevice(h->device);
    m->tmp.release();
    m->cnt.release();
    m->part.release();
    if (m->ready) (void)hipEventDestroy(m->ready);
    if (m->hub) wq_hub_destroy(m->hub);
    delete m;
    h->multi = nullptr;
}

}  // namespace wq

using namespace wq;

extern "C" int wq_router_create_multi_mode(uint16_t cube_size, int n_gpus, const int* devices, int mode,
                                           wq_router** out) {
    if (!out || cube_size == 0 || n_gpus < 1 || n_gpus > WQ_MAX_SHARDS || !devices ||
        (mode != WQ_MULTI_CUBE_HASH && mode != WQ_MULTI_REPLICATE))
        return WQ_E_INVALID;
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
    m->mode = mode;
    m->dev.assign(devices, devices + G);
    m->sub.assign(G, nullptr);
    m->in.resize(G);
    m->out.resize(G);
    m->vout.resize(G);
    m->vcap.assign(G, 0);
    m->vP.assign(G, 0);
    m->copied.assign(G, nullptr);
    m->ops0.resize(G);
    m->ops1.resize(G);
    m->cap.assign(G, 0);
    m->P.assign(G, 0);
    m->flip.assign(G, 0);
    m->rc.assign(G, 0);
    if (hipEventCreateWithFlags(&m->ready, hipEventDisableTiming) != hipSuccess) rc = WQ_E_HIP;
    if (rc == WQ_OK && mode == WQ_MULTI_CUBE_HASH) rc = wq_hub_create(G, &m->hub);
    for (uint32_t g = 0; g < G && rc == WQ_OK; ++g) {
        rc = wq_router_create(cube_size, devices[g], &m->sub[g]);
        if (rc == WQ_OK) {  // recorded on sub-handle g's stream: created on its device
            (void)hipSetDevice(devices[g]);
            if (hipEventCreateWithFlags(&m->copied[g], hipEventDisableTiming) != hipSuccess) rc = WQ_E_HIP;
            else (void)hipEventRecord(m->copied[g], m->sub[g]->stream);  // complete from the start
        }
        if (rc == WQ_OK && mode == WQ_MULTI_CUBE_HASH) rc = wq_shard_attach_hub(m->sub[g], m->hub, g);
        if (rc) h->err = std::string("device ") + std::to_string(g) + ": " + wq_last_error(m->sub[g]);
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

extern "C" int wq_router_create_multi(uint16_t cube_size, int n_gpus, const int* devices, wq_router** out) {
    return wq_router_create_multi_mode(cube_size, n_gpus, devices, WQ_MULTI_CUBE_HASH, out);
}

extern "C" int wq_multi_info(wq_router* h, uint32_t* n_gpus) {
    if (!h || !n_gpus) return WQ_E_INVALID;
    *n_gpus = h->multi ? h->multi->G : 1;
    return WQ_OK;
}

extern "C" int wq_multi_mode(wq_router* h, int* mode) {
    if (!h || !mode) return WQ_E_INVALID;
    *mode = h->multi ? h->multi->mode : -1;
    return WQ_OK;
}

extern "C" int wq_route_tick_slices_device(wq_router* h, const wq_msg_slice* in, int with_msgs, wq_slice_view* out) {
    if (!h || !in || !out) return WQ_E_INVALID;
    if (!h->multi) return set_error(h, WQ_E_INVALID, "wq_route_tick_slices_device needs a multi-GPU handle");
    WQ_HIP(h, hipSetDevice(h->device));
    return multi_route_slices(h, in, with_msgs, out);
}
