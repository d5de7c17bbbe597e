// wq_table.hip — building the cube -> peer-list hash table on the GPU.
//
// Replaces the mutation side of the reference subscription table:
//   AreaMap::add_subscription     worldql_server/src/subscriptions/area_map.rs:72-85
//   AreaMap::remove_subscription  area_map.rs:88-119
//   AreaMap::remove_peer / WorldMap::remove_peer  area_map.rs:124-135, world_map.rs:41-61
// The reference applies ops one by one on a single task (processing/thread.rs:113-148). Here a
// batch of ops is applied at once with identical results: the state is the SET of live
// (world, cube, peer) triples, and for each triple the last op of the batch decides its
// presence (sub and unsub are single-element set ops).
//
// Pipeline (all on the handle's stream):
//   events  = live entries (as "present" events) ++ ops (quantised by kernel (1), hashed)
//   order   = stable radix sort by (hash, peer)  [exact multi-key sort if two cubes share a hash]
//   state'  = last event of every (cube, peer) run that is a subscribe
//   derived = per-cube peer lists (list[off] = count, then ascending peers), the open-addressed
//             slot table (32-byte records, load <= 1/2), and sorted unique (world<<32 | peer)
//             keys for is_peer_subscribed_any / get_subscribed_any_peers (area_map.rs:46-67).
// Sorting uses rocPRIM's radix sort (AMD's native primitive library); every other step is a
// kernel in this file.
#include <cstring>

#include <algorithm>

#include <cstdlib>
#include "table_prims.hpp"

namespace wq {

namespace {

__global__ void k_ops_to_events(const wq_op* __restrict__ ops, uint32_t n, uint64_t base,
                                double sf, int64_t si, uint64_t hmask, uint64_t* ev_h,
                                uint32_t* ev_w, int64_t* ev_kx, int64_t* ev_ky, int64_t* ev_kz,
                                uint32_t* ev_p, uint8_t* ev_kind, uint32_t* flag) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const wq_op o = ops[i];
    if (o.kind > WQ_OP_UNSUBSCRIBE || o.world == WQ_WORLD_INVALID) atomicOr(flag, 2u);  // bad op
    int64_t k0, k1, k2;
    if (o.key_is_raw) {  // impl ToCubeArea for CubeArea: identity (cube_area.rs:65-70)
        k0 = o.u.key[0];
        k1 = o.u.key[1];
        k2 = o.u.key[2];
    } else {  // impl ToCubeArea for Vector3 -> CubeArea::from_vector3 (cube_area.rs:50-56)
        k0 = coord_clamp_dev(o.u.pos[0], sf, si);
        k1 = coord_clamp_dev(o.u.pos[1], sf, si);
        k2 = coord_clamp_dev(o.u.pos[2], sf, si);
    }
    const uint64_t e = base + i;
    ev_h[e] = cube_hash(o.world, k0, k1, k2) & hmask;
    ev_w[e] = o.world;
    ev_kx[e] = k0;
    ev_ky[e] = k1;
    ev_kz[e] = k2;
    ev_p[e] = o.peer;
    ev_kind[e] = (o.kind == WQ_OP_SUBSCRIBE) ? 1 : 0;
}

__global__ void k_fill_u8(uint8_t* a, uint64_t n, uint8_t v) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) a[i] = v;
}

struct EvView {
    const uint64_t* h;
    const uint32_t* w;
    const int64_t *kx, *ky, *kz;
    const uint32_t* p;
    __device__ bool same_cube(uint32_t a, uint32_t b) const {
        return h[a] == h[b] && w[a] == w[b] && kx[a] == kx[b] && ky[a] == ky[b] && kz[a] == kz[b];
    }
};

// After the (hash, peer) sort: two different cubes with one hash in adjacent positions.
__global__ void k_detect_collision(EvView ev, const uint32_t* __restrict__ order, uint64_t n,
                                   uint32_t* flag) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i == 0 || i >= n) return;
    const uint32_t a = order[i - 1], b = order[i];
    if (ev.h[a] == ev.h[b] && !ev.same_cube(a, b)) atomicOr(flag, 1u);
}

// keep[i] = event i (in sorted order) is the last one of its (cube, peer) run and subscribes.
__global__ void k_mark_last(EvView ev, const uint8_t* __restrict__ kind,
                            const uint32_t* __restrict__ order, uint64_t n, uint32_t* keep) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = order[i];
    bool last = true;
    if (i + 1 < n) {
        const uint32_t b = order[i + 1];
        last = !(ev.p[a] == ev.p[b] && ev.same_cube(a, b));
    }
    keep[i] = (last && kind[a]) ? 1u : 0u;
}

struct StOut {
    uint64_t* h;
    uint32_t* w;
    int64_t *kx, *ky, *kz;
    uint32_t* p;
};

__global__ void k_scatter_state(EvView ev, const uint32_t* __restrict__ order,
                                const uint32_t* __restrict__ keep, const uint32_t* __restrict__ pos,
                                uint64_t n, StOut out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !keep[i]) return;
    const uint32_t a = order ? order[i] : (uint32_t)i;
    const uint32_t j = pos[i];
    out.h[j] = ev.h[a];
    out.w[j] = ev.w[a];
    out.kx[j] = ev.kx[a];
    out.ky[j] = ev.ky[a];
    out.kz[j] = ev.kz[a];
    out.p[j] = ev.p[a];
}

__global__ void k_cube_heads(EvView st, uint64_t n, uint32_t* head) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || !st.same_cube((uint32_t)i - 1, (uint32_t)i)) ? 1u : 0u;
}

// cid = inclusive scan of head: cube index of entry i is cid[i] - 1.
__global__ void k_cube_start(const uint32_t* __restrict__ head, const uint32_t* __restrict__ cid,
                             uint64_t n, uint32_t n_cubes, uint32_t* cube_start) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && head[i]) cube_start[cid[i] - 1] = (uint32_t)i;
    if (i == 0) cube_start[n_cubes] = (uint32_t)n;
}

// Words of cube c's list block: [count, peers..., headroom] (list_capacity, wq_device.hpp). With
// `align`, a cube with more than kInline peers (the only lists a tick reads) gets its block in a
// region of its own, sized in whole 128-byte lines with its count in the last word of the first line,
// so its peers start on a line: the emit copies a list of L peers from ceil(L / 32) lines instead of
// straddling one more half of the time (C3: 3.2M list reads per tick). words_s / words_l: the block in
// the short / long region (the other is 0).
constexpr uint32_t kListLine = 32;  // words per 128-byte line
__global__ void k_list_words(const uint32_t* __restrict__ cube_start, uint32_t n_cubes, uint32_t* words_s,
                             uint32_t* words_l, int align) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= n_cubes) return;
    const uint32_t cnt = cube_start[c + 1] - cube_start[c];
    const uint32_t cap = list_capacity(cnt);
    const bool lng = align && cnt > (uint32_t)kInline;
    words_s[c] = lng ? 0u : 1u + cap;
    words_l[c] = lng ? kListLine + ((cap + kListLine - 1) / kListLine) * kListLine : 0u;
}

// Final list offsets (into loff_s, in place): long blocks first (count word at the end of their first
// line), the short region after them.
__global__ void k_list_offsets(uint32_t* loff_s, const uint32_t* __restrict__ words_l,
                               const uint32_t* __restrict__ loff_l, uint32_t n_cubes, uint32_t total_l) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= n_cubes) return;
    loff_s[c] = words_l[c] ? loff_l[c] + (kListLine - 1) : total_l + loff_s[c];
}

// Cube c's entries [s_c, s_{c+1}) land at list[loff_c + 1 ...], its count at list[loff_c].
__global__ void k_fill_lists(const uint32_t* __restrict__ st_p, const uint32_t* __restrict__ head,
                             const uint32_t* __restrict__ cid, const uint32_t* __restrict__ cube_start,
                             const uint32_t* __restrict__ loff, uint64_t n, uint32_t* list) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = cid[i] - 1;
    const uint32_t j = (uint32_t)i - cube_start[c];
    list[loff[c] + 1 + j] = st_p[i];
    if (head[i]) list[loff[c]] = cube_start[c + 1] - (uint32_t)i;
}

// Regular cubes -> 128-byte records (one line per lookup); the rest -> 32-byte full-key slots.
__global__ void k_insert_cubes(EvView st, const uint32_t* __restrict__ cube_start,
                               const uint32_t* __restrict__ loff, uint32_t n_cubes, uint32_t* rclaim, Record* recs, uint64_t rmask, int rshift, uint32_t* claim,
                               Slot* slots, uint64_t mask, int shift, uint64_t hmask, double sf) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= n_cubes) return;
    const uint32_t j = cube_start[c];
    const uint32_t cnt = cube_start[c + 1] - j;
    uint64_t pk;
    uint32_t ext;
    if (pack_key(st.w[j], st.kx[j], st.ky[j], st.kz[j], sf, &pk, &ext)) {
        uint64_t s = slot_of(rec_hash(pk, ext) & hmask, rshift);
        // claim words: 0 free, 1 being claimed, >= 2 holds a key (wq_delta.hip); c + 2 < 2^31, as
        // 2^31 records would take 256 GiB
        while (atomicCAS(&rclaim[s], 0u, c + 2) != 0u) s = (s + 1) & rmask;
        Record& r = recs[s];
        r.pk = pk;
        r.ext = ext;
        r.count = cnt;
        r.list_off = loff[c];
        uint64_t sig = 0;
        for (uint32_t i = 0; i < cnt; ++i) sig |= peer_sig(st.p[j + i]);
        r.sig = sig;
        r.cap = list_capacity(cnt);
#pragma unroll 2
        for (int i = 0; i < kInline; ++i) r.peers[i] = (uint32_t)i < cnt ? st.p[j + i] : 0xFFFFFFFFu;
        return;
    }
    uint64_t s = slot_of(st.h[j], shift);
    while (atomicCAS(&claim[s], 0u, c + 1) != 0u) s = (s + 1) & mask;
    Slot r;
    r.k[0] = st.kx[j];
    r.k[1] = st.ky[j];
    r.k[2] = st.kz[j];
    r.world = st.w[j];
    r.off = loff[c];
    slots[s] = r;
}

__global__ void k_max_peer(const uint32_t* __restrict__ p, uint64_t n, uint32_t* out) {
    __shared__ uint32_t wmax[kBlock / 64];
    uint32_t v = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        v = max(v, p[i]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 1; k < kBlock / 64; ++k) v = max(v, wmax[k]);
        atomicMax(out, v);  // one atomic per block
    }
}

__global__ void k_box_init(uint32_t* box, uint32_t n_peers) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n_peers) {
        uint32_t* b = box + (uint64_t)kBoxWords * i;
        b[0] = b[2] = b[4] = b[6] = 0xFFFFFFFFu;  // minima
        b[1] = b[3] = b[5] = b[7] = 0u;           // maxima
    }
    if (i == 0) box[(uint64_t)kBoxWords * n_peers] = 1u;  // valid
}

// Every live entry of a record cube widens its peer's box.
__global__ void k_box_build(EvView st, uint64_t n, double sf, uint32_t* box) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint64_t pk;
    uint32_t ext;
    if (pack_key(st.w[i], st.kx[i], st.ky[i], st.kz[i], sf, &pk, &ext))
        box_add(box + (uint64_t)kBoxWords * st.p[i], pk, ext);
}

__global__ void k_any_keys(const uint32_t* __restrict__ w, const uint32_t* __restrict__ p, uint64_t n,
                           uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = ((uint64_t)w[i] << 32) | p[i];
}

__global__ void k_unique_flags(const uint64_t* __restrict__ a, uint64_t n, uint32_t* flags) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) flags[i] = (i == 0 || a[i] != a[i - 1]) ? 1u : 0u;
}

__global__ void k_scatter_flagged_u64(const uint64_t* __restrict__ a, const uint32_t* __restrict__ flags,
                                      const uint32_t* __restrict__ pos, uint64_t n, uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && flags[i]) out[pos[i]] = a[i];
}

EvView ev_view(wq_router* h) {
    return EvView{h->ev_h.as<uint64_t>(), h->ev_w.as<uint32_t>(), h->ev_kx.as<int64_t>(),
                  h->ev_ky.as<int64_t>(), h->ev_kz.as<int64_t>(), h->ev_p.as<uint32_t>()};
}
EvView st_view(const State& s) {
    return EvView{s.h.as<uint64_t>(), s.w.as<uint32_t>(), s.kx.as<int64_t>(), s.ky.as<int64_t>(),
                  s.kz.as<int64_t>(), s.p.as<uint32_t>()};
}


// Stable LSD sort of `order` by one key column (gathered through the current order).
template <typename K>
int refine_by(wq_router* h, const K* column, uint64_t n, int bits) {
    uint32_t* cur = h->idx_b.as<uint32_t>();
    uint32_t* nxt = h->idx_a.as<uint32_t>();
    K* kg = reinterpret_cast<K*>(h->key64_a.p);
    K* ks = reinterpret_cast<K*>(h->key64_b.p);
    hipLaunchKernelGGL(k_gather<K>, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, column, cur, kg, n);
    int rc = sort_pairs<K>(h, kg, ks, cur, nxt, n, bits);
    if (rc) return rc;
    WQ_HIP(h, hipMemcpyAsync(cur, nxt, n * 4, hipMemcpyDeviceToDevice, h->stream));
    return WQ_OK;
}

}  // namespace

int build_any(wq_router* h);

int set_error(wq_router* h, int code, const char* what, hipError_t e) {
    if (h) {
        h->err = what;
        if (e != hipSuccess) {
            h->err += ": ";
            h->err += hipGetErrorString(e);
        }
    }
    return code;
}

// Apply one batch of subscribe / unsubscribe ops (no REMOVE_PEER inside).
int table_rebuild_batch(wq_router* h, size_t n_ops);

int table_apply_segment(wq_router* h, const wq_op* ops, size_t n_ops, bool on_device) {
    if (n_ops == 0) return WQ_OK;
    hipStream_t s = h->stream;
    // the previous incremental batch first (it may need re-applying from h->d_ops, so before the
    // upload below overwrites it)
    int rc = table_resolve(h, true);
    if (rc) return rc;
    h->table_gen++;
    h->tab.hdr_ok = false;  // an in-place batch leaves the dense headers behind; a rebuild refills them
    if (on_device) {
        h->cur_ops = ops;
    } else {
        WQ_ALLOC(h, h->d_ops, n_ops * sizeof(wq_op));
        WQ_HIP(h, hipMemcpyAsync(h->d_ops.p, ops, n_ops * sizeof(wq_op), hipMemcpyHostToDevice, s));
        h->cur_ops = h->d_ops.as<wq_op>();
    }
    // small batches against a built table: update the touched cubes in place (wq_delta.hip). The
    // entry count may lag by REMOVE_PEER deltas not yet read back: it only picks the path.
    if (h->st.n && h->tab.n_cubes && 4 * n_ops <= h->st.n) {
        bool applied = false;
        if ((rc = table_apply_delta(h, n_ops, &applied))) return rc;
        if (applied) return WQ_OK;
    }
    return table_rebuild_batch(h, n_ops);
}

// The full rebuild: the live state plus the batch h->cur_ops, sorted and reduced "last op wins".
int table_rebuild_batch(wq_router* h, size_t n_ops) {
    hipStream_t s = h->stream;
    int rc;
    if ((rc = table_sync_delta_stats(h))) return rc;
    const uint64_t S = h->st.n;
    const uint64_t N = S + n_ops;
    if (N >= 0xFFFFFFFFull) return set_error(h, WQ_E_INVALID, "more than 2^32-1 subscription events");
    WQ_ALLOC(h, h->ev_h, N * 8);
    WQ_ALLOC(h, h->ev_w, N * 4);
    WQ_ALLOC(h, h->ev_kx, N * 8);
    WQ_ALLOC(h, h->ev_ky, N * 8);
    WQ_ALLOC(h, h->ev_kz, N * 8);
    WQ_ALLOC(h, h->ev_p, N * 4);
    WQ_ALLOC(h, h->ev_kind, N);
    WQ_ALLOC(h, h->idx_a, N * 4);
    WQ_ALLOC(h, h->idx_b, N * 4);
    WQ_ALLOC(h, h->key32_a, N * 4);
    WQ_ALLOC(h, h->key64_a, N * 8);
    WQ_ALLOC(h, h->key64_b, N * 8);
    WQ_ALLOC(h, h->flags, N * 4);
    WQ_ALLOC(h, h->scan, N * 4);
    WQ_ALLOC(h, h->small, 64);
    if (h->st_stale && (rc = table_materialize(h))) return rc;
    // live entries first: they are the earliest "present" events
    if (S) {
        WQ_HIP(h, hipMemcpyAsync(h->ev_h.p, h->st.h.p, S * 8, hipMemcpyDeviceToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(h->ev_w.p, h->st.w.p, S * 4, hipMemcpyDeviceToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(h->ev_kx.p, h->st.kx.p, S * 8, hipMemcpyDeviceToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(h->ev_ky.p, h->st.ky.p, S * 8, hipMemcpyDeviceToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(h->ev_kz.p, h->st.kz.p, S * 8, hipMemcpyDeviceToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(h->ev_p.p, h->st.p.p, S * 4, hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_fill_u8, dim3(grid_for(S)), dim3(kBlock), 0, s, h->ev_kind.as<uint8_t>(), S,
                           (uint8_t)1);
    }
    uint32_t* dflag = h->small.as<uint32_t>();
    WQ_HIP(h, hipMemsetAsync(dflag, 0, 4, s));
    hipLaunchKernelGGL(k_ops_to_events, dim3(grid_for(n_ops)), dim3(kBlock), 0, s, h->cur_ops,
                       (uint32_t)n_ops, S, (double)h->cube_size, (int64_t)h->cube_size, h->hash_mask,
                       h->ev_h.as<uint64_t>(), h->ev_w.as<uint32_t>(), h->ev_kx.as<int64_t>(),
                       h->ev_ky.as<int64_t>(), h->ev_kz.as<int64_t>(), h->ev_p.as<uint32_t>(),
                       h->ev_kind.as<uint8_t>(), dflag);
    WQ_HIP(h, hipGetLastError());

    // order = stable sort by (hash, peer): sort by peer, then stably by hash
    uint32_t* idx_a = h->idx_a.as<uint32_t>();
    uint32_t* idx_b = h->idx_b.as<uint32_t>();
    hipLaunchKernelGGL(k_iota, dim3(grid_for(N)), dim3(kBlock), 0, s, idx_a, N);
    rc = sort_pairs<uint32_t>(h, h->ev_p.as<uint32_t>(), h->key32_a.as<uint32_t>(), idx_a, idx_b, N, 32);
    if (rc) return rc;
    hipLaunchKernelGGL(k_gather<uint64_t>, dim3(grid_for(N)), dim3(kBlock), 0, s, h->ev_h.as<uint64_t>(),
                       idx_b, h->key64_a.as<uint64_t>(), N);
    rc = sort_pairs<uint64_t>(h, h->key64_a.as<uint64_t>(), h->key64_b.as<uint64_t>(), idx_b, idx_a, N, 64);
    if (rc) return rc;
    uint32_t* order = idx_a;

    EvView ev = ev_view(h);
    hipLaunchKernelGGL(k_detect_collision, dim3(grid_for(N)), dim3(kBlock), 0, s, ev, order, N, dflag);
    uint32_t collided = 0;
    rc = read_u32(h, dflag, 0, &collided);
    if (rc) return rc;
    if (collided & 2u) return set_error(h, WQ_E_INVALID, "bad op (kind or reserved world id)");
    if (collided & 1u) {
        // exact path: LSD passes peer, kz, ky, kx, world, hash over the original event order
        h->hash_fallbacks++;
        hipLaunchKernelGGL(k_iota, dim3(grid_for(N)), dim3(kBlock), 0, s, idx_b, N);
        if ((rc = refine_by<uint32_t>(h, h->ev_p.as<uint32_t>(), N, 32))) return rc;
        if ((rc = refine_by<uint64_t>(h, reinterpret_cast<const uint64_t*>(h->ev_kz.p), N, 64))) return rc;
        if ((rc = refine_by<uint64_t>(h, reinterpret_cast<const uint64_t*>(h->ev_ky.p), N, 64))) return rc;
        if ((rc = refine_by<uint64_t>(h, reinterpret_cast<const uint64_t*>(h->ev_kx.p), N, 64))) return rc;
        if ((rc = refine_by<uint32_t>(h, h->ev_w.as<uint32_t>(), N, 32))) return rc;
        if ((rc = refine_by<uint64_t>(h, h->ev_h.as<uint64_t>(), N, 64))) return rc;
        order = idx_b;
    }

    // last op wins per (cube, peer)
    uint32_t* keep = h->flags.as<uint32_t>();
    uint32_t* pos = h->scan.as<uint32_t>();
    hipLaunchKernelGGL(k_mark_last, dim3(grid_for(N)), dim3(kBlock), 0, s, ev, h->ev_kind.as<uint8_t>(),
                       order, N, keep);
    if ((rc = scan_u32(h, keep, pos, N, false))) return rc;
    uint32_t last_pos = 0, last_keep = 0;
    if ((rc = read_u32(h, pos, N - 1, &last_pos))) return rc;
    if ((rc = read_u32(h, keep, N - 1, &last_keep))) return rc;
    const uint64_t S_new = (uint64_t)last_pos + last_keep;
    if ((rc = ensure_state(h, h->st_next, S_new))) return rc;
    StOut out{h->st_next.h.as<uint64_t>(), h->st_next.w.as<uint32_t>(), h->st_next.kx.as<int64_t>(),
              h->st_next.ky.as<int64_t>(), h->st_next.kz.as<int64_t>(), h->st_next.p.as<uint32_t>()};
    hipLaunchKernelGGL(k_scatter_state, dim3(grid_for(N)), dim3(kBlock), 0, s, ev, order, keep, pos, N, out);
    WQ_HIP(h, hipGetLastError());
    std::swap(h->st, h->st_next);
    h->st.n = S_new;
    return table_rebuild_derived(h);
}

// WorldMap::remove_peer / AreaMap::remove_peer for sorted unique (world << 32 | peer) keys
// (world_map.rs:41-61, area_map.rs:124-135).
int table_remove_peers(wq_router* h, const uint64_t* keys, size_t n_rm) {
    // one in-place pass over every cube's list (wq_delta.hip); the state and any-keys go stale
    if (int rc = table_resolve(h, true)) return rc;
    if (n_rm == 0 || (h->st.n == 0 && !h->dstat_pending)) return WQ_OK;
    h->table_gen++;
    h->tab.hdr_ok = false;
    return table_remove_peers_inplace(h, keys, n_rm);
}

// Compact headers: every occupied record (ext != 0; emptied cubes keep theirs) claims the first free
// slot of its probe run in the header table by a CAS on the header's ext word (each cube is inserted
// once, so a claimed slot is simply passed), then writes {pk, count, list_off | sig, record slot}.
__global__ void k_hdr_compact(const uint4* __restrict__ recs, uint64_t n, uint4* __restrict__ hdr, uint64_t hmask,
                              int hshift, uint64_t hash_mask, uint32_t blk) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint4 a = recs[8 * i], b = recs[8 * i + 1];
    if (b.w == 0) return;  // an empty record slot
    const uint64_t pk = ((uint64_t)a.y << 32) | a.x;
    uint64_t s = hdr_home(pk, b.w, hash_mask, hshift, blk);
    for (;;) {
        uint32_t* ext_word = reinterpret_cast<uint32_t*>(hdr + 2 * s + 1) + 3;
        if (atomicCAS(ext_word, 0u, b.w) == 0u) break;
        s = (s + 1) & hmask;
    }
    hdr[2 * s] = a;
    uint2* w2 = reinterpret_cast<uint2*>(hdr + 2 * s + 1);
    w2[0] = make_uint2(b.x, b.y);                           // sig
    reinterpret_cast<uint32_t*>(hdr + 2 * s + 1)[2] = (uint32_t)i;  // the record slot (ext already set)
}

__global__ void k_hdr_fill(const uint4* __restrict__ recs, uint64_t n, uint4* __restrict__ hdr) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    hdr[2 * i] = recs[8 * i];
    hdr[2 * i + 1] = recs[8 * i + 1];
}

// Per-cube lists, slot table and the (world, peer) "any" keys from the sorted state.
int table_rebuild_derived(wq_router* h) {
    hipStream_t s = h->stream;
    const uint64_t S = h->st.n;
    Table& t = h->tab;
    int rc;
    uint32_t n_cubes = 0;
    uint64_t list_words = 0;
    EvView st = st_view(h->st);
    if (S) {
        WQ_ALLOC(h, h->flags, S * 4);
        WQ_ALLOC(h, h->scan, S * 4);
        uint32_t* head = h->flags.as<uint32_t>();
        uint32_t* cid = h->scan.as<uint32_t>();
        hipLaunchKernelGGL(k_cube_heads, dim3(grid_for(S)), dim3(kBlock), 0, s, st, S, head);
        if ((rc = scan_u32(h, head, cid, S, true))) return rc;
        if ((rc = read_u32(h, cid, S - 1, &n_cubes))) return rc;
        WQ_ALLOC(h, h->cube_start, ((uint64_t)n_cubes + 1) * 4);
        hipLaunchKernelGGL(k_cube_start, dim3(grid_for(S)), dim3(kBlock), 0, s, head, cid, S, n_cubes,
                           h->cube_start.as<uint32_t>());
        // list blocks with headroom (list_capacity), then room for lists that incremental updates
        // relocate (wq_delta.hip)
        WQ_ALLOC(h, h->cube_id, (uint64_t)n_cubes * 16);
        uint32_t* words = h->cube_id.as<uint32_t>();
        uint32_t* loff = words + n_cubes;  // the final offsets end up here (k_insert_cubes reads them)
        uint32_t* words_l = loff + n_cubes;
        uint32_t* loff_l = words_l + n_cubes;
        // aligned long lists (default; WQ_LIST_ALIGN=0: every block packed back to back, as before)
        static const int align = !getenv("WQ_LIST_ALIGN") || atoi(getenv("WQ_LIST_ALIGN")) != 0;
        hipLaunchKernelGGL(k_list_words, dim3(grid_for(n_cubes)), dim3(kBlock), 0, s, h->cube_start.as<uint32_t>(),
                           n_cubes, words, words_l, align);
        if ((rc = scan_u32(h, words, loff, n_cubes, false))) return rc;
        if ((rc = scan_u32(h, words_l, loff_l, n_cubes, false))) return rc;
        uint32_t lw = 0, lo = 0, lwl = 0, lol = 0;
        if ((rc = read_u32(h, words, n_cubes - 1, &lw))) return rc;
        if ((rc = read_u32(h, loff, n_cubes - 1, &lo))) return rc;
        if ((rc = read_u32(h, words_l, n_cubes - 1, &lwl))) return rc;
        if ((rc = read_u32(h, loff_l, n_cubes - 1, &lol))) return rc;
        const uint64_t total_l = (uint64_t)lol + lwl;
        if (total_l + (uint64_t)lo + lw >= 0xFFFFFFFFull) return set_error(h, WQ_E_INVALID, "subscription lists exceed 2^32 words");
        hipLaunchKernelGGL(k_list_offsets, dim3(grid_for(n_cubes)), dim3(kBlock), 0, s, loff, words_l, loff_l, n_cubes,
                           (uint32_t)total_l);
        list_words = total_l + (uint64_t)lo + lw;
        if (list_words + list_words / 2 + 65536 >= 0xFFFFFFFFull)
            return set_error(h, WQ_E_INVALID, "subscription lists exceed 2^32 words");
        WQ_ALLOC(h, t.list, (list_words + list_words / 2 + 65536) * 4);
        hipLaunchKernelGGL(k_fill_lists, dim3(grid_for(S)), dim3(kBlock), 0, s, h->st.p.as<uint32_t>(), head,
                           cid, h->cube_start.as<uint32_t>(), loff, S, t.list.as<uint32_t>());
    } else {
        WQ_ALLOC(h, t.list, 4);
    }
    // slot table: capacity = pow2 >= max(1024, 2 * cubes), so every probe walk meets an empty slot
    uint64_t cap = 1024;
    int log2cap = 10;
    while (cap < 2ull * n_cubes) {
        cap <<= 1;
        log2cap++;
    }
    WQ_ALLOC(h, t.slots, cap * sizeof(Slot));
    WQ_ALLOC(h, t.claim, cap * 4);
    WQ_HIP(h, hipMemsetAsync(t.slots.p, 0xFF, cap * sizeof(Slot), s));
    WQ_HIP(h, hipMemsetAsync(t.claim.p, 0, cap * 4, s));
    t.cap = cap;
    t.shift = 64 - log2cap;
    // record table: load <= 1/8, so ~97% of lookups end at the home slot (one round trip). The
    // untouched slots cost memory, not time: a tick touches one line per cube whatever the capacity
    uint64_t rcap = 1024;
    int log2r = 10;
    while (rcap < (uint64_t)h->rec_slack * n_cubes) {
        rcap <<= 1;
        log2r++;
    }
    // Round 6: the count probes the compact headers (their own table), so past them a tick only reads
    // a record at a known slot and the record table's load barely matters — its footprint does.
    // WQ_REC_CAP_GB=G halves a default-slack table of more than G GiB while its load stays <= 1/4
    // (C3: 17.2 -> 8.6 GB of records). Opt-in: four boxes measured the C3 tick with and without it
    // (profiles/r06_record_cap_ab.json) — faster on one (emit 977 -> 900 us), slower on one
    // (900 -> 970 us), equal on two; the 900/975 us emit modes follow the box and the allocation, not
    // the table size. An explicit wq_debug_set_record_slack is kept as is.
    static const double cap_gb = getenv("WQ_REC_CAP_GB") ? atof(getenv("WQ_REC_CAP_GB")) : 0.0;
    while (cap_gb > 0.0 && !h->rec_slack_set && (double)rcap * sizeof(Record) > cap_gb * 1073741824.0 && rcap / 2 >= 4ull * n_cubes) {
        rcap >>= 1;
        log2r--;
    }
    // WQ_CONTIG=1: the record table as one hipDeviceMallocContiguous allocation (hipMalloc if that
    // fails). Measured equal to hipMalloc on a box in the fast emit mode (r06_record_cap_ab.json).
    static const bool contig = getenv("WQ_CONTIG") && atoi(getenv("WQ_CONTIG")) != 0;
    t.recs.flags = t.hdr.flags = contig ? hipDeviceMallocContiguous : 0u;
    WQ_ALLOC(h, t.recs, rcap * sizeof(Record));
    if (contig) fprintf(stderr, "wq: WQ_CONTIG record table %.2f GB contiguous: %d\n", t.recs.bytes / 1e9, (int)t.recs.flagged);
    WQ_ALLOC(h, t.rclaim, rcap * 4);
    WQ_HIP(h, hipMemsetAsync(t.recs.p, 0, rcap * sizeof(Record), s));
    WQ_HIP(h, hipMemsetAsync(t.rclaim.p, 0, rcap * 4, s));
    t.rec_cap = rcap;
    t.rec_shift = 64 - log2r;
    if (n_cubes)
        hipLaunchKernelGGL(k_insert_cubes, dim3(grid_for(n_cubes)), dim3(kBlock), 0, s, st,
                           h->cube_start.as<uint32_t>(), h->cube_id.as<uint32_t>() + n_cubes, n_cubes,
                           t.rclaim.as<uint32_t>(), t.recs.as<Record>(),
                           rcap - 1, t.rec_shift, t.claim.as<uint32_t>(), t.slots.as<Slot>(), cap - 1, t.shift,
                           h->hash_mask, (double)h->cube_size);
    // per-peer boxes (PeerBox, wq_device.hpp) for the peers the build holds; an incremental batch
    // switches them off until the next build (wq_delta.hip)
    t.n_pbox = 0;
    if (S) {
        uint32_t* mx = h->small.as<uint32_t>();
        WQ_HIP(h, hipMemsetAsync(mx, 0, 4, s));
        hipLaunchKernelGGL(k_max_peer, dim3(std::min<unsigned>(grid_for(S), 2048u)), dim3(kBlock), 0, s,
                           h->st.p.as<uint32_t>(), S, mx);
        uint32_t max_peer = 0;
        if ((rc = read_u32(h, mx, 0, &max_peer))) return rc;
        const uint64_t cap = (uint64_t)max_peer + 1;
        if (cap < 0xFFFFFFF0ull) {
            WQ_ALLOC(h, t.pbox, (cap * kBoxWords + 1) * 4);
            hipLaunchKernelGGL(k_box_init, dim3(grid_for(cap)), dim3(kBlock), 0, s, t.pbox.as<uint32_t>(),
                               (uint32_t)cap);
            hipLaunchKernelGGL(k_box_build, dim3(grid_for(S)), dim3(kBlock), 0, s, st, S, (double)h->cube_size,
                               t.pbox.as<uint32_t>());
            t.n_pbox = (uint32_t)cap;
        }
    }
    // dense headers (TableView::hdr): the records' first 32 bytes at the same slot index, 4 per line,
    // read by the count pass's probes (C3: count 368 -> 351 us, tick -1.4%, same box; WQ_HDR=0: off)
    t.hdr_ok = false;
    t.hdr_cap = 0;
    t.hdr_shift = 64;
    t.hdr_blk = 0;
    static const bool want_hdr = !getenv("WQ_HDR") || atoi(getenv("WQ_HDR")) != 0;
    // compact headers (default): their own table of >= WQ_HDR_SLOTS header slots per cube (default 4:
    // load <= 1/4, 1/8 after the power-of-two rounding of C3's 8.56M cubes; C3 count 344.5-345.2 us
    // with one header per record slot, 350.6 at 2 slots per cube, 453 at 1 — the probe runs, not the
    // lines' reuse, decide); WQ_HDR_COMPACT=0: the round-4 layout, one header per record slot
    static const bool compact = !getenv("WQ_HDR_COMPACT") || atoi(getenv("WQ_HDR_COMPACT")) != 0;
    static const uint64_t hslots = getenv("WQ_HDR_SLOTS") ? std::max(1ul, strtoul(getenv("WQ_HDR_SLOTS"), nullptr, 10)) : 4ul;
    if (want_hdr && compact) {
        uint64_t hcap = 1024;
        int log2h = 10;
        while (hcap < hslots * n_cubes || hcap < n_cubes + 1) {
            hcap <<= 1;
            log2h++;
        }
        WQ_ALLOC(h, t.hdr, hcap * 32);
        WQ_HIP(h, hipMemsetAsync(t.hdr.p, 0, hcap * 32, s));
        t.hdr_cap = hcap;
        t.hdr_shift = 64 - log2h;
        // WQ_HDR_BLOCK = 4 / 8: neighbouring cubes' headers grouped per 2 x 2 / 2 x 2 x 2 block
        // (wq_device.hpp hdr_home; round-5 verdict item 6)
        static const uint32_t blk_env = getenv("WQ_HDR_BLOCK") ? (uint32_t)atoi(getenv("WQ_HDR_BLOCK")) : 0u;
        t.hdr_blk = blk_env == 4 || blk_env == 8 ? blk_env : 0u;
        hipLaunchKernelGGL(k_hdr_compact, dim3(grid_for(rcap)), dim3(kBlock), 0, s, t.recs.as<uint4>(), rcap,
                           t.hdr.as<uint4>(), hcap - 1, t.hdr_shift, h->hash_mask, t.hdr_blk);
        t.hdr_ok = true;
    } else if (want_hdr) {
        WQ_ALLOC(h, t.hdr, rcap * 32);
        hipLaunchKernelGGL(k_hdr_fill, dim3(grid_for(rcap)), dim3(kBlock), 0, s, t.recs.as<uint4>(), rcap,
                           t.hdr.as<uint4>());
        t.hdr_ok = true;
    }
    t.n_cubes = n_cubes;
    t.n_recs = n_cubes;
    t.list_used = list_words;
    t.list_cap = t.list.bytes / 4;
    h->st_stale = false;
    if ((rc = build_any(h))) return rc;
    WQ_HIP(h, hipGetLastError());
    WQ_HIP(h, hipStreamSynchronize(s));
    return WQ_OK;
}

// Sorted unique (world << 32 | peer) keys from the (fresh) state.
int build_any(wq_router* h) {
    hipStream_t s = h->stream;
    const uint64_t S = h->st.n;
    Table& t = h->tab;
    int rc;
    t.n_any = 0;
    if (S) {
        WQ_ALLOC(h, h->key64_a, S * 8);
        WQ_ALLOC(h, h->key64_b, S * 8);
        WQ_ALLOC(h, h->flags, S * 4);
        WQ_ALLOC(h, h->scan, S * 4);
        hipLaunchKernelGGL(k_any_keys, dim3(grid_for(S)), dim3(kBlock), 0, s, h->st.w.as<uint32_t>(),
                           h->st.p.as<uint32_t>(), S, h->key64_a.as<uint64_t>());
        if ((rc = sort_keys_u64(h, h->key64_a.as<uint64_t>(), h->key64_b.as<uint64_t>(), S))) return rc;
        uint32_t* fl = h->flags.as<uint32_t>();
        uint32_t* ps = h->scan.as<uint32_t>();
        hipLaunchKernelGGL(k_unique_flags, dim3(grid_for(S)), dim3(kBlock), 0, s, h->key64_b.as<uint64_t>(), S,
                           fl);
        if ((rc = scan_u32(h, fl, ps, S, false))) return rc;
        uint32_t lp = 0, lf = 0;
        if ((rc = read_u32(h, ps, S - 1, &lp))) return rc;
        if ((rc = read_u32(h, fl, S - 1, &lf))) return rc;
        t.n_any = (uint64_t)lp + lf;
        WQ_ALLOC(h, t.any, t.n_any * 8);
        hipLaunchKernelGGL(k_scatter_flagged_u64, dim3(grid_for(S)), dim3(kBlock), 0, s,
                           h->key64_b.as<uint64_t>(), fl, ps, S, t.any.as<uint64_t>());
    } else {
        WQ_ALLOC(h, t.any, 8);
    }
    h->any_stale = false;
    return WQ_OK;
}

int table_ensure_any(wq_router* h) {
    if (!h->any_stale) return WQ_OK;
    int rc;
    if (h->st_stale && (rc = table_materialize(h))) return rc;
    if ((rc = build_any(h))) return rc;
    WQ_HIP(h, hipGetLastError());
    WQ_HIP(h, hipStreamSynchronize(h->stream));
    return WQ_OK;
}

}  // namespace wq
