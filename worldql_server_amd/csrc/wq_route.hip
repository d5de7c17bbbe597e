// wq_route.hip — the LocalMessage hot path on gfx950: one tick of messages in ONE launch.
//
// Replaces, per message, worldql_server/src/processing/local_message.rs:52-86:
//   world_map.get(world) -> Vector3::to_cube_area (cube_area.rs:72-77 -> coord_clamp :23-44)
//   -> AreaMap::get_subscribed_peers (area_map.rs:52-60) -> replication filter (:60-86).
//
// route_kernel (256 threads = 4 waves, one tile of kTile messages per workgroup):
//   phase 1  quantise (kernel 1), hash, probe the open-addressed table (kernel 2), read the
//            bucket's peer count and binary-search the sender in its ascending peer list, so the
//            filtered count e_m and a branch-free "output j -> list index" map are known;
//            per-message (list base, skipped index) are staged in LDS.
//   phase 2  workgroup exclusive scan of e_m (wave shuffles + LDS), then a single-pass
//            decoupled look-back over per-tile status words (one 8-byte agent-scope atomic each:
//            flag + value, so no separate payload hand-off) gives the tile's global output base.
//            Tile ids come from an atomic ticket, so every tile a workgroup waits on is already
//            running: no dependence on dispatch order (cdna_hip_programming.md §6 G16).
//   phase 3  load-balanced expand + compaction (kernel 3): the workgroup's T pairs are written
//            as one contiguous, coalesced stream; output j finds its message by binary search in
//            the LDS offsets. Skewed fan-out (hot cubes) costs the same per pair as light cubes.
// Output: CSR offsets[M+1] (message-major), peers[P], optional msgs[P].
#include "wq_internal.hpp"

namespace wq {

constexpr int kRouteBlock = 256;
constexpr int kIPT = 4;  // messages per thread
constexpr int kTile = kRouteBlock * kIPT;

constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagPre = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;

struct RouteParams {
    const double* pos;
    const int64_t* keys;
    const uint32_t* world;
    const uint32_t* sender;
    const uint8_t* repl;
    uint32_t M;
    uint32_t n_tiles;
    const Slot* slots;
    uint64_t slot_mask;
    int slot_shift;
    uint64_t hash_mask;
    const uint32_t* list;
    uint32_t* offsets;
    uint32_t* peers;
    uint32_t* msgs;
    uint64_t capacity;
    uint64_t* ws;  // [0] P, [1] F, [2] overflow|error<<32, [3] tile ticket, [4..) status
    double sf;
    int64_t si;
};

__device__ __forceinline__ uint64_t ld_status(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

template <bool RAW_KEYS>
__global__ __launch_bounds__(kRouteBlock) void route_kernel(RouteParams p) {
    __shared__ uint32_t s_base[kTile];
    __shared__ uint32_t s_skip[kTile];
    __shared__ uint32_t s_off[kTile];
    __shared__ uint32_t s_wave[kRouteBlock / 64];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_prefix;
    __shared__ uint64_t s_F[kRouteBlock / 64];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    uint64_t* ws = p.ws;
    uint64_t* status = ws + 4;

    if (tid == 0) s_tile = atomicAdd(reinterpret_cast<uint32_t*>(ws + 3), 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t m0 = tile * kTile;

    // ---- phase 1: quantise, probe, filtered count ----
    uint64_t F_local = 0;
#pragma unroll
    for (int i = 0; i < kIPT; ++i) {
        const uint32_t j = i * kRouteBlock + tid;
        const uint32_t m = m0 + j;
        uint32_t e = 0, base = 0, skip = kNone;
        if (m < p.M) {
            const uint32_t w = p.world[m];
            int64_t x, y, z;
            if (RAW_KEYS) {
                x = p.keys[3ull * m];
                y = p.keys[3ull * m + 1];
                z = p.keys[3ull * m + 2];
            } else {
                x = coord_clamp_dev(p.pos[3ull * m], p.sf, p.si);
                y = coord_clamp_dev(p.pos[3ull * m + 1], p.sf, p.si);
                z = coord_clamp_dev(p.pos[3ull * m + 2], p.sf, p.si);
            }
            const uint64_t h = cube_hash(w, x, y, z) & p.hash_mask;
            const uint32_t off = probe(p.slots, p.slot_mask, p.slot_shift, h, w, x, y, z);
            if (off != kNone) {
                const uint32_t cnt = p.list[off];
                const uint32_t* peers = p.list + off + 1;
                F_local += cnt;
                const uint8_t r = p.repl[m];
                if (r == WQ_REPL_INCLUDING_SELF) {  // local_message.rs:70-75
                    e = cnt;
                    base = off + 1;
                } else {
                    const uint32_t me = p.sender[m];
                    const uint32_t at = lower_bound_dev(peers, cnt, me);
                    const bool has = at < cnt && peers[at] == me;
                    if (r == WQ_REPL_ONLY_SELF) {  // :77-85, the sender only if subscribed
                        e = has ? 1u : 0u;
                        base = off + 1 + at;
                    } else {  // ExceptSelf and unknown codes (replication.rs:40), :61-68
                        e = cnt - (has ? 1u : 0u);
                        base = off + 1;
                        skip = has ? at : kNone;
                    }
                }
            }
        }
        s_base[j] = base;
        s_skip[j] = skip;
        s_off[j] = e;
    }
    __syncthreads();

    // ---- phase 2: tile scan (thread t owns messages t*kIPT .. t*kIPT+kIPT-1) ----
    uint32_t c[kIPT];
    uint32_t tsum = 0;
#pragma unroll
    for (int k = 0; k < kIPT; ++k) {
        c[k] = s_off[tid * kIPT + k];
        tsum += c[k];
    }
    const uint32_t incl = wave_incl_scan(tsum, lane);
    if (lane == 63) s_wave[wave] = incl;
    const uint64_t Fw = wave_sum_u64(F_local);
    if (lane == 0) s_F[wave] = Fw;
    __syncthreads();
    uint32_t wbase = 0, T = 0;
#pragma unroll
    for (int w = 0; w < kRouteBlock / 64; ++w) {
        const uint32_t v = s_wave[w];
        if (w < wave) wbase += v;
        T += v;
    }
    uint32_t run = wbase + incl - tsum;
#pragma unroll
    for (int k = 0; k < kIPT; ++k) {
        s_off[tid * kIPT + k] = run;
        run += c[k];
    }

    // decoupled look-back (wave 0)
    if (wave == 0) {
        uint64_t excl = 0;
        if (tile == 0) {
            if (lane == 0) st_status(&status[0], kFlagPre | T);
        } else {
            if (lane == 0) st_status(&status[tile], kFlagAgg | T);
            int64_t q0 = (int64_t)tile - 1;
            uint32_t spins = 0;
            for (;;) {
                const int64_t q = q0 - lane;
                const uint64_t sv = (q >= 0) ? ld_status(&status[q]) : kFlagPre;
                const uint64_t fl = sv >> 62;
                const uint64_t pre = __ballot(fl == 2);
                const uint64_t zero = __ballot(fl == 0);
                const int first_pre = pre ? __builtin_ctzll(pre) : 64;
                const uint64_t need = (first_pre >= 63) ? ~0ull : ((2ull << first_pre) - 1);
                if ((zero & need) && spins < kSpinLimit) {
                    ++spins;
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                if (zero & need) {  // gave up: flag the error, count missing values as 0
                    if (lane == 0) atomicOr(reinterpret_cast<uint32_t*>(ws + 2) + 1, 1u);
                }
                const uint64_t v = (lane <= first_pre && fl != 0) ? (sv & kValMask) : 0;
                excl += wave_sum_u64(v);
                if (first_pre < 64) break;
                q0 -= 64;
            }
            if (lane == 0) st_status(&status[tile], kFlagPre | (excl + T));
        }
        if (lane == 0) {
            s_prefix = excl;
            uint64_t Fb = 0;
#pragma unroll
            for (int w = 0; w < kRouteBlock / 64; ++w) Fb += s_F[w];
            if (Fb) atomicAdd(reinterpret_cast<unsigned long long*>(ws + 1), (unsigned long long)Fb);
            if (tile == p.n_tiles - 1) {
                const uint64_t P = excl + T;
                ws[0] = P;
                p.offsets[p.M] = (uint32_t)P;
                if (P > p.capacity) atomicOr(reinterpret_cast<uint32_t*>(ws + 2), 1u);
            }
        }
    }
    __syncthreads();
    const uint64_t prefix = s_prefix;

#pragma unroll
    for (int i = 0; i < kIPT; ++i) {
        const uint32_t j = i * kRouteBlock + tid;
        const uint32_t m = m0 + j;
        if (m < p.M) p.offsets[m] = (uint32_t)(prefix + s_off[j]);
    }

    // ---- phase 3: load-balanced expand + compaction ----
    const uint32_t n_here = (p.M - m0) < (uint32_t)kTile ? (p.M - m0) : (uint32_t)kTile;
    for (uint32_t j = tid; j < T; j += kRouteBlock) {
        // last message k with s_off[k] <= j (it has e_k > 0)
        uint32_t lo = 0, hi = n_here;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_off[mid] <= j)
                lo = mid;
            else
                hi = mid;
        }
        const uint32_t r = j - s_off[lo];
        const uint32_t idx = s_base[lo] + r + (r >= s_skip[lo] ? 1u : 0u);
        const uint64_t out = prefix + j;
        if (out < p.capacity) {
            p.peers[out] = p.list[idx];
            if (p.msgs) p.msgs[out] = m0 + lo;
        }
    }
}

__global__ void quantize_kernel(const double* __restrict__ in, uint64_t n, double sf, int64_t si,
                                int64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = coord_clamp_dev(in[i], sf, si);
}

__global__ void is_subscribed_kernel(const uint32_t* __restrict__ world, const uint32_t* __restrict__ peer,
                                     int raw, const void* __restrict__ kp, uint32_t n, const Slot* slots,
                                     uint64_t mask, int shift, uint64_t hmask, const uint32_t* list,
                                     double sf, int64_t si, uint8_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int64_t x, y, z;
    if (raw) {
        const int64_t* k = static_cast<const int64_t*>(kp) + 3ull * i;
        x = k[0];
        y = k[1];
        z = k[2];
    } else {
        const double* q = static_cast<const double*>(kp) + 3ull * i;
        x = coord_clamp_dev(q[0], sf, si);
        y = coord_clamp_dev(q[1], sf, si);
        z = coord_clamp_dev(q[2], sf, si);
    }
    const uint32_t w = world[i];
    const uint32_t off = probe(slots, mask, shift, cube_hash(w, x, y, z) & hmask, w, x, y, z);
    uint8_t r = 0;
    if (off != kNone) {
        const uint32_t cnt = list[off];
        const uint32_t at = lower_bound_dev(list + off + 1, cnt, peer[i]);
        r = (at < cnt && list[off + 1 + at] == peer[i]) ? 1 : 0;
    }
    out[i] = r;
}

__global__ void is_subscribed_any_kernel(const uint32_t* __restrict__ world, const uint32_t* __restrict__ peer,
                                         uint32_t n, const uint64_t* any, uint64_t n_any, uint8_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = ((uint64_t)world[i] << 32) | peer[i];
    uint64_t lo = 0, hi = n_any;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (any[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    out[i] = (lo < n_any && any[lo] == key) ? 1 : 0;
}

// [lo, hi) of world w in the sorted any-keys (one thread).
__global__ void world_range_kernel(const uint64_t* any, uint64_t n_any, uint32_t w, uint64_t* out) {
    uint64_t a = 0, b = n_any;
    const uint64_t k0 = (uint64_t)w << 32;
    while (a < b) {
        const uint64_t mid = (a + b) >> 1;
        if (any[mid] < k0)
            a = mid + 1;
        else
            b = mid;
    }
    uint64_t c = a, d = n_any;
    const uint64_t k1 = k0 | 0xFFFFFFFFull;
    while (c < d) {
        const uint64_t mid = (c + d) >> 1;
        if (any[mid] <= k1)
            c = mid + 1;
        else
            d = mid;
    }
    out[0] = a;
    out[1] = c;
}

__global__ void low32_kernel(const uint64_t* in, uint64_t n, uint32_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = (uint32_t)in[i];
}

// ---- host launchers (used by wq_router.hip) ----

int launch_route(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                 const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                 uint32_t* d_peers, uint32_t* d_msgs, size_t capacity) {
    const uint32_t n_tiles = (uint32_t)((M + kTile - 1) / kTile);
    const size_t ws_bytes = (4 + (size_t)(n_tiles ? n_tiles : 1)) * 8;
    WQ_ALLOC(h, h->route_ws, ws_bytes);
    hipStream_t s = h->stream;
    WQ_HIP(h, hipMemsetAsync(h->route_ws.p, 0, ws_bytes, s));
    if (M == 0) {
        WQ_HIP(h, hipMemsetAsync(d_offsets, 0, 4, s));
        return WQ_OK;
    }
    RouteParams p;
    p.pos = d_pos;
    p.keys = d_keys;
    p.world = d_world;
    p.sender = d_sender;
    p.repl = d_repl;
    p.M = (uint32_t)M;
    p.n_tiles = n_tiles;
    p.slots = h->tab.slots.as<Slot>();
    p.slot_mask = h->tab.cap - 1;
    p.slot_shift = h->tab.shift;
    p.hash_mask = h->hash_mask;
    p.list = h->tab.list.as<uint32_t>();
    p.offsets = d_offsets;
    p.peers = d_peers;
    p.msgs = d_msgs;
    p.capacity = capacity;
    p.ws = h->route_ws.as<uint64_t>();
    p.sf = (double)h->cube_size;
    p.si = (int64_t)h->cube_size;

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
    if (d_keys)
        hipLaunchKernelGGL(route_kernel<true>, dim3(n_tiles), dim3(kRouteBlock), 0, s, p);
    else
        hipLaunchKernelGGL(route_kernel<false>, dim3(n_tiles), dim3(kRouteBlock), 0, s, p);
    WQ_HIP(h, hipGetLastError());
    if (pr.enabled) {
        WQ_HIP(h, hipEventRecord(pr.stop[pr.used], s));
        pr.used++;
    }
    return WQ_OK;
}

int launch_quantize(hipStream_t s, const double* d_in, size_t n, uint16_t cube_size, int64_t* d_out) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(quantize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_in, (uint64_t)n,
                       (double)cube_size, (int64_t)cube_size, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_is_subscribed(wq_router* h, const uint32_t* d_w, const uint32_t* d_p, int raw, const void* d_kp,
                         uint32_t n, uint8_t* d_out) {
    hipLaunchKernelGGL(is_subscribed_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, d_w, d_p, raw, d_kp, n,
                       h->tab.slots.as<Slot>(), h->tab.cap - 1, h->tab.shift, h->hash_mask,
                       h->tab.list.as<uint32_t>(), (double)h->cube_size, (int64_t)h->cube_size, d_out);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

int launch_is_subscribed_any(wq_router* h, const uint32_t* d_w, const uint32_t* d_p, uint32_t n, uint8_t* d_out) {
    hipLaunchKernelGGL(is_subscribed_any_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, d_w, d_p, n,
                       h->tab.any.as<uint64_t>(), h->tab.n_any, d_out);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

int launch_world_range(wq_router* h, uint32_t w, uint64_t* d_out) {
    hipLaunchKernelGGL(world_range_kernel, dim3(1), dim3(1), 0, h->stream, h->tab.any.as<uint64_t>(), h->tab.n_any,
                       w, d_out);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

int launch_low32(wq_router* h, const uint64_t* d_in, uint64_t n, uint32_t* d_out) {
    if (!n) return WQ_OK;
    hipLaunchKernelGGL(low32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, d_in, n, d_out);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

}  // namespace wq
