// wq_router.hip — the C ABI (include/wq_router.h): handle lifetime, host<->device staging,
// op-stream segmentation and dispatch to the kernels in wq_route.hip / wq_table.hip.
// Every compute call runs on the GPU; without a gfx950 device the calls fail with WQ_E_NODEV
// (there is no CPU fallback anywhere in this library).
#include <algorithm>
#include <cstring>
#include <vector>

#include "wq_internal.hpp"

namespace wq {
int launch_route(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                 const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t* d_offsets,
                 uint32_t* d_peers, uint32_t* d_msgs, size_t capacity);
int launch_quantize(hipStream_t s, const double* d_in, size_t n, uint16_t cube_size, int64_t* d_out);
int launch_is_subscribed(wq_router* h, const uint32_t* d_w, const uint32_t* d_p, int raw, const void* d_kp,
                         uint32_t n, uint8_t* d_out);
int launch_is_subscribed_any(wq_router* h, const uint32_t* d_w, const uint32_t* d_p, uint32_t n, uint8_t* d_out);
int launch_world_range(wq_router* h, uint32_t w, uint64_t* d_out);
int launch_low32(wq_router* h, const uint64_t* d_in, uint64_t n, uint32_t* d_out);
int launch_shard_messages(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                          const uint32_t* d_sender, const uint8_t* d_repl, size_t M, uint32_t G, wq_msg_rec* d_out,
                          uint32_t* d_counts);
int launch_op_owner(wq_router* h, const wq_op* d_ops, size_t n, uint32_t G, uint32_t* d_owner);
int launch_route_records(wq_router* h, const wq_msg_rec* d_recs, size_t M, uint32_t* d_offsets, uint32_t* d_peers,
                         uint32_t* d_msgs, size_t capacity);
int launch_peer_major(wq_router* h, const uint32_t* d_offsets, const uint32_t* d_peers, size_t M, size_t P,
                      const uint32_t* d_connected, uint32_t n_peers, uint32_t* d_peer_offsets, uint32_t* d_msgs_out);
int launch_route_global(wq_router* h, const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                        size_t M, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity);
}  // namespace wq

using namespace wq;

namespace {

constexpr size_t kAutoShapeMinMsgs = 256;  // one route block
thread_local std::string g_err;  // errors before a handle exists

int check_device(int device, std::string* why) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        *why = "no HIP device visible (this library has no CPU fallback)";
        return WQ_E_NODEV;
    }
    if (device < 0 || device >= n) {
        *why = "device index out of range";
        return WQ_E_INVALID;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        *why = "hipGetDeviceProperties failed";
        return WQ_E_NODEV;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        *why = std::string("device is ") + prop.gcnArchName + ", this build targets gfx950 only";
        return WQ_E_NODEV;
    }
    return WQ_OK;
}

// Host-staging helper: copies `bytes` from host into h->h_in at `offset` (aligned 256).
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Reads a host-form tick's CSR back (offsets at dout, peers at dout + op, msgs at dout + om).
int read_back(wq_router* h, size_t M, const char* dout, size_t op, size_t om, size_t cap, size_t capacity,
              uint32_t* offsets, uint32_t* peers, uint32_t* msgs, size_t* n_pairs) {
    hipStream_t s = h->stream;
    wq_route_counters cnt;
    WQ_HIP(h, hipMemcpyAsync(&cnt, h->rws.last, sizeof(cnt), hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));
    if (M == 0) cnt.n_pairs = 0;
    *n_pairs = cnt.n_pairs;
    if (cnt.error & 4u) return set_error(h, WQ_E_TIMEOUT, "route look-back spin gave up");
    if (cnt.n_pairs > 0xFFFFFFFFull || cnt.error) return set_error(h, WQ_E_CAPACITY, "more than 2^32-1 pairs in one tick");
    const size_t P = cnt.n_pairs;
    WQ_HIP(h, hipMemcpyAsync(offsets, dout, (M + 1) * 4, hipMemcpyDeviceToHost, s));
    const size_t ncopy = std::min(P, cap);
    if (ncopy) {
        WQ_HIP(h, hipMemcpyAsync(peers, dout + op, ncopy * 4, hipMemcpyDeviceToHost, s));
        if (msgs) WQ_HIP(h, hipMemcpyAsync(msgs, dout + om, ncopy * 4, hipMemcpyDeviceToHost, s));
    }
    WQ_HIP(h, hipStreamSynchronize(s));
    if (P > capacity) return set_error(h, WQ_E_CAPACITY, "output capacity too small (required size in *n_pairs)");
    return WQ_OK;
}

}  // namespace

extern "C" {

int wq_host_alloc(size_t bytes, void** out) {
    if (!out || bytes == 0) return WQ_E_INVALID;
    *out = nullptr;
    return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess ? WQ_OK : WQ_E_OOM;
}

int wq_host_free(void* p) {
    if (!p) return WQ_E_INVALID;
    return hipHostFree(p) == hipSuccess ? WQ_OK : WQ_E_HIP;
}

int wq_router_create(uint16_t cube_size, int device, wq_router** out) {
    if (!out || cube_size == 0) return WQ_E_INVALID;  // args.rs: cube_size is NonZeroU16
    *out = nullptr;
    int rc = check_device(device, &g_err);
    if (rc) return rc;
    if (hipSetDevice(device) != hipSuccess) return WQ_E_HIP;
    wq_router* h = new (std::nothrow) wq_router();
    if (!h) return WQ_E_OOM;
    h->device = device;
    h->cube_size = cube_size;
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return WQ_E_HIP;
    }
    h->stream = h->own_stream;
    rc = table_rebuild_derived(h);  // empty table: all slots empty
    if (rc) {
        g_err = h->err;
        wq_router_destroy(h);
        return rc;
    }
    *out = h;
    return WQ_OK;
}

int wq_router_destroy(wq_router* h) {
    if (!h) return WQ_E_INVALID;
    multi_release(h);
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    shard_release(h);
    for (auto* v : {&h->prof.start, &h->prof.stop, &h->prof.mid1, &h->prof.mid2})
        for (auto e : *v) (void)hipEventDestroy(e);
    DevBuf* bufs[] = {&h->st.h, &h->st.w, &h->st.kx, &h->st.ky, &h->st.kz, &h->st.p,
                      &h->st_next.h, &h->st_next.w, &h->st_next.kx, &h->st_next.ky, &h->st_next.kz,
                      &h->st_next.p, &h->tab.slots, &h->tab.claim, &h->tab.list, &h->tab.any,
                      &h->ev_h, &h->ev_w, &h->ev_kx, &h->ev_ky, &h->ev_kz, &h->ev_p, &h->ev_kind,
                      &h->d_ops, &h->idx_a, &h->idx_b, &h->key32_a, &h->key32_b, &h->key64_a,
                      &h->key64_b, &h->flags, &h->scan, &h->sort_tmp, &h->small, &h->cube_id,
                      &h->cube_start, &h->rws.buf, &h->rws.info, &h->rws.e, &h->rws.tiles,
                      &h->h_in, &h->h_out, &h->tab.recs, &h->tab.rclaim, &h->tab.pbox, &h->shard_hist,
                      &h->rec_keys, &h->rec_w, &h->rec_s, &h->rec_r, &h->ppos, &h->ppos4, &h->pcode, &h->qbox, &h->rws.agg, &h->rws.spill, &h->rws.scan_tmp,
                      &h->rws.carry, &h->tab.hdr, &h->dws.sort_cnt, &h->dws.sort_tot,
                      &h->dws.part, &h->dws.summ, &h->dws.dstat, &h->dws.rm_bits, &h->tab.stale};
    for (DevBuf* b : bufs) b->release();
    if (h->pend.ev) (void)hipEventDestroy(h->pend.ev);
    for (auto e : h->rws.cev) (void)hipEventDestroy(e);
    if (h->rws.ev_in) (void)hipEventDestroy(h->rws.ev_in);
    if (h->rws.side) (void)hipStreamDestroy(h->rws.side);
    if (h->pend.pinned) (void)hipHostFree(h->pend.pinned);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return WQ_OK;
}

const char* wq_last_error(const wq_router* h) { return h ? h->err.c_str() : g_err.c_str(); }

int wq_set_stream(wq_router* h, void* stream) {
    if (!h) return WQ_E_INVALID;
    h->stream = stream ? static_cast<hipStream_t>(stream) : h->own_stream;
    return WQ_OK;
}

int wq_get_stats(wq_router* h, wq_stats* out) {
    if (!h || !out) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    if (h->multi) return multi_stats(h, out);
    int rc = table_ensure_any(h);
    if (rc) return rc;
    if ((rc = table_sync_delta_stats(h))) return rc;
    out->n_entries = h->st.n;
    out->n_cubes = h->tab.n_cubes;
    out->n_any = h->tab.n_any;
    out->table_slots = h->tab.cap;
    out->hash_fallbacks = h->hash_fallbacks;
    out->cube_size = h->cube_size;
    out->device = h->device;
    return WQ_OK;
}

int wq_debug_route_config_count(void) { return route_config_count(); }

// The positions' bounding box (finite coordinates only) as order-preserving u64 keys: 6 words
// {min x, y, z, max x, y, z}; a few hundred blocks, one atomic per block and word.
__device__ __forceinline__ uint64_t ord_key(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __forceinline__ double ord_val(uint64_t k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & ~(1ull << 63)) : ~k));
}

// One pass over the positions (round 6: it was two, k_pos_f32 then k_pos_box): the radius filter's
// f32 copy (round to nearest, as the error bound in within_radius assumes; with copy64 the f64 rows
// too, device to device) and the bounding box of the finite coordinates as order-preserving u64 keys
// — 6 words {min x, y, z, max x, y, z} in `box`, reset by the previous call's k_pos_code (two box
// slots alternate); a few hundred blocks, one atomic per block and word.
static __global__ __launch_bounds__(256) void k_pos_f32_box(const double* __restrict__ pos, uint64_t n,
                                                            float4* __restrict__ out, double* __restrict__ copy64,
                                                            unsigned long long* __restrict__ box) {
    __shared__ uint64_t part[4][6];
    uint64_t lo[3] = {~0ull, ~0ull, ~0ull}, hi[3] = {0, 0, 0};
    constexpr int U = 4;  // positions per thread per round, all loads in flight first
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += U * stride) {
        double v[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * stride, j = i < n ? i : i0;  // (i0 < n)
            v[u][0] = pos[3 * j];
            v[u][1] = pos[3 * j + 1];
            v[u][2] = pos[3 * j + 2];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * stride;
            if (i >= n) continue;
            out[i] = make_float4((float)v[u][0], (float)v[u][1], (float)v[u][2], 0.0f);
            if (copy64) {
                copy64[3 * i] = v[u][0];
                copy64[3 * i + 1] = v[u][1];
                copy64[3 * i + 2] = v[u][2];
            }
            if (!(isfinite(v[u][0]) && isfinite(v[u][1]) && isfinite(v[u][2]))) continue;
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const uint64_t k = ord_key(v[u][d]);
                lo[d] = k < lo[d] ? k : lo[d];
                hi[d] = k > hi[d] ? k : hi[d];
            }
        }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint64_t a = __shfl_xor(lo[d], o, 64), b = __shfl_xor(hi[d], o, 64);
            lo[d] = a < lo[d] ? a : lo[d];
            hi[d] = b > hi[d] ? b : hi[d];
        }
    if ((threadIdx.x & 63) == 0)
        for (int d = 0; d < 3; ++d) {
            part[threadIdx.x >> 6][d] = lo[d];
            part[threadIdx.x >> 6][3 + d] = hi[d];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        uint64_t v = part[0][threadIdx.x];
        for (int w = 1; w < 4; ++w) {
            const uint64_t x = part[w][threadIdx.x];
            v = threadIdx.x < 3 ? (x < v ? x : v) : (x > v ? x : v);
        }
        if (threadIdx.x < 3) atomicMin(box + threadIdx.x, (unsigned long long)v);
        else atomicMax(box + threadIdx.x, (unsigned long long)v);
    }
}

// The box -> {lo, step} (kept at box + 6 as doubles for the count pass) and every peer's code.
static __global__ __launch_bounds__(256) void k_pos_code(const double* __restrict__ pos, uint64_t n,
                                                         const unsigned long long* __restrict__ box,
                                                         double* __restrict__ dec, unsigned long long* __restrict__ next,
                                                         uint32_t* __restrict__ code) {
    double qb[6];
    bool any = true;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const uint64_t klo = box[d], khi = box[3 + d];
        any = any && klo <= khi;  // no finite position at all: klo = ~0, khi = 0
        const double lo = ord_val(klo), hi = ord_val(khi);
        const double steps = d < 2 ? (double)kQMaxXY : (double)kQMaxZ;
        qb[d] = lo;
        qb[3 + d] = hi > lo ? (hi - lo) / steps : 1.0;
    }
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) dec[k] = qb[k];
    }
    if (i < 6) next[i] = i < 3 ? ~0ull : 0ull;  // the other box slot, for the next call
    if (i >= n) return;
    const double x = pos[3 * i], y = pos[3 * i + 1], z = pos[3 * i + 2];
    uint32_t c = any ? pos_code(x, y, z, qb) : kQNone;
    if (c != kQNone) {  // belt and braces: a code must decode within half a step (+ rounding)
        const uint32_t u[3] = {c & kQMaxXY, (c >> 11) & kQMaxXY, c >> 22};
        const double v[3] = {x, y, z};
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const double q = qb[d] + (double)u[d] * qb[3 + d];
            if (!(fabs(v[d] - q) <= qb[3 + d] * 0.5 * (1.0 + 0x1p-40) + (fabs(qb[d]) + fabs(q) + (double)u[d] * qb[3 + d]) * 0x1p-49))
                c = kQNone;
        }
    }
    code[i] = c;
}

static int set_peer_positions(wq_router* h, const double* pos, size_t n, hipMemcpyKind kind) {
    if (!h || (n && !pos) || n > 0xFFFFFFFFull) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    if (h->multi) return multi_set_positions(h, pos, n, kind == hipMemcpyDeviceToDevice);
    WQ_ALLOC(h, h->ppos, (n ? n : 1) * 24);
    WQ_ALLOC(h, h->ppos4, (n ? n : 1) * 16);
    const bool d2d = kind == hipMemcpyDeviceToDevice;
    if (n && !d2d) WQ_HIP(h, hipMemcpyAsync(h->ppos.p, pos, n * 24, kind, h->stream));
    WQ_ALLOC(h, h->pcode, (n ? n : 1) * 4);
    // qbox: u64 box slot A [0, 6), the decoded {lo, step} doubles [6, 12) (TableView::qbox), slot B
    // [12, 18); the slots alternate between calls, each call's k_pos_code resetting the other one
    if (!h->qbox.p) h->qbox_phase = -1;
    WQ_ALLOC(h, h->qbox, 192);
    if (n) {
        unsigned long long* q = h->qbox.as<unsigned long long>();
        if (h->qbox_phase < 0) {  // first use: both slots reset (one memset pair, once per handle)
            WQ_HIP(h, hipMemsetAsync(q, 0xFF, 24, h->stream));
            WQ_HIP(h, hipMemsetAsync(q + 3, 0, 24, h->stream));
            WQ_HIP(h, hipMemsetAsync(q + 12, 0xFF, 24, h->stream));
            WQ_HIP(h, hipMemsetAsync(q + 15, 0, 24, h->stream));
            h->qbox_phase = 0;
        }
        unsigned long long* cur = q + (h->qbox_phase ? 12 : 0);
        unsigned long long* nxt = q + (h->qbox_phase ? 0 : 12);
        const unsigned gb = (unsigned)std::min<size_t>(256, (n + 255) / 256);
        hipLaunchKernelGGL(k_pos_f32_box, dim3(gb), dim3(256), 0, h->stream, d2d ? pos : h->ppos.as<double>(),
                           (uint64_t)n, h->ppos4.as<float4>(), d2d ? h->ppos.as<double>() : nullptr, cur);
        WQ_HIP(h, hipGetLastError());
        hipLaunchKernelGGL(k_pos_code, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream,
                           h->ppos.as<double>(), (uint64_t)n, cur, reinterpret_cast<double*>(q + 6), nxt,
                           h->pcode.as<uint32_t>());
        WQ_HIP(h, hipGetLastError());
        h->qbox_phase ^= 1;
    }
    if (kind == hipMemcpyHostToDevice) WQ_HIP(h, hipStreamSynchronize(h->stream));
    h->n_ppos = n;
    return WQ_OK;
}

int wq_set_peer_positions(wq_router* h, const double* pos, size_t n_peers) {
    return set_peer_positions(h, pos, n_peers, hipMemcpyHostToDevice);
}

int wq_set_peer_positions_device(wq_router* h, const double* d_pos, size_t n_peers) {
    return set_peer_positions(h, d_pos, n_peers, hipMemcpyDeviceToDevice);
}

int wq_set_radius(wq_router* h, double radius) {
    if (!h) return WQ_E_INVALID;
    h->radius = (radius > 0.0) ? radius : 0.0;  // NaN compares false: off
    if (h->multi) return multi_set_radius(h, radius);
    return WQ_OK;
}

int wq_set_fanout_hint(wq_router* h, double pairs_per_message) {
    if (!h) return WQ_E_INVALID;
    if (h->multi) return multi_set_hint(h, pairs_per_message);
    if (!(pairs_per_message >= 0.0)) {  // negative or NaN: back to the automatic choice
        h->fanout_auto = true;
        return WQ_OK;
    }
    h->heavy_fanout = pairs_per_message >= WQ_HEAVY_FANOUT;
    h->fanout_auto = false;  // the caller decides from now on
    return WQ_OK;
}

int wq_debug_route_shape(wq_router* h, int* heavy_fanout, int* fanout_auto) {
    if (!h || !heavy_fanout || !fanout_auto) return WQ_E_INVALID;
    *heavy_fanout = h->heavy_fanout ? 1 : 0;
    *fanout_auto = h->fanout_auto ? 1 : 0;
    return WQ_OK;
}

int wq_route_health(wq_router* h, uint32_t* error_bits, uint32_t* overflow) {
    if (!h || !error_bits || !overflow) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    *error_bits = 0;
    *overflow = 0;
    if (h->multi) {
        if (int rc = multi_health(h, error_bits, overflow)) return rc;
    }
    if (!h->rws.buf.p) return WQ_OK;  // no route call yet (the multi handle's own: global routes)
    uint32_t w[2];
    WQ_HIP(h, hipMemcpyAsync(w, h->rws.buf.p, 8, hipMemcpyDeviceToHost, h->stream));
    WQ_HIP(h, hipMemsetAsync(h->rws.buf.p, 0, 8, h->stream));
    WQ_HIP(h, hipStreamSynchronize(h->stream));
    // OR, not assign: a multi handle's shard bits are already in (and cleared on the shards)
    *error_bits |= w[0];
    *overflow |= w[1];
    return WQ_OK;
}

int wq_debug_set_route_config(wq_router* h, int cfg) {
    if (!h || cfg < 0 || cfg >= route_config_count()) return WQ_E_INVALID;
    h->route_cfg = cfg;
    return WQ_OK;
}

int wq_debug_set_route_chunks(wq_router* h, int chunks) {
    if (!h || chunks < 0 || chunks > 64) return WQ_E_INVALID;
    h->route_chunks = (uint32_t)chunks;
    return WQ_OK;
}

int wq_debug_update_counts(wq_router* h, uint64_t* incremental, uint64_t* rebuild_fallbacks,
                           uint64_t* wave_batches) {
    if (!h || !incremental || !rebuild_fallbacks || !wave_batches) return WQ_E_INVALID;
    if (int rc = table_resolve(h, true)) return rc;
    *incremental = h->n_delta_applies;
    *rebuild_fallbacks = h->n_delta_fallbacks;
    *wave_batches = h->n_delta_wave_batches;
    return WQ_OK;
}

int wq_debug_set_timeline(wq_router* h, uint64_t* d_stamps) {
    if (!h) return WQ_E_INVALID;
    h->rws.stamps = d_stamps;
    return WQ_OK;
}

int wq_debug_set_record_slack(wq_router* h, uint32_t slots_per_cube) {
    if (!h || slots_per_cube < 2 || slots_per_cube > 1024) return WQ_E_INVALID;
    h->rec_slack = slots_per_cube;  // takes effect at the next rebuild
    h->rec_slack_set = true;        // ... exactly (no footprint cap, wq_table.hip)
    return WQ_OK;
}

int wq_debug_set_hash_bits(wq_router* h, int bits) {
    if (!h || bits < 1 || bits > 64) return WQ_E_INVALID;
    if (h->st.n) return set_error(h, WQ_E_INVALID, "hash bits can only change on an empty table");
    h->hash_mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
    return WQ_OK;
}

int wq_apply_ops(wq_router* h, const wq_op* ops, size_t n) {
    if (!h || (n && !ops)) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    for (size_t i = 0; i < n; ++i)
        if (ops[i].kind > WQ_OP_REMOVE_PEER ||
            (ops[i].kind != WQ_OP_REMOVE_PEER && ops[i].world == WQ_WORLD_INVALID))
            return set_error(h, WQ_E_INVALID, "bad op (kind or reserved world id)");
    if (h->multi) return multi_apply_ops(h, ops, n);
    // Split at REMOVE_PEER runs so the reference's sequential order is kept (thread.rs:122-146).
    size_t i = 0;
    std::vector<uint64_t> rm;
    while (i < n) {
        size_t j = i;
        if (ops[i].kind != WQ_OP_REMOVE_PEER) {
            while (j < n && ops[j].kind != WQ_OP_REMOVE_PEER) ++j;
            int rc = table_apply_segment(h, ops + i, j - i);
            if (rc) return rc;
        } else {
            rm.clear();
            for (; j < n && ops[j].kind == WQ_OP_REMOVE_PEER; ++j)
                rm.push_back(((uint64_t)ops[j].world << 32) | ops[j].peer);
            std::sort(rm.begin(), rm.end());
            rm.erase(std::unique(rm.begin(), rm.end()), rm.end());
            int rc = table_remove_peers(h, rm.data(), rm.size());
            if (rc) return rc;
        }
        i = j;
    }
    return WQ_OK;
}

int wq_apply_ops_device(wq_router* h, const wq_op* d_ops, size_t n) {
    if (!h || (n && !d_ops)) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    if (h->multi) return multi_apply_ops_device(h, d_ops, n);
    return table_apply_segment(h, d_ops, n, true);
}

int wq_remove_peers(wq_router* h, const uint32_t* peers, size_t n) {
    if (!h || (n && !peers)) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    if (h->multi) return multi_remove_peers(h, peers, n);
    std::vector<uint64_t> rm(n);
    for (size_t i = 0; i < n; ++i) rm[i] = ((uint64_t)WQ_WORLD_INVALID << 32) | peers[i];
    std::sort(rm.begin(), rm.end());
    rm.erase(std::unique(rm.begin(), rm.end()), rm.end());
    return table_remove_peers(h, rm.data(), rm.size());
}

int wq_route_tick_device(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                         const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs, uint32_t* d_offsets,
                         uint32_t* d_peers, uint32_t* d_msgs, size_t capacity, wq_route_counters* d_counters) {
    if (!h || !d_offsets || (n_msgs && (!d_world || !d_sender || !d_repl || (!d_pos && !d_keys))) ||
        (capacity && !d_peers))
        return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    if (capacity > 0xFFFFFFFFull) capacity = 0xFFFFFFFFull;  // u32 CSR offsets
    WQ_HIP(h, hipSetDevice(h->device));
    if (h->multi) {
        size_t P = 0;
        const int rc = multi_route_tick(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, d_offsets, d_peers, d_msgs,
                                        capacity, &P, true);
        if ((rc == WQ_OK || rc == WQ_E_CAPACITY) && d_counters) {  // P (F reported as P), overflow
            wq_route_counters c{P, P, P > capacity ? 1u : 0u, 0u};
            WQ_HIP(h, hipMemcpyAsync(d_counters, &c, sizeof(c), hipMemcpyHostToDevice, h->stream));
            WQ_HIP(h, hipStreamSynchronize(h->stream));
        }
        return rc == WQ_E_CAPACITY ? WQ_OK : rc;  // as the single-GPU form: the counters report overflow
    }
    // the three-launch shape's scan writes d_counters itself once they are final (no copy launch)
    h->rws.out = d_counters;
    h->rws.out_done = false;
    int rc = launch_route(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, d_offsets, d_peers, d_msgs, capacity);
    h->rws.out = nullptr;
    if (rc) return rc;
    if (d_counters && !h->rws.out_done)
        WQ_HIP(h, hipMemcpyAsync(d_counters, h->rws.last, sizeof(wq_route_counters), hipMemcpyDeviceToDevice,
                                 h->stream));
    return WQ_OK;
}

int wq_route_tick(wq_router* h, const double* pos, const int64_t* keys, const uint32_t* world,
                  const uint32_t* sender, const uint8_t* repl, size_t M, uint32_t* offsets, uint32_t* peers,
                  uint32_t* msgs, size_t capacity, size_t* n_pairs) {
    if (!h || !offsets || !n_pairs || (M && (!world || !sender || !repl || (!pos && !keys))) ||
        (capacity && !peers))
        return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    if (h->multi) {
        if (M >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
        return multi_route_tick(h, pos, keys, world, sender, repl, M, offsets, peers, msgs,
                                std::min<size_t>(capacity, 0xFFFFFFFFull), n_pairs, false);
    }
    const size_t b_pos = keys ? M * 24 : (pos ? M * 24 : 0);
    const size_t o_pos = 0, o_w = align256(o_pos + b_pos), o_s = align256(o_w + M * 4),
                 o_r = align256(o_s + M * 4), n_in = align256(o_r + M + 1);
    WQ_ALLOC(h, h->h_in, n_in);
    char* din = h->h_in.as<char>();
    hipStream_t s = h->stream;
    if (M) {
        WQ_HIP(h, hipMemcpyAsync(din + o_pos, keys ? (const void*)keys : (const void*)pos, b_pos,
                                 hipMemcpyHostToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(din + o_w, world, M * 4, hipMemcpyHostToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(din + o_s, sender, M * 4, hipMemcpyHostToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(din + o_r, repl, M, hipMemcpyHostToDevice, s));
    }
    const size_t cap = std::min<size_t>(capacity, 0xFFFFFFFFull);
    const size_t oo = 0, op = align256((M + 1) * 4), om = align256(op + cap * 4), n_out = align256(om + (msgs ? cap * 4 : 0));
    WQ_ALLOC(h, h->h_out, n_out + 256);
    char* dout = h->h_out.as<char>();
    int rc = launch_route(h, keys ? nullptr : reinterpret_cast<const double*>(din + o_pos),
                          keys ? reinterpret_cast<const int64_t*>(din + o_pos) : nullptr,
                          reinterpret_cast<const uint32_t*>(din + o_w), reinterpret_cast<const uint32_t*>(din + o_s),
                          reinterpret_cast<const uint8_t*>(din + o_r), M, reinterpret_cast<uint32_t*>(dout + oo),
                          cap ? reinterpret_cast<uint32_t*>(dout + op) : nullptr,
                          (msgs && cap) ? reinterpret_cast<uint32_t*>(dout + om) : nullptr, cap);
    if (rc) return rc;
    rc = read_back(h, M, dout, op, om, cap, capacity, offsets, peers, msgs, n_pairs);
    // the next tick's shape, from ticks of at least one block of messages (a single-message query
    // such as AreaMap::get_subscribed_peers says nothing about a tick's fan-out)
    if ((rc == WQ_OK || rc == WQ_E_CAPACITY) && h->fanout_auto && M >= kAutoShapeMinMsgs)
        h->heavy_fanout = (double)*n_pairs >= WQ_HEAVY_FANOUT * (double)M;
    return rc;
}

int wq_route_global_device(wq_router* h, const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                           size_t n_msgs, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity,
                           wq_route_counters* d_counters) {
    if (!h || !d_offsets || (n_msgs && (!d_world || !d_sender || !d_repl)) || (capacity && !d_peers))
        return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    if (capacity > 0xFFFFFFFFull) capacity = 0xFFFFFFFFull;
    WQ_HIP(h, hipSetDevice(h->device));
    int rc = h->multi ? multi_merge_any(h) : table_ensure_any(h);
    if (rc) return rc;
    rc = launch_route_global(h, d_world, d_sender, d_repl, n_msgs, d_offsets, d_peers, d_msgs, capacity);
    if (rc) return rc;
    if (d_counters)
        WQ_HIP(h, hipMemcpyAsync(d_counters, h->rws.last, sizeof(wq_route_counters), hipMemcpyDeviceToDevice,
                                 h->stream));
    return WQ_OK;
}

int wq_route_global(wq_router* h, const uint32_t* world, const uint32_t* sender, const uint8_t* repl, size_t M,
                    uint32_t* offsets, uint32_t* peers, uint32_t* msgs, size_t capacity, size_t* n_pairs) {
    if (!h || !offsets || !n_pairs || (M && (!world || !sender || !repl)) || (capacity && !peers))
        return WQ_E_INVALID;
    if (M >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    for (size_t i = 0; i < M; ++i)
        if (world[i] == WQ_WORLD_INVALID) return set_error(h, WQ_E_INVALID, "reserved world id in a GlobalMessage");
    WQ_HIP(h, hipSetDevice(h->device));
    int rc0 = h->multi ? multi_merge_any(h) : table_ensure_any(h);
    if (rc0) return rc0;
    const size_t o_w = 0, o_s = align256(M * 4), o_r = align256(o_s + M * 4), n_in = align256(o_r + M + 1);
    WQ_ALLOC(h, h->h_in, n_in);
    char* din = h->h_in.as<char>();
    hipStream_t s = h->stream;
    if (M) {
        WQ_HIP(h, hipMemcpyAsync(din + o_w, world, M * 4, hipMemcpyHostToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(din + o_s, sender, M * 4, hipMemcpyHostToDevice, s));
        WQ_HIP(h, hipMemcpyAsync(din + o_r, repl, M, hipMemcpyHostToDevice, s));
    }
    const size_t cap = std::min<size_t>(capacity, 0xFFFFFFFFull);
    const size_t op = align256((M + 1) * 4), om = align256(op + cap * 4), n_out = align256(om + (msgs ? cap * 4 : 0));
    WQ_ALLOC(h, h->h_out, n_out + 256);
    char* dout = h->h_out.as<char>();
    int rc = launch_route_global(h, reinterpret_cast<const uint32_t*>(din + o_w),
                                 reinterpret_cast<const uint32_t*>(din + o_s),
                                 reinterpret_cast<const uint8_t*>(din + o_r), M, reinterpret_cast<uint32_t*>(dout),
                                 cap ? reinterpret_cast<uint32_t*>(dout + op) : nullptr,
                                 (msgs && cap) ? reinterpret_cast<uint32_t*>(dout + om) : nullptr, cap);
    if (rc) return rc;
    return read_back(h, M, dout, op, om, cap, capacity, offsets, peers, msgs, n_pairs);
}

int wq_shard_ops(wq_router* h, const wq_op* ops, size_t n, uint32_t n_shards, uint32_t* owner) {
    if (!h || (n && (!ops || !owner)) || n_shards == 0 || n_shards > WQ_MAX_SHARDS) return WQ_E_INVALID;
    if (n == 0) return WQ_OK;
    if (n >= 0xFFFFFFFFull) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    const size_t o_o = align256(n * sizeof(wq_op));
    WQ_ALLOC(h, h->h_in, o_o + n * 4);
    char* d = h->h_in.as<char>();
    hipStream_t s = h->stream;
    WQ_HIP(h, hipMemcpyAsync(d, ops, n * sizeof(wq_op), hipMemcpyHostToDevice, s));
    int rc = launch_op_owner(h, reinterpret_cast<const wq_op*>(d), n, n_shards, reinterpret_cast<uint32_t*>(d + o_o));
    if (rc) return rc;
    WQ_HIP(h, hipMemcpyAsync(owner, d + o_o, n * 4, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));
    return WQ_OK;
}

int wq_shard_messages_device(wq_router* h, const double* d_pos, const int64_t* d_keys, const uint32_t* d_world,
                             const uint32_t* d_sender, const uint8_t* d_repl, size_t n_msgs, uint32_t n_shards,
                             wq_msg_rec* d_out, uint32_t* d_counts) {
    if (!h || !d_counts || n_shards == 0 || n_shards > WQ_MAX_SHARDS ||
        (n_msgs && (!d_world || !d_sender || !d_repl || (!d_pos && !d_keys) || !d_out)))
        return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    WQ_HIP(h, hipSetDevice(h->device));
    return launch_shard_messages(h, d_pos, d_keys, d_world, d_sender, d_repl, n_msgs, n_shards, d_out, d_counts);
}

int wq_route_records_device(wq_router* h, const wq_msg_rec* d_recs, size_t n_msgs, uint32_t* d_offsets,
                            uint32_t* d_peers, uint32_t* d_msgs, size_t capacity, wq_route_counters* d_counters) {
    if (!h || !d_offsets || (n_msgs && !d_recs) || (capacity && !d_peers)) return WQ_E_INVALID;
    if (n_msgs >= 0xFFFFFC00ull) return set_error(h, WQ_E_INVALID, "n_msgs must be < 2^32 - 1024 per tick");
    if (capacity > 0xFFFFFFFFull) capacity = 0xFFFFFFFFull;
    WQ_HIP(h, hipSetDevice(h->device));
    int rc = launch_route_records(h, d_recs, n_msgs, d_offsets, d_peers, d_msgs, capacity);
    if (rc) return rc;
    if (d_counters)
        WQ_HIP(h, hipMemcpyAsync(d_counters, h->rws.last, sizeof(wq_route_counters), hipMemcpyDeviceToDevice,
                                 h->stream));
    return WQ_OK;
}

int wq_peer_major_device(wq_router* h, const uint32_t* d_offsets, const uint32_t* d_peers, size_t n_msgs,
                         size_t n_pairs, const uint32_t* d_connected, uint32_t n_peers, uint32_t* d_peer_offsets,
                         uint32_t* d_msgs_out) {
    if (!h || !d_peer_offsets || (n_msgs && !d_offsets) || (n_pairs && (!d_peers || !d_msgs_out)) ||
        n_peers == 0xFFFFFFFFu || n_pairs > 0xFFFFFFFFull || n_msgs >= 0xFFFFFFFFull)
        return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    return launch_peer_major(h, d_offsets, d_peers, n_msgs, n_pairs, d_connected, n_peers, d_peer_offsets,
                             d_msgs_out);
}

int wq_is_subscribed(wq_router* h, size_t n, const uint32_t* world, const uint32_t* peer, int key_is_raw,
                     const void* key_or_pos, uint8_t* out) {
    if (!h || (n && (!world || !peer || !key_or_pos || !out))) return WQ_E_INVALID;
    if (n == 0) return WQ_OK;
    if (n >= 0xFFFFFFFFull) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    if (h->multi) return multi_is_subscribed(h, n, world, peer, key_is_raw, key_or_pos, out);
    if (int rc0 = table_resolve(h, true)) return rc0;
    const size_t o_w = 0, o_p = align256(n * 4), o_k = align256(o_p + n * 4), o_o = align256(o_k + n * 24);
    WQ_ALLOC(h, h->h_in, o_o + n);
    char* d = h->h_in.as<char>();
    hipStream_t s = h->stream;
    WQ_HIP(h, hipMemcpyAsync(d + o_w, world, n * 4, hipMemcpyHostToDevice, s));
    WQ_HIP(h, hipMemcpyAsync(d + o_p, peer, n * 4, hipMemcpyHostToDevice, s));
    WQ_HIP(h, hipMemcpyAsync(d + o_k, key_or_pos, n * 24, hipMemcpyHostToDevice, s));
    int rc = launch_is_subscribed(h, reinterpret_cast<uint32_t*>(d + o_w), reinterpret_cast<uint32_t*>(d + o_p),
                                  key_is_raw ? 1 : 0, d + o_k, (uint32_t)n, reinterpret_cast<uint8_t*>(d + o_o));
    if (rc) return rc;
    WQ_HIP(h, hipMemcpyAsync(out, d + o_o, n, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));
    return WQ_OK;
}

int wq_is_subscribed_any(wq_router* h, size_t n, const uint32_t* world, const uint32_t* peer, uint8_t* out) {
    if (!h || (n && (!world || !peer || !out))) return WQ_E_INVALID;
    if (n == 0) return WQ_OK;
    if (n >= 0xFFFFFFFFull) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    int rc0 = h->multi ? multi_merge_any(h) : table_ensure_any(h);
    if (rc0) return rc0;
    const size_t o_w = 0, o_p = align256(n * 4), o_o = align256(o_p + n * 4);
    WQ_ALLOC(h, h->h_in, o_o + n);
    char* d = h->h_in.as<char>();
    hipStream_t s = h->stream;
    WQ_HIP(h, hipMemcpyAsync(d + o_w, world, n * 4, hipMemcpyHostToDevice, s));
    WQ_HIP(h, hipMemcpyAsync(d + o_p, peer, n * 4, hipMemcpyHostToDevice, s));
    int rc = launch_is_subscribed_any(h, reinterpret_cast<uint32_t*>(d + o_w), reinterpret_cast<uint32_t*>(d + o_p),
                                      (uint32_t)n, reinterpret_cast<uint8_t*>(d + o_o));
    if (rc) return rc;
    WQ_HIP(h, hipMemcpyAsync(out, d + o_o, n, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));
    return WQ_OK;
}

int wq_world_peers(wq_router* h, uint32_t world, uint32_t* out, size_t capacity, size_t* n_out) {
    if (!h || !n_out || (capacity && !out)) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    int rc0 = h->multi ? multi_merge_any(h) : table_ensure_any(h);
    if (rc0) return rc0;
    WQ_ALLOC(h, h->small, 64);
    hipStream_t s = h->stream;
    int rc = launch_world_range(h, world, h->small.as<uint64_t>());
    if (rc) return rc;
    uint64_t range[2];
    WQ_HIP(h, hipMemcpyAsync(range, h->small.p, 16, hipMemcpyDeviceToHost, s));
    WQ_HIP(h, hipStreamSynchronize(s));
    const uint64_t n = range[1] - range[0];
    *n_out = n;
    const uint64_t nc = std::min<uint64_t>(n, capacity);
    if (nc) {
        WQ_ALLOC(h, h->h_out, nc * 4);
        rc = launch_low32(h, h->tab.any.as<uint64_t>() + range[0], nc, h->h_out.as<uint32_t>());
        if (rc) return rc;
        WQ_HIP(h, hipMemcpyAsync(out, h->h_out.p, nc * 4, hipMemcpyDeviceToHost, s));
        WQ_HIP(h, hipStreamSynchronize(s));
    }
    if (n > capacity) return set_error(h, WQ_E_CAPACITY, "world_peers capacity too small");
    return WQ_OK;
}

int wq_quantize(const double* coords, size_t n, uint16_t cube_size, int64_t* out) {
    if (cube_size == 0 || (n && (!coords || !out))) return WQ_E_INVALID;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int rc = check_device(dev, &g_err);
    if (rc) return rc;
    if (n == 0) return WQ_OK;
    void *din = nullptr, *dout = nullptr;
    if (hipMalloc(&din, n * 8) != hipSuccess) return WQ_E_OOM;
    if (hipMalloc(&dout, n * 8) != hipSuccess) {
        (void)hipFree(din);
        return WQ_E_OOM;
    }
    int status = WQ_OK;
    if (hipMemcpy(din, coords, n * 8, hipMemcpyHostToDevice) != hipSuccess ||
        launch_quantize(nullptr, static_cast<const double*>(din), n, cube_size, static_cast<int64_t*>(dout)) != 0 ||
        hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost) != hipSuccess)
        status = WQ_E_HIP;
    (void)hipFree(din);
    (void)hipFree(dout);
    return status;
}

int wq_quantize_device(wq_router* h, const double* d_coords, size_t n, int64_t* d_out) {
    if (!h || (n && (!d_coords || !d_out))) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    if (launch_quantize(h->stream, d_coords, n, h->cube_size, d_out) != 0)
        return set_error(h, WQ_E_HIP, "quantize launch failed");
    return WQ_OK;
}

int wq_profile_enable(wq_router* h, int enable) {
    if (!h) return WQ_E_INVALID;
    h->prof.enabled = enable != 0;
    h->prof.used = 0;
    return WQ_OK;
}

int wq_profile_read(wq_router* h, double* kernel_ms, uint64_t* launches) {
    if (!h || !kernel_ms || !launches) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    double total = 0.0;
    for (size_t i = 0; i < h->prof.used; ++i) {
        WQ_HIP(h, hipEventSynchronize(h->prof.stop[i]));
        float ms = 0.0f;
        WQ_HIP(h, hipEventElapsedTime(&ms, h->prof.start[i], h->prof.stop[i]));
        total += ms;
    }
    *kernel_ms = total;
    *launches = h->prof.used;
    h->prof.used = 0;
    return WQ_OK;
}

int wq_profile_read_phases(wq_router* h, double* kernel_ms, uint64_t* launches, double* phase_ms,
                           uint64_t* phased) {
    if (!h || !kernel_ms || !launches || !phase_ms || !phased) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    ProfileEvents& pr = h->prof;
    double ph[3] = {0.0, 0.0, 0.0};
    uint64_t np = 0;
    for (size_t i = 0; i < pr.used; ++i) {
        if (!pr.phased[i]) continue;
        WQ_HIP(h, hipEventSynchronize(pr.stop[i]));
        const hipEvent_t ev[4] = {pr.start[i], pr.mid1[i], pr.mid2[i], pr.stop[i]};
        for (int k = 0; k < 3; ++k) {
            float ms = 0.0f;
            WQ_HIP(h, hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
            ph[k] += ms;
        }
        ++np;
    }
    for (int k = 0; k < 3; ++k) phase_ms[k] = ph[k];
    *phased = np;
    return wq_profile_read(h, kernel_ms, launches);
}

// The shader clock the GPU runs at right now: every workgroup spins on dependent VALU work between
// two reads of the shader-clock counter (s_memtime) and of the constant-rate wall clock
// (s_memrealtime, hipDeviceAttributeWallClockRate); cycles / wall time per workgroup, median.
static __global__ __launch_bounds__(256) void k_sclk_probe(uint64_t* out, uint32_t iters) {
    const uint64_t c0 = clock64(), w0 = wall_clock64();
    float x = (float)threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i) x = __builtin_fmaf(x, 0.9999999f, 1e-7f);
    const uint64_t c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = c1 - c0;
        out[2 * blockIdx.x + 1] = w1 - w0;
    }
    if (x == -1.0f) out[0] = 0;  // keeps the loop
}

int wq_probe_sclk(wq_router* h, double* mhz) {
    if (!h || !mhz) return WQ_E_INVALID;
    WQ_HIP(h, hipSetDevice(h->device));
    int rate_khz = 0;
    WQ_HIP(h, hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, h->device));
    if (rate_khz <= 0) return set_error(h, WQ_E_HIP, "no wall clock rate");
    constexpr unsigned kBlocks = 1024;
    uint64_t* d = nullptr;
    WQ_HIP(h, hipMalloc(&d, kBlocks * 16));
    hipLaunchKernelGGL(k_sclk_probe, dim3(kBlocks), dim3(256), 0, h->stream, d, 200000u);
    std::vector<uint64_t> v(2 * kBlocks);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(v.data(), d, kBlocks * 16, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return set_error(h, WQ_E_HIP, "sclk probe", e);
    std::vector<double> f;
    for (unsigned b = 0; b < kBlocks; ++b)
        if (v[2 * b + 1]) f.push_back((double)v[2 * b] / (double)v[2 * b + 1] * rate_khz / 1e3);
    if (f.empty()) return set_error(h, WQ_E_HIP, "sclk probe: no wall-clock ticks");
    std::nth_element(f.begin(), f.begin() + f.size() / 2, f.end());
    *mhz = f[f.size() / 2];
    return WQ_OK;
}

}  // extern "C"
