// wq_query.hip — kernel (1) on its own (CubeArea::coord_clamp over a coordinate array,
// worldql_server/src/subscriptions/cube_area.rs:23-44) and the table queries the reference
// exposes for its unit tests: AreaMap::is_peer_subscribed / is_peer_subscribed_any /
// get_subscribed_any_peers (worldql_server/src/subscriptions/area_map.rs:33-67).
#include "wq_internal.hpp"

namespace wq {

__global__ void quantize_kernel(const double* __restrict__ in, uint64_t n, double sf, int64_t si,
                                int64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = coord_clamp_dev(in[i], sf, si);
}

__global__ void is_subscribed_kernel(const uint32_t* __restrict__ world, const uint32_t* __restrict__ peer,
                                     int raw, const void* __restrict__ kp, uint32_t n, TableView t,
                                     int64_t si, uint8_t* out) {
    const double sf = t.sf;
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
    uint32_t cnt = 0;
    const uint32_t* lp = find_peers(t, w, x, y, z, &cnt);
    const uint32_t at = lower_bound_dev(lp, cnt, peer[i]);
    out[i] = (at < cnt && lp[at] == peer[i]) ? 1 : 0;
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

int launch_quantize(hipStream_t s, const double* d_in, size_t n, uint16_t cube_size, int64_t* d_out) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(quantize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_in, (uint64_t)n,
                       (double)cube_size, (int64_t)cube_size, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_is_subscribed(wq_router* h, const uint32_t* d_w, const uint32_t* d_p, int raw, const void* d_kp,
                         uint32_t n, uint8_t* d_out) {
    hipLaunchKernelGGL(is_subscribed_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, d_w, d_p, raw, d_kp, n,
                       table_view(h), (int64_t)h->cube_size, d_out);
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
