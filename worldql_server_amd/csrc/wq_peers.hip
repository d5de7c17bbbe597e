// wq_peers.hip — per-peer send lists for the transport.
//
// After a tick the reference calls PeerMap::broadcast_to once per message
// (worldql_server/src/transport/peer_map.rs:151-163): it intersects the recipients with the
// connected peers and sends the message to each. A GPU tick hands the host a message-major CSR;
// a transport that batches per socket wants the transpose — for every peer, the messages it must
// receive — with the disconnected peers already dropped. Here:
//   expand   one lane per message writes (peer or sentinel, message) for each of its recipients;
//            peers outside the `connected` bitmap (or >= n_peers) get the sentinel n_peers
//   sort     one stable radix sort by peer over log2(n_peers + 1) bits (message order kept)
//   offsets  one lane per peer: lower bound of the peer in the sorted keys
// The kept messages of peer p are msgs_out[peer_offsets[p] .. peer_offsets[p + 1]), ascending.
#include "table_prims.hpp"

namespace wq {

namespace {

__global__ void k_pm_expand(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ peers, uint32_t M,
                            const uint32_t* __restrict__ connected, uint32_t n_peers, uint32_t* key, uint32_t* msg) {
    const uint32_t m = blockIdx.x * kBlock + threadIdx.x;
    if (m >= M) return;
    const uint32_t a = offsets[m], b = offsets[m + 1];
    for (uint32_t j = a; j < b; ++j) {
        const uint32_t p = peers[j];
        const bool on = p < n_peers && (!connected || ((connected[p >> 5] >> (p & 31)) & 1u));
        key[j] = on ? p : n_peers;
        msg[j] = m;
    }
}

__global__ void k_pm_offsets(const uint32_t* __restrict__ skey, uint32_t P, uint32_t n_peers, uint32_t* out) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p > n_peers) return;
    uint32_t lo = 0, hi = P;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (skey[mid] < p)
            lo = mid + 1;
        else
            hi = mid;
    }
    out[p] = lo;
}

}  // namespace

int launch_peer_major(wq_router* h, const uint32_t* d_offsets, const uint32_t* d_peers, size_t M, size_t P,
                      const uint32_t* d_connected, uint32_t n_peers, uint32_t* d_peer_offsets, uint32_t* d_msgs_out) {
    hipStream_t s = h->stream;
    if (P == 0) {
        hipLaunchKernelGGL(k_pm_offsets, dim3(grid_for((uint64_t)n_peers + 1)), dim3(kBlock), 0, s, d_peer_offsets,
                           0u, n_peers, d_peer_offsets);
        WQ_HIP(h, hipGetLastError());
        return WQ_OK;
    }
    WQ_ALLOC(h, h->key32_a, P * 4);
    WQ_ALLOC(h, h->key32_b, P * 4);
    WQ_ALLOC(h, h->idx_a, P * 4);
    uint32_t* key = h->key32_a.as<uint32_t>();
    uint32_t* skey = h->key32_b.as<uint32_t>();
    uint32_t* msg = h->idx_a.as<uint32_t>();
    if (M)
        hipLaunchKernelGGL(k_pm_expand, dim3(grid_for(M)), dim3(kBlock), 0, s, d_offsets, d_peers, (uint32_t)M,
                           d_connected, n_peers, key, msg);
    int bits = 1;
    while ((1ull << bits) <= n_peers) bits++;
    int rc = sort_pairs<uint32_t>(h, key, skey, msg, d_msgs_out, P, bits);
    if (rc) return rc;
    hipLaunchKernelGGL(k_pm_offsets, dim3(grid_for((uint64_t)n_peers + 1)), dim3(kBlock), 0, s, skey, (uint32_t)P,
                       n_peers, d_peer_offsets);
    WQ_HIP(h, hipGetLastError());
    return WQ_OK;
}

}  // namespace wq
