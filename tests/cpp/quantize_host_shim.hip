// Test-only shim: runs the __host__ __device__ quantiser of wq_device.hpp on the CPU so the
// exact-divisibility rewrite of `abs % size == 0.0` is checked against the
// oracle's fmod form without a GPU. The GPU instance is checked in tests/test_gpu_routing.py
// (test_quantize_*).
#include <stddef.h>
#include <stdint.h>

#include "../../worldql_server_amd/csrc/wq_device.hpp"

extern "C" void wq_test_coord_clamp_host(const double* x, size_t n, uint16_t s, int64_t* out) {
    for (size_t i = 0; i < n; ++i) out[i] = wq::coord_clamp_dev(x[i], (double)s, (int64_t)s);
}

extern "C" uint64_t wq_test_cube_hash_host(uint32_t w, int64_t x, int64_t y, int64_t z) {
    return wq::cube_hash(w, x, y, z);
}

extern "C" void wq_test_shard_of_host(const uint32_t* w, const int64_t* k, size_t n, uint32_t G, uint32_t* out) {
    for (size_t i = 0; i < n; ++i) out[i] = wq::shard_of(w[i], k[3 * i], k[3 * i + 1], k[3 * i + 2], G);
}
