// Calibration micro-benchmark: random cache-line reads vs footprint on gfx950.
// Each lane reads one 16-B word from a pseudo-random 128-B line of a buffer of S bytes
// (mode 0), or 8 lanes read one whole random line (mode 1), or lanes stream (mode 2).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void rnd(const uint4* __restrict__ buf, uint64_t n_lines, uint64_t iters, uint32_t* out, int mode) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t x = gid * 0x9E3779B97F4A7C15ull + 12345;
    uint32_t acc = 0;
    for (uint64_t it = 0; it < iters; ++it) {
        x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33;
        uint64_t line;
        uint32_t part;
        if (mode == 0) { line = x % n_lines; part = 0; }
        else if (mode == 1) { const uint64_t g = __shfl(x, (threadIdx.x & 63) & ~7, 64); line = g % n_lines; part = threadIdx.x & 7; }
        else { line = (gid + it * gridDim.x * blockDim.x / 8) / 8 % n_lines; part = gid & 7; }
        const uint4 v = buf[line * 8 + part];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678) out[0] = acc;
}

int main() {
    const uint64_t sizes[] = {4ull << 20, 16ull << 20, 64ull << 20, 128ull << 20, 256ull << 20, 1ull << 30, 4ull << 30};
    uint4* buf; uint32_t* out;
    hipMalloc(&buf, 4ull << 30); hipMalloc(&out, 4);
    hipMemset(buf, 1, 4ull << 30);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int mode = 0; mode < 3; ++mode) {
        for (uint64_t S : sizes) {
            const uint64_t n_lines = S / 128;
            const int blocks = 256 * 8, threads = 256;
            const uint64_t iters = 64;
            hipLaunchKernelGGL(rnd, dim3(blocks), dim3(threads), 0, 0, buf, n_lines, iters, out, mode);
            hipEventRecord(a);
            hipLaunchKernelGGL(rnd, dim3(blocks), dim3(threads), 0, 0, buf, n_lines, iters, out, mode);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            const double reqs = (double)blocks * threads * iters;
            const double lines = mode == 0 ? reqs : reqs / 8;
            printf("mode %d size %6llu MB: %.1f us, %.2f G lane-req/s, %.2f G lines/s, %.2f TB/s of lines\n", mode,
                   (unsigned long long)(S >> 20), ms * 1e3, reqs / ms / 1e6, lines / ms / 1e6, lines * 128 / ms / 1e9);
        }
    }
    return 0;
}
