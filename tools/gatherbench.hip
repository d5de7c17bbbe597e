// Calibration: random 16-B gathers per second vs footprint, flat vs XCD-partitioned.
// Each lane issues K independent random loads per round (all in flight), R rounds.
//   flat : every block reads the whole footprint S
//   xcd  : block b reads only region (b % 8) of size S/8 (one XCD's L2 holds its region)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/gatherbench tools/gatherbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return x;
}

template <int K, int XCD, int LINE, int ACT = 8>
__global__ __launch_bounds__(256) void gather(const uint4* __restrict__ buf, uint64_t n16, int rounds,
                                              uint32_t* out) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t region = n16, base = 0;
    if (XCD) {
        region = n16 / 8;
        base = (blockIdx.x & 7) * region;
    }
    uint32_t acc = 0;
    uint64_t x = gid * 0x9E3779B97F4A7C15ull + 1;
    for (int r = 0; r < rounds; ++r) {
        uint4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x = mix(x + k);
            // LINE: 8 lanes share one 128-B line (whole-line reads) when LINE == 1
            uint64_t idx;
            if (LINE) {
                const uint64_t g = __shfl(x, (threadIdx.x & 63) & ~7, 64);
                idx = base + ((g % (region / 8)) * 8 + (threadIdx.x & 7));
            } else {
                idx = base + (x % region);
            }
            if (!LINE || ACT == 8 || (threadIdx.x & 7) < ACT) v[k] = buf[idx];
            else v[k] = make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k].x ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t sizes[] = {2ull << 20, 16ull << 20, 128ull << 20};
    uint4* buf;
    uint32_t* out;
    hipMalloc(&buf, 512ull << 20);
    hipMalloc(&out, 4);
    hipMemset(buf, 1, 512ull << 20);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 2048, rounds = 16;
    auto run = [&](const char* nm, auto launch, int K, bool line) {
        for (uint64_t S : sizes) {
            const uint64_t n16 = S / 16;
            launch(n16);
            hipEventRecord(a);
            for (int i = 0; i < 5; ++i) launch(n16);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double t = ms / 5 * 1e-3;
            const double reqs = (double)blocks * 256 * rounds * K;
            const double lines = line ? reqs / 8 : reqs;
            printf("%-14s S %4llu MB: %7.1f us  %6.1f G lane-loads/s  %6.1f G lines/s\n", nm,
                   (unsigned long long)(S >> 20), t * 1e6, reqs / t / 1e9, lines / t / 1e9);
        }
    };
#define GO(K, X, L, NM)                                                                                        \
    run(NM, [&](uint64_t n16) { hipLaunchKernelGGL((gather<K, X, L>), dim3(blocks), dim3(256), 0, 0, buf, n16, rounds, out); }, K, L)
    GO(8, 0, 0, "flat K8");
    GO(8, 1, 0, "xcd K8");
    GO(8, 0, 1, "flat line K8");
#define GA(A, NM) run(NM, [&](uint64_t n16) { hipLaunchKernelGGL((gather<8, 0, 1, A>), dim3(blocks), dim3(256), 0, 0, buf, n16, rounds, out); }, 8, true)
    GA(1, "line act1");
    GA(2, "line act2");
    GA(3, "line act3");
    GA(4, "line act4");
    return 0;
}
