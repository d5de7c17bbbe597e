// Probe: lane exchanges by DPP / permlane swaps against __shfl_xor (gfx950). Prints OK or mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../worldql_server_amd/csrc/lane_xchg.hpp"

__global__ void k(unsigned* out) {
    const int lane = threadIdx.x;
    const unsigned v = lane * 7919u + 13u;
    out[0 * 64 + lane] = wq::xchg_u32<1>(v, lane) ^ __shfl_xor(v, 1, 64);
    out[1 * 64 + lane] = wq::xchg_u32<2>(v, lane) ^ __shfl_xor(v, 2, 64);
    out[2 * 64 + lane] = wq::xchg_u32<4>(v, lane) ^ __shfl_xor(v, 4, 64);
    out[3 * 64 + lane] = wq::xchg_u32<8>(v, lane) ^ __shfl_xor(v, 8, 64);
    out[4 * 64 + lane] = wq::xchg_u32<16>(v, lane) ^ __shfl_xor(v, 16, 64);
    out[5 * 64 + lane] = wq::xchg_u32<32>(v, lane) ^ __shfl_xor(v, 32, 64);
}

int main() {
    unsigned* d;
    unsigned h[6 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int j = 0; j < 6; ++j)
        for (int l = 0; l < 64; ++l)
            if (h[j * 64 + l]) { if (bad < 10) printf("mismatch xor %d lane %d\n", 1 << j, l); ++bad; }
    printf(bad ? "FAIL %d\n" : "OK\n", bad);
    return bad ? 1 : 0;
}
