// Calibration: the count pass's memory shape on gfx950, without its arithmetic.
// M messages, lane per message: stream 33 B of inputs, read one random 128-B line of a table
// (all 8 x 16 B by the lane), optionally a dependent second line for a fraction of lanes (a
// linear-probe collision), write 12 B. Lines are drawn from `distinct` occupied lines of a
// table of `table_lines` slots, as the C2 record table (286k cubes in 1M slots).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probebench tools/probebench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int IPT, int LINE_WORDS>
__global__ __launch_bounds__(256) void probe(const uint4* __restrict__ tab, const uint32_t* __restrict__ occ,
                                             uint32_t n_occ, uint32_t tab_mask, const double* __restrict__ pos,
                                             const uint32_t* __restrict__ w, uint32_t M, uint32_t collide_pct,
                                             int with_inputs, uint32_t* __restrict__ e, uint2* __restrict__ info) {
    const uint32_t m0 = blockIdx.x * 256 * IPT + threadIdx.x;
    double px[IPT];
    uint32_t wv[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * 256;
        const uint32_t mm = m < M ? m : 0;
        px[i] = with_inputs ? pos[3ull * mm] + pos[3ull * mm + 1] + pos[3ull * mm + 2] : 0.0;
        wv[i] = with_inputs ? w[mm] : 0u;
    }
    uint32_t sl[IPT];
    uint4 v[IPT][LINE_WORDS];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * 256;
        const uint64_t h = mix(m + (uint64_t)__double_as_longlong(px[i]) * 0 + wv[i] * 0);
        sl[i] = occ[h % n_occ];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i)
#pragma unroll
        for (int q = 0; q < LINE_WORDS; ++q) v[i][q] = tab[(uint64_t)sl[i] * 8 + q];
    bool again[IPT];
    bool any = false;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        again[i] = (mix(m0 + i * 256 + 77) % 100) < collide_pct && (v[i][0].x != 0xdeadbeef);
        any |= again[i];
    }
    if (__any(any)) {
#pragma unroll
        for (int i = 0; i < IPT; ++i)
            if (again[i])
#pragma unroll
                for (int q = 0; q < LINE_WORDS; ++q) v[i][q] = tab[(uint64_t)((sl[i] + 1) & tab_mask) * 8 + q];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * 256;
        uint32_t acc = 0;
#pragma unroll
        for (int q = 0; q < LINE_WORDS; ++q) acc += v[i][q].x ^ v[i][q].y ^ v[i][q].z ^ v[i][q].w;
        if (m < M) {
            e[m] = acc;
            info[m] = make_uint2(sl[i], acc);
        }
    }
}

__global__ void flush(uint4* buf, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        buf[i] = make_uint4(i, 0, 0, 0);
}

int main() {
    const uint32_t M = 1000000, T = 1u << 20, n_occ = 286341;
    uint4* tab;
    uint32_t *occ, *w, *e;
    double* pos;
    uint2* info;
    hipMalloc(&tab, (size_t)T * 128);
    hipMalloc(&occ, n_occ * 4);
    hipMalloc(&pos, (size_t)M * 24);
    hipMalloc(&w, M * 4);
    hipMalloc(&e, M * 4);
    hipMalloc(&info, M * 8);
    hipMemset(tab, 1, (size_t)T * 128);
    hipMemset(pos, 0, (size_t)M * 24);
    hipMemset(w, 0, M * 4);
    uint32_t* h = new uint32_t[n_occ];
    uint64_t x = 1;
    for (uint32_t i = 0; i < n_occ; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        h[i] = (uint32_t)(x >> 33) & (T - 1);
    }
    hipMemcpy(occ, h, n_occ * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    uint4* fl;
    const uint64_t fl_n = (128ull << 20) / 16;  // 128 MB streamed between probes (an emit pass's worth)
    hipMalloc(&fl, fl_n * 16);
    struct V {
        const char* name;
        int ipt, words, collide, inputs;
    } vs[] = {
        {"1 line, no collide, inputs", 1, 8, 0, 1},   {"1 line, 18% collide, inputs", 1, 8, 18, 1},
        {"IPT2 line, 18% collide, inputs", 2, 8, 18, 1}, {"IPT2 line, 0% collide, inputs", 2, 8, 0, 1},
        {"header only (16B), 0% collide", 1, 1, 0, 1}, {"header only IPT2, 18% collide", 2, 1, 18, 1},
        {"IPT4 header only, 0%", 4, 1, 0, 1},           {"1 line, 0%, no inputs", 1, 8, 0, 0},
    };
    for (auto& vv : vs) {
        auto launch = [&]() {
            const unsigned grid = (M + 256 * vv.ipt - 1) / (256 * vv.ipt);
#define L(I, W)                                                                                                 \
    if (vv.ipt == I && vv.words == W)                                                                           \
        hipLaunchKernelGGL((probe<I, W>), dim3(grid), dim3(256), 0, 0, tab, occ, n_occ, T - 1, pos, w, M,       \
                           (uint32_t)vv.collide, vv.inputs, e, info);
            L(1, 8) L(2, 8) L(1, 1) L(2, 1) L(4, 1)
#undef L
        };
        for (int r = 0; r < 3; ++r) launch();
        hipEventRecord(a);
        for (int r = 0; r < 20; ++r) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        float cold = 0;
        for (int r = 0; r < 20; ++r) {
            hipLaunchKernelGGL(flush, dim3(2048), dim3(256), 0, 0, fl, fl_n);
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float t;
            hipEventElapsedTime(&t, a, b);
            cold += t;
        }
        printf("%-34s warm %7.1f us   after 128 MB stream %7.1f us\n", vv.name, ms * 1e3 / 20, cold * 1e3 / 20);
    }
    // HBM-bound sector test: 8M messages over 8M distinct lines of a 2 GB table (past the 256 MB
    // Infinity Cache): does reading 16 / 64 B of a line cost less than the whole 128 B?
    {
        const uint32_t M2 = 8u << 20, T2 = 16u << 20, occ2 = 8u << 20;
        uint4* tab2;
        uint32_t *o2, *e2;
        uint2* i2;
        double* p2;
        uint32_t* w2;
        hipMalloc(&tab2, (size_t)T2 * 128);
        hipMalloc(&o2, (size_t)occ2 * 4);
        hipMalloc(&e2, (size_t)M2 * 4);
        hipMalloc(&i2, (size_t)M2 * 8);
        hipMalloc(&p2, (size_t)M2 * 24);
        hipMalloc(&w2, (size_t)M2 * 4);
        hipMemset(tab2, 1, (size_t)T2 * 128);
        uint32_t* hh = new uint32_t[occ2];
        for (uint32_t i = 0; i < occ2; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            hh[i] = (uint32_t)(x >> 33) & (T2 - 1);
        }
        hipMemcpy(o2, hh, (size_t)occ2 * 4, hipMemcpyHostToDevice);
        for (int words : {1, 2, 4, 8}) {
            auto go = [&]() {
                const unsigned grid = (M2 + 511) / 512;
#define L2(W) if (words == W) hipLaunchKernelGGL((probe<2, W>), dim3(grid), dim3(256), 0, 0, tab2, o2, occ2, T2 - 1, p2, w2, M2, 0u, 0, e2, i2);
                L2(1) L2(2) L2(4) L2(8)
#undef L2
            };
            go();
            hipEventRecord(a);
            for (int r = 0; r < 5; ++r) go();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double t = ms / 5 * 1e-3;
            printf("HBM-bound: %3d B of each random line: %8.1f us  %.2f G lines/s  %.2f TB/s if whole lines\n",
                   words * 16, t * 1e6, M2 / t / 1e9, M2 * 128.0 / t / 1e12);
        }
    }
    return 0;
}
