// fetchcal — what rocprofv3's FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ report on gfx950 for the
// access shapes of the route kernels, against byte counts known by construction (VERDICT r3
// "calibrate roofline.traffic"). Every shape runs over a 4 GiB buffer (16x the 256 MiB Infinity
// Cache; every line touched once per launch where the shape is random), once per launch:
//   stream16_rd   64 lanes x 16 B coalesced, the whole span once                  (inputs, e/info)
//   stream4_rd    64 lanes x 4 B coalesced, the whole span once                   (e, offsets)
//   line32_rd     per lane the first 32 B (two 16-B loads) of one random 128-B line (count: header)
//   line64_rd     per lane the first 64 B (four 16-B loads) of one random line
//   line128_rd    per lane the whole 128-B line (eight 16-B loads)                 (count FULL, radius)
//   run_rd        per wave one run of 64 consecutive 4-B words at a random 4-B aligned offset
//                 (emit: a cube's list, 256 B that straddle 2-3 lines)
//   word4_rd      per lane one random 4-B word                                     (position codes)
//   stream16_wr   64 lanes x 16 B coalesced stores                                 (tick copy-out)
//   stream4_wr    64 lanes x 4 B coalesced stores                                  (emit peers / msgs)
// Every random index is a permutation-free hash of the lane id over the span's lines (repeats are
// counted in `lines_distinct`, computed on the host), so the known byte counts are exact.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetchcal tools/fetchcal.hip
// Run (GPU box): rocprofv3 --pmc FETCH_SIZE -- tools/fetchcal   (one counter group per pass),
// then tools/fetchcal_summary.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

__host__ __device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

constexpr uint64_t kBytes = 4ull << 30;  // 4 GiB
constexpr uint64_t kLines = kBytes / 128;

// sinks keep the loads alive without a store per lane (one store per wave)
__global__ void stream16_rd(const uint4* __restrict__ a, uint64_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void stream4_rd(const uint32_t* __restrict__ a, uint64_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) acc ^= a[i];
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <int Q>
__global__ void line_rd(const uint4* __restrict__ a, uint64_t n_lanes, uint32_t* __restrict__ sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_lanes) return;
    const uint64_t line = mix(i * 0x9E3779B97F4A7C15ull + 1) % kLines;
    uint4 v[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = a[line * 8 + q];
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// per lane: the first 32 B of a random line, then — after that load has returned — bytes 64-95 of
// the same line: a hit in L2 (TCC_HIT) iff the first request brought the whole 128-B line in
__global__ void halves_rd(const uint4* __restrict__ a, uint64_t n_lanes, uint32_t* __restrict__ sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_lanes) return;
    const uint64_t line = mix(i * 0x9E3779B97F4A7C15ull + 1) % kLines;
    const uint4 v0 = a[line * 8], v1 = a[line * 8 + 1];
    const uint64_t dep = (v0.x ^ v1.y) == 0x9e3779b9u ? 1 : 0;  // the address waits for the data
    const uint4 w0 = a[(line + dep) * 8 + 4], w1 = a[(line + dep) * 8 + 5];
    const uint32_t acc = v0.x ^ v1.y ^ w0.z ^ w1.w;
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void run_rd(const uint32_t* __restrict__ a, uint64_t n_waves, uint32_t* __restrict__ sink) {
    const uint64_t w = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    if (w >= n_waves) return;
    const uint64_t start = mix(w * 0x9E3779B97F4A7C15ull + 7) % (kBytes / 4 - 64);
    const uint32_t v = a[start + (threadIdx.x & 63)];
    if (v == 0x9e3779b9u) sink[0] = v;
}

__global__ void word4_rd(const uint32_t* __restrict__ a, uint64_t n_lanes, uint32_t* __restrict__ sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_lanes) return;
    const uint32_t v = a[mix(i * 0x9E3779B97F4A7C15ull + 3) % (kBytes / 4)];
    if (v == 0x9e3779b9u) sink[0] = v;
}

__global__ void stream16_wr(uint4* __restrict__ a, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        a[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ void stream4_wr(uint32_t* __restrict__ a, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        a[i] = (uint32_t)i;
}

// distinct lines (and for run_rd: distinct 128-B lines its runs touch) of a shape's random indices
static uint64_t distinct_lines(uint64_t n, int kind) {
    std::vector<uint8_t> seen(kLines / 8 + 1, 0);
    uint64_t d = 0;
    auto mark = [&](uint64_t l) {
        if (!(seen[l >> 3] & (1u << (l & 7)))) {
            seen[l >> 3] |= (uint8_t)(1u << (l & 7));
            ++d;
        }
    };
    for (uint64_t i = 0; i < n; ++i) {
        if (kind == 0) {
            mark(mix(i * 0x9E3779B97F4A7C15ull + 1) % kLines);
        } else if (kind == 1) {
            const uint64_t s = mix(i * 0x9E3779B97F4A7C15ull + 7) % (kBytes / 4 - 64);
            for (uint64_t l = (s * 4) / 128; l <= (s * 4 + 255) / 128; ++l) mark(l);
        } else {
            mark((mix(i * 0x9E3779B97F4A7C15ull + 3) % (kBytes / 4)) * 4 / 128);
        }
    }
    return d;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    void* buf = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 0x5a, kBytes));
    CHECK(hipDeviceSynchronize());
    const uint64_t n_rand = 16ull << 20;  // 16M random lanes (of 33.5M lines)
    const uint64_t n_runs = 4ull << 20;   // 4M runs of 256 B
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    printf("{\"buffer_bytes\": %llu, \"shapes\": [\n", (unsigned long long)kBytes);
    struct Shape {
        const char* name;
        int kind;  // for distinct counts: 0 line, 1 run, 2 word, -1 streaming
        uint64_t units;
        double req_bytes;  // bytes requested by the shape's loads / stores per launch
    };
    const Shape shapes[] = {
        {"stream16_rd", -1, kBytes / 16, (double)kBytes},
        {"stream4_rd", -1, kBytes / 4, (double)kBytes},
        {"line32_rd", 0, n_rand, 32.0 * n_rand},
        {"line64_rd", 0, n_rand, 64.0 * n_rand},
        {"line128_rd", 0, n_rand, 128.0 * n_rand},
        {"run_rd", 1, n_runs, 256.0 * n_runs},
        {"halves_rd", 0, n_rand, 64.0 * n_rand},
        {"word4_rd", 2, n_rand, 4.0 * n_rand},
        {"stream16_wr", -1, kBytes / 16, (double)kBytes},
        {"stream4_wr", -1, kBytes / 4, (double)kBytes},
    };
    const unsigned grid_stream = 256 * 32;
    for (size_t k = 0; k < sizeof(shapes) / sizeof(shapes[0]); ++k) {
        const Shape& s = shapes[k];
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CHECK(hipEventRecord(e0));
            switch (k) {
                case 0: hipLaunchKernelGGL(stream16_rd, dim3(grid_stream), dim3(256), 0, 0, (const uint4*)buf, s.units, sink); break;
                case 1: hipLaunchKernelGGL(stream4_rd, dim3(grid_stream), dim3(256), 0, 0, (const uint32_t*)buf, s.units, sink); break;
                case 2: hipLaunchKernelGGL(line_rd<2>, dim3((unsigned)(s.units / 256)), dim3(256), 0, 0, (const uint4*)buf, s.units, sink); break;
                case 3: hipLaunchKernelGGL(line_rd<4>, dim3((unsigned)(s.units / 256)), dim3(256), 0, 0, (const uint4*)buf, s.units, sink); break;
                case 4: hipLaunchKernelGGL(line_rd<8>, dim3((unsigned)(s.units / 256)), dim3(256), 0, 0, (const uint4*)buf, s.units, sink); break;
                case 5: hipLaunchKernelGGL(run_rd, dim3((unsigned)(s.units * 64 / 256)), dim3(256), 0, 0, (const uint32_t*)buf, s.units, sink); break;
                case 6: hipLaunchKernelGGL(halves_rd, dim3((unsigned)(s.units / 256)), dim3(256), 0, 0, (const uint4*)buf, s.units, sink); break;
                case 7: hipLaunchKernelGGL(word4_rd, dim3((unsigned)(s.units / 256)), dim3(256), 0, 0, (const uint32_t*)buf, s.units, sink); break;
                case 8: hipLaunchKernelGGL(stream16_wr, dim3(grid_stream), dim3(256), 0, 0, (uint4*)buf, s.units); break;
                case 9: hipLaunchKernelGGL(stream4_wr, dim3(grid_stream), dim3(256), 0, 0, (uint32_t*)buf, s.units); break;
            }
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const uint64_t distinct = s.kind >= 0 ? distinct_lines(s.units, s.kind) : (uint64_t)(s.req_bytes / 128);
        printf("  {\"shape\": \"%s\", \"units\": %llu, \"requested_bytes\": %.0f, \"lines_distinct\": %llu, "
               "\"best_ms\": %.4f, \"requested_GBps\": %.1f, \"lines_G_per_s\": %.2f}%s\n",
               s.name, (unsigned long long)s.units, s.req_bytes, (unsigned long long)distinct, best,
               s.req_bytes / best / 1e6, distinct / best / 1e6, k + 1 < sizeof(shapes) / sizeof(shapes[0]) ? "," : "");
        fflush(stdout);
    }
    printf("], \"reps\": %d}\n", reps);
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
