// Calibration: does an XCD-partitioned probe (radix-partitioned hash join) beat the flat one?
// C2-shaped synthetic tick: 286,341 cubes with 5..14 peers each, 1M messages, random senders.
//   bin        : read 33 B/msg of inputs, group messages into 8 bins by cube hash (16-B records)
//   probe_bin  : blocks b = j (mod 8) probe bin j against sub-table j (compact 16-B slots + lists),
//                so each XCD's L2 holds one eighth of the table; writes e[m], loc[m] scattered
//   probe_flat : the same probe in message order against one flat table (no bin pass)
//   emit_lds   : message order; gathers each list into LDS at its output offset, then one
//                coalesced copy of peers + msg ids
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/partbench tools/partbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            printf("HIP error %s at %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

__host__ __device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
__host__ __device__ __forceinline__ uint32_t part_of(uint32_t c) { return (uint32_t)(mix(c + 7) >> 61); }
__host__ __device__ __forceinline__ uint64_t slot_hash(uint32_t c) { return mix(c * 0x9E3779B97F4A7C15ull + 3); }

struct SubTab {
    uint64_t base;  // first slot (uint4 index) of this sub-table
    uint32_t mask;
    uint32_t pad;
};

// record: x = cube+1 (key), y = sender, z = m, w = 0
template <int IPT>
__global__ __launch_bounds__(256) void k_bin(const double* __restrict__ pos, const uint32_t* __restrict__ cube,
                                             const uint32_t* __restrict__ sender, const uint8_t* __restrict__ repl,
                                             uint32_t M, uint4* __restrict__ bins, uint64_t bin_cap,
                                             uint32_t* __restrict__ cursor) {
    __shared__ uint32_t hist[8], start[8], gbase[8];
    __shared__ uint4 stage[256 * IPT];
    __shared__ uint8_t sbin[256 * IPT];
    const int tid = threadIdx.x;
    if (tid < 8) hist[tid] = 0;
    __syncthreads();
    const uint32_t m0 = blockIdx.x * 256 * IPT;
    uint4 rec[IPT];
    uint32_t pb[IPT], rk[IPT];
    bool ok[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * 256 + tid;
        ok[i] = m < M;
        const uint32_t mm = ok[i] ? m : 0;
        const double s = pos[3ull * mm] + pos[3ull * mm + 1] + pos[3ull * mm + 2];
        const uint32_t c = cube[mm] + (s == 12345.5 ? 1u : 0u) + repl[mm];
        rec[i] = make_uint4(c + 1, sender[mm], m, 0);
        pb[i] = part_of(c);
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) rk[i] = ok[i] ? atomicAdd(&hist[pb[i]], 1u) : 0u;
    __syncthreads();
    if (tid == 0) {
        uint32_t s = 0;
        for (int j = 0; j < 8; ++j) {
            start[j] = s;
            s += hist[j];
            gbase[j] = hist[j] ? atomicAdd(&cursor[j], hist[j]) : 0u;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IPT; ++i)
        if (ok[i]) {
            stage[start[pb[i]] + rk[i]] = rec[i];
            sbin[start[pb[i]] + rk[i]] = (uint8_t)pb[i];
        }
    __syncthreads();
    const uint32_t n = min((uint32_t)(256 * IPT), M - m0);
    for (uint32_t i = tid; i < n; i += 256) {
        const uint32_t j = sbin[i];
        bins[(uint64_t)j * bin_cap + gbase[j] + (i - start[j])] = stage[i];
    }
}

__device__ __forceinline__ void probe_one(const uint4* __restrict__ slots, const SubTab& st, uint32_t key,
                                          uint32_t me, const uint4* __restrict__ lists4, uint32_t* e_out,
                                          uint2* loc_out) {
    uint64_t i = (slot_hash(key - 1) & st.mask);
    uint4 s = slots[st.base + i];
    while (s.x != key && s.x != 0) {
        i = (i + 1) & st.mask;
        s = slots[st.base + i];
    }
    const uint32_t off = s.z, cnt = s.x ? s.w : 0u;  // off: word offset, 16-B aligned
    uint32_t skip = 0xFFFFFFFFu;
    for (uint32_t q = 0; q < cnt; q += 4) {
        const uint4 v = lists4[(off + q) >> 2];
        skip = (v.x == me) ? q : skip;
        skip = (q + 1 < cnt && v.y == me) ? q + 1 : skip;
        skip = (q + 2 < cnt && v.z == me) ? q + 2 : skip;
        skip = (q + 3 < cnt && v.w == me) ? q + 3 : skip;
    }
    *e_out = cnt - (skip != 0xFFFFFFFFu ? 1u : 0u);
    *loc_out = make_uint2(off, (cnt << 16) | (skip & 0xFFFFu));
}

// BIN_OF_BLOCK: 0 = bin j = b % 8 (XCD-local), 1 = bin j = (b / 8) % 8 (spread over all XCDs)
template <int IPT, int BIN_OF_BLOCK>
__global__ __launch_bounds__(256) void k_probe_bin(const uint4* __restrict__ bins, uint64_t bin_cap,
                                                   const uint32_t* __restrict__ cursor,
                                                   const uint4* __restrict__ slots, const SubTab* __restrict__ subs,
                                                   const uint4* __restrict__ lists4, uint32_t* __restrict__ e,
                                                   uint2* __restrict__ loc) {
    const uint32_t nb = gridDim.x / 8;
    const uint32_t j = BIN_OF_BLOCK == 0 ? (blockIdx.x & 7) : ((blockIdx.x / nb) & 7);
    const uint32_t k = BIN_OF_BLOCK == 0 ? (blockIdx.x >> 3) : (blockIdx.x % nb);
    const uint32_t n = cursor[j];
    const SubTab st = subs[j];
    const uint4* b = bins + (uint64_t)j * bin_cap;
    for (uint32_t s0 = k * 256 * IPT; s0 < n; s0 += nb * 256 * IPT) {
        uint4 r[IPT];
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            const uint32_t s = s0 + i * 256 + threadIdx.x;
            r[i] = s < n ? b[s] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
            if (r[i].x == 0) continue;
            uint32_t ev;
            uint2 lv;
            probe_one(slots, st, r[i].x, r[i].y, lists4, &ev, &lv);
            e[r[i].z] = ev;
            loc[r[i].z] = lv;
        }
    }
}

template <int IPT>
__global__ __launch_bounds__(256) void k_probe_flat(const double* __restrict__ pos, const uint32_t* __restrict__ cube,
                                                    const uint32_t* __restrict__ sender,
                                                    const uint8_t* __restrict__ repl, uint32_t M,
                                                    const uint4* __restrict__ slots, SubTab st,
                                                    const uint4* __restrict__ lists4, uint32_t* __restrict__ e,
                                                    uint2* __restrict__ loc) {
    const uint32_t m0 = blockIdx.x * 256 * IPT;
    uint32_t key[IPT], me[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * 256 + threadIdx.x;
        const uint32_t mm = m < M ? m : 0;
        const double s = pos[3ull * mm] + pos[3ull * mm + 1] + pos[3ull * mm + 2];
        key[i] = cube[mm] + 1 + (s == 12345.5 ? 1u : 0u) + repl[mm];
        me[i] = sender[mm];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const uint32_t m = m0 + i * 256 + threadIdx.x;
        if (m >= M) continue;
        uint32_t ev;
        uint2 lv;
        probe_one(slots, st, key[i], me[i], lists4, &ev, &lv);
        e[m] = ev;
        loc[m] = lv;
    }
}

// message order; offs = exact exclusive prefix of e (precomputed: the scan is not measured here)
constexpr int kEmitMsgs = 512;
constexpr int kEmitCap = kEmitMsgs * 16;
__global__ __launch_bounds__(256) void k_emit_lds(const uint2* __restrict__ loc, const uint32_t* __restrict__ offs,
                                                  uint32_t M, const uint4* __restrict__ lists4,
                                                  uint32_t* __restrict__ out_p, uint32_t* __restrict__ out_m) {
    __shared__ uint32_t sp[kEmitCap], sm[kEmitCap];
    const uint32_t m0 = blockIdx.x * kEmitMsgs;
    const uint32_t mend = min(M, m0 + kEmitMsgs);
    const uint32_t o0 = offs[m0];
    const uint32_t o1 = offs[mend];
    for (int i = 0; i < kEmitMsgs / 256; ++i) {
        const uint32_t m = m0 + i * 256 + threadIdx.x;
        if (m >= mend) continue;
        const uint2 l = loc[m];
        const uint32_t cnt = l.y >> 16, skip = l.y & 0xFFFFu;
        uint32_t o = offs[m] - o0;
        for (uint32_t q = 0; q < cnt; q += 4) {
            const uint4 v = lists4[(l.x + q) >> 2];
            const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t idx = q + t;
                if (idx < cnt && idx != skip) {
                    sp[o] = vv[t];
                    sm[o] = m;
                    ++o;
                }
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < o1 - o0; i += 256) {
        out_p[o0 + i] = sp[i];
        out_m[o0 + i] = sm[i];
    }
}

__global__ void flush(uint4* buf, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        buf[i] = make_uint4(i, 0, 0, 0);
}

int main() {
    const uint32_t M = 1000000, NC = 286341, NP = 100000;
    // ---- host table ----
    std::vector<uint32_t> cnt(NC), part(NC), off(NC);
    uint64_t x = 42;
    for (uint32_t c = 0; c < NC; ++c) {
        cnt[c] = 5 + (uint32_t)(mix(c * 31 + 1) % 10);
        part[c] = part_of(c);
    }
    std::vector<uint32_t> lists;
    uint32_t np[8] = {0};
    for (uint32_t j = 0; j < 8; ++j)
        for (uint32_t c = 0; c < NC; ++c)
            if (part[c] == j) {
                np[j]++;
                off[c] = (uint32_t)lists.size();
                uint32_t p = (uint32_t)(mix(c * 7 + 11) % (NP / 2));
                for (uint32_t q = 0; q < cnt[c]; ++q) {
                    lists.push_back(p);
                    p += 1 + (uint32_t)(mix(c * 1000 + q) % 8);
                }
                while (lists.size() % 4) lists.push_back(0xFFFFFFFFu);
            }
    std::vector<SubTab> subs(8);
    uint64_t total_slots = 0;
    for (int j = 0; j < 8; ++j) {
        uint32_t cap = 1024;
        while (cap < 2 * np[j]) cap <<= 1;
        subs[j].base = total_slots;
        subs[j].mask = cap - 1;
        total_slots += cap;
    }
    std::vector<uint4> slots(total_slots, make_uint4(0, 0, 0, 0));
    uint32_t fcap = 1024;
    while (fcap < 2 * NC) fcap <<= 1;
    std::vector<uint4> fslots(fcap, make_uint4(0, 0, 0, 0));
    for (uint32_t c = 0; c < NC; ++c) {
        const SubTab& st = subs[part[c]];
        uint64_t i = slot_hash(c) & st.mask;
        while (slots[st.base + i].x) i = (i + 1) & st.mask;
        slots[st.base + i] = make_uint4(c + 1, 0, off[c], cnt[c]);
        uint64_t f = slot_hash(c) & (fcap - 1);
        while (fslots[f].x) f = (f + 1) & (fcap - 1);
        fslots[f] = make_uint4(c + 1, 0, off[c], cnt[c]);
    }
    std::vector<uint32_t> mc(M), ms(M);
    std::vector<uint8_t> mr(M, 0);
    std::vector<double> mp(3ull * M, 1.0);
    for (uint32_t m = 0; m < M; ++m) {
        mc[m] = (uint32_t)(mix(m * 3 + 5) % NC);
        const uint32_t c = mc[m];
        // half the senders are subscribed to the cube
        ms[m] = (m & 1) ? lists[off[c] + (uint32_t)(mix(m) % cnt[c])] : (uint32_t)(mix(m + 99) % NP);
    }
    std::vector<uint32_t> ex(M + 1, 0);
    for (uint32_t m = 0; m < M; ++m) {
        const uint32_t c = mc[m];
        uint32_t has = 0;
        for (uint32_t q = 0; q < cnt[c]; ++q) has |= lists[off[c] + q] == ms[m];
        ex[m + 1] = ex[m] + cnt[c] - has;
    }
    const uint64_t P = ex[M];
    printf("cubes %u, slots %llu (%.1f MB), flat %u (%.1f MB), lists %.1f MB, P %llu\n", NC,
           (unsigned long long)total_slots, total_slots * 16 / 1e6, fcap, fcap * 16 / 1e6, lists.size() * 4 / 1e6,
           (unsigned long long)P);
    // ---- device ----
    double* d_pos;
    uint32_t *d_c, *d_s, *d_e, *d_e2, *d_cur, *d_offs, *d_lists, *d_op, *d_om;
    uint8_t* d_r;
    uint4 *d_bins, *d_slots, *d_fslots;
    uint2 *d_loc, *d_loc2;
    SubTab* d_subs;
    const uint64_t bin_cap = M;
    CK(hipMalloc(&d_pos, 24ull * M));
    CK(hipMalloc(&d_c, 4ull * M));
    CK(hipMalloc(&d_s, 4ull * M));
    CK(hipMalloc(&d_r, M));
    CK(hipMalloc(&d_e, 4ull * M));
    CK(hipMalloc(&d_e2, 4ull * M));
    CK(hipMalloc(&d_loc, 8ull * M));
    CK(hipMalloc(&d_loc2, 8ull * M));
    CK(hipMalloc(&d_cur, 64));
    CK(hipMalloc(&d_offs, 4ull * (M + 1)));
    CK(hipMalloc(&d_bins, 16ull * 8 * bin_cap));
    CK(hipMalloc(&d_slots, 16ull * total_slots));
    CK(hipMalloc(&d_fslots, 16ull * fcap));
    CK(hipMalloc(&d_lists, 4ull * lists.size()));
    CK(hipMalloc(&d_subs, sizeof(SubTab) * 8));
    CK(hipMalloc(&d_op, 4ull * P + 64));
    CK(hipMalloc(&d_om, 4ull * P + 64));
    CK(hipMemcpy(d_pos, mp.data(), 24ull * M, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_c, mc.data(), 4ull * M, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_s, ms.data(), 4ull * M, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_r, mr.data(), M, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_offs, ex.data(), 4ull * (M + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_slots, slots.data(), 16ull * total_slots, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_fslots, fslots.data(), 16ull * fcap, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lists, lists.data(), 4ull * lists.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_subs, subs.data(), sizeof(SubTab) * 8, hipMemcpyHostToDevice));
    const uint4* lists4 = reinterpret_cast<const uint4*>(d_lists);
    SubTab fst{0, fcap - 1, 0};

    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto fn, int reps = 20) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-44s %8.1f us\n", name, ms * 1e3 / reps);
        return ms * 1e3 / reps;
    };
    auto bin = [&]() {
        CK(hipMemsetAsync(d_cur, 0, 64));
        hipLaunchKernelGGL((k_bin<2>), dim3((M + 511) / 512), dim3(256), 0, 0, d_pos, d_c, d_s, d_r, M, d_bins,
                           bin_cap, d_cur);
    };
    timeit("bin (memset + 8-way partition, 16-B recs)", bin);
    std::vector<uint32_t> hc(8);
    CK(hipMemcpy(hc.data(), d_cur, 32, hipMemcpyDeviceToHost));
    printf("bin sizes: %u %u %u %u %u %u %u %u\n", hc[0], hc[1], hc[2], hc[3], hc[4], hc[5], hc[6], hc[7]);
    for (int grid : {1024, 2048, 4096}) {
        char nm[96];
        snprintf(nm, sizeof nm, "probe_bin xcd-local IPT2 grid %d", grid);
        timeit(nm, [&]() {
            hipLaunchKernelGGL((k_probe_bin<2, 0>), dim3(grid), dim3(256), 0, 0, d_bins, bin_cap, d_cur, d_slots,
                               d_subs, lists4, d_e, d_loc);
        });
        snprintf(nm, sizeof nm, "probe_bin xcd-local IPT4 grid %d", grid);
        timeit(nm, [&]() {
            hipLaunchKernelGGL((k_probe_bin<4, 0>), dim3(grid), dim3(256), 0, 0, d_bins, bin_cap, d_cur, d_slots,
                               d_subs, lists4, d_e, d_loc);
        });
        snprintf(nm, sizeof nm, "probe_bin spread IPT2 grid %d", grid);
        timeit(nm, [&]() {
            hipLaunchKernelGGL((k_probe_bin<2, 1>), dim3(grid), dim3(256), 0, 0, d_bins, bin_cap, d_cur, d_slots,
                               d_subs, lists4, d_e, d_loc);
        });
    }
    timeit("probe_flat IPT2 (message order, one table)", [&]() {
        hipLaunchKernelGGL((k_probe_flat<2>), dim3((M + 511) / 512), dim3(256), 0, 0, d_pos, d_c, d_s, d_r, M,
                           d_fslots, fst, lists4, d_e2, d_loc2);
    });
    timeit("probe_flat IPT4", [&]() {
        hipLaunchKernelGGL((k_probe_flat<4>), dim3((M + 1023) / 1024), dim3(256), 0, 0, d_pos, d_c, d_s, d_r, M,
                           d_fslots, fst, lists4, d_e2, d_loc2);
    });
    // parity of the two probes
    {
        std::vector<uint32_t> e1(M), e2(M);
        CK(hipMemcpy(e1.data(), d_e, 4ull * M, hipMemcpyDeviceToHost));
        CK(hipMemcpy(e2.data(), d_e2, 4ull * M, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint32_t m = 0; m < M; ++m) bad += (e1[m] != e2[m]) || (e1[m] != ex[m + 1] - ex[m]);
        printf("probe parity: %llu mismatches\n", (unsigned long long)bad);
    }
    timeit("emit_lds (gather lists, coalesced copy)", [&]() {
        hipLaunchKernelGGL(k_emit_lds, dim3((M + kEmitMsgs - 1) / kEmitMsgs), dim3(256), 0, 0, d_loc, d_offs, M,
                           lists4, d_op, d_om);
    });
    {
        std::vector<uint32_t> op(P);
        CK(hipMemcpy(op.data(), d_op, 4ull * P, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint32_t m = 0; m < M; m += 97) {
            const uint32_t c = mc[m];
            uint32_t o = ex[m];
            for (uint32_t q = 0; q < cnt[c]; ++q)
                if (lists[off[c] + q] != ms[m]) bad += op[o++] != lists[off[c] + q];
        }
        printf("emit parity (sampled): %llu mismatches\n", (unsigned long long)bad);
    }
    timeit("bin + probe_bin(2048) + emit", [&]() {
        bin();
        hipLaunchKernelGGL((k_probe_bin<2, 0>), dim3(2048), dim3(256), 0, 0, d_bins, bin_cap, d_cur, d_slots, d_subs,
                           lists4, d_e, d_loc);
        hipLaunchKernelGGL(k_emit_lds, dim3((M + kEmitMsgs - 1) / kEmitMsgs), dim3(256), 0, 0, d_loc, d_offs, M,
                           lists4, d_op, d_om);
    });
    printf("write-only floor: %.1f MB out\n", P * 8 / 1e6);
    return 0;
}
