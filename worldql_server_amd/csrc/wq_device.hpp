// wq_device.hpp — device-side building blocks shared by the route and table kernels.
//
//  * coord_clamp_dev: kernel (1), CubeArea::coord_clamp (worldql_server/src/subscriptions/
//    cube_area.rs:23-44) + round_by_multiple (worldql_server/src/utils/round.rs:1-13), bit-exact.
//  * cube_hash: the 64-bit bucket hash of (world, CubeArea). The table is keyed by the FULL key;
//    the hash only places buckets, so hash collisions never change a result.
//  * Slot: one 32-byte open-addressed bucket record in HBM.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace wq {

constexpr uint32_t kWorldEmpty = 0xFFFFFFFFu;  // == WQ_WORLD_INVALID: marks an empty slot
constexpr uint32_t kNone = 0xFFFFFFFFu;

// One bucket: the full cube key, its world, and the offset of its peer list in `list`
// (list[off] = count, list[off+1 .. off+count] = ascending peer ids). 32 bytes, 32-aligned:
// a probe is two 16-byte loads from one 64-byte half line.
struct __attribute__((aligned(32))) Slot {
    int64_t k[3];
    uint32_t world;
    uint32_t off;
};
static_assert(sizeof(Slot) == 32, "Slot must be 32 bytes");

// Rust `f64 as i64`: truncation toward zero, saturating, NaN -> 0 (C's cast is UB out of range).
__host__ __device__ __forceinline__ int64_t sat_i64(double x) {
    if (x != x) return 0;
    if (x >= 9223372036854775808.0) return INT64_MAX;
    if (x <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)x;
}

// cube_area.rs:23-44, release-build semantics (wrapping i64 + and *). The reference's
// `abs % size == 0.0` (an f64 fmod) is replaced by an exact divisibility test that needs no
// fmod loop: a is a multiple of s  <=>  q = a/s is an integer and q*s == a exactly, checked
// with one fused multiply-add (exact residual, never rounds a non-zero residual to 0).
// Both sides of the equivalence are proven in DESIGN.md §Kernel 1; inf/NaN make the test false,
// exactly like fmod's NaN result. q is then reused for ceil(a/s) (round_by_multiple's n/m).
__host__ __device__ __forceinline__ int64_t coord_clamp_dev(double c, double sf, int64_t si) {
    const double a = fabs(c);
    const double q = a / sf;
    const bool is_mult = (q == trunc(q)) && (fma(q, sf, -a) == 0.0) && (c != 0.0);
    if (is_mult) return sat_i64(c);
    const double r = (a == 0.0) ? sf : ceil(q) * sf;  // round_by_multiple(a, s)
    int64_t res = sat_i64(r);
    if (!(r > c)) res = (int64_t)((uint64_t)res + (uint64_t)si);
    return (c < 0.0) ? (int64_t)(0ull - (uint64_t)res) : res;
}

__host__ __device__ __forceinline__ uint64_t cube_hash(uint32_t w, int64_t x, int64_t y, int64_t z) {
    uint64_t h = (uint64_t)x * 0x9E3779B97F4A7C15ull;
    h ^= (uint64_t)y * 0xC2B2AE3D27D4EB4Full;
    h ^= (uint64_t)z * 0x165667B19E3779F9ull;
    h ^= ((uint64_t)w + 0x27D4EB2F165667C5ull) * 0xD6E8FEB86659FD93ull;
    h ^= h >> 32;
    h *= 0xD6E8FEB86659FD93ull;
    h ^= h >> 29;
    h *= 0x94D049BB133111EBull;
    h ^= h >> 32;
    return h;
}

// Slot index from the hash's high bits. shift = 64 - log2(capacity), capacity >= 1024.
__device__ __forceinline__ uint64_t slot_of(uint64_t h, int shift) { return h >> shift; }

struct SlotView {
    int64_t k0, k1, k2;
    uint32_t world, off;
};

__device__ __forceinline__ SlotView load_slot(const Slot* slots, uint64_t i) {
    const uint4* p = reinterpret_cast<const uint4*>(slots + i);
    const uint4 a = p[0];
    const uint4 b = p[1];
    SlotView s;
    s.k0 = (int64_t)(((uint64_t)a.y << 32) | a.x);
    s.k1 = (int64_t)(((uint64_t)a.w << 32) | a.z);
    s.k2 = (int64_t)(((uint64_t)b.y << 32) | b.x);
    s.world = b.z;
    s.off = b.w;
    return s;
}

// Linear-probe lookup of (w, k). Returns the list offset or kNone. The table always keeps at
// least half its slots empty, so the walk ends at an empty slot.
__device__ __forceinline__ uint32_t probe(const Slot* slots, uint64_t mask, int shift, uint64_t h,
                                          uint32_t w, int64_t x, int64_t y, int64_t z) {
    uint64_t i = slot_of(h, shift);
    for (;;) {
        const SlotView s = load_slot(slots, i);
        if (s.world == kWorldEmpty) return kNone;
        if (s.world == w && s.k0 == x && s.k1 == y && s.k2 == z) return s.off;
        i = (i + 1) & mask;
    }
}

// First index in sorted a[0..n) with a[i] >= v.
template <typename T>
__device__ __forceinline__ uint32_t lower_bound_dev(const T* a, uint32_t n, T v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

}  // namespace wq
