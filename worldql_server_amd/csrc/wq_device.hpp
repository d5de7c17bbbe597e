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
// Branch-free (selects only), so the compiler can keep a wave's loads in flight across it.
__host__ __device__ __forceinline__ int64_t sat_i64(double x) {
    const bool nan = x != x;
    const bool hi = x >= 9223372036854775808.0;
    const bool lo = x <= -9223372036854775808.0;
    const double t = (nan | hi | lo) ? 0.0 : x;  // in range: the cast below is defined
    int64_t v = (int64_t)t;
    v = hi ? INT64_MAX : v;
    v = lo ? INT64_MIN : v;
    return v;
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
    // exact multiple (and not +-0): the reference returns `c as i64` (cube_area.rs:30-32)
    const bool is_mult = (q == trunc(q)) && (fma(q, sf, -a) == 0.0) && (c != 0.0);
    const double r = (a == 0.0) ? sf : ceil(q) * sf;  // round_by_multiple(a, s)
    int64_t res = sat_i64(is_mult ? c : r);
    const bool add = !is_mult & !(r > c);             // `if r > c {r} else {r + size}`, wrapping
    res = add ? (int64_t)((uint64_t)res + (uint64_t)si) : res;
    const bool neg = !is_mult & (c < 0.0);            // `* mult`, wrapping
    return neg ? (int64_t)(0ull - (uint64_t)res) : res;
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

// Owner of a bucket. Decorrelated from rec_hash / the slot hash (both use cube_hash directly), so
// a shard's local table still spreads over all of its slots. Never affected by hash_bits.
__host__ __device__ __forceinline__ uint32_t shard_of(uint32_t w, int64_t x, int64_t y, int64_t z, uint32_t G) {
    uint64_t v = cube_hash(w, x, y, z);
    v ^= v >> 31;
    v *= 0xBF58476D1CE4E5B9ull;
    v ^= v >> 29;
    return (uint32_t)(((v >> 32) * (uint64_t)G) >> 32);
}

// ---- bucket records (the table the hot path probes) --------------------------------------
// A "regular" cube — world < 2^24 - 1 and every key coordinate an exact multiple k = a*s of the
// cube size with a in [-2^23, 2^23) — has an exact 96-bit packed key
//   V = (world + 1) << 72 | (ax + 2^23) << 48 | (ay + 2^23) << 24 | (az + 2^23)
// held as pk = V mod 2^64 (header words 0-1) and ext = V >> 64 (word 7). ext is never 0 for a key
// (world + 1 >= 1), so ext == 0 marks an empty record. Every key a Vector3 can produce within
// +-2^23 cubes of the origin (+-134M units at the default cube_size 16, far past Minecraft's
// +-3e7) in any of 16M worlds is regular.
// Regular cubes live in 128-byte records (one cache line: one fabric request per lookup):
//   chunk 0 (bytes 0-15)   pk, peer count, offset of the cube's full list in `list`
//   chunk 1 (16-31)        sig: 64-bit Bloom signature of the cube's peers (peer_sig), the list
//                          block's capacity, ext
//   chunks 2-7 (32-127)    p0 .. p23, four per chunk
// so peer i sits in word 8 + i: output quad q of a message without a skipped sender is chunk
// 2 + q verbatim (route_emit.hpp). The count pass reads chunks 0-1 (key, count, signature) in its
// first round (route_count.hpp).
// Everything else (raw off-grid keys, NaN/inf/saturated coordinates, the last world ids) lives in
// the 32-byte full-key Slot table. Both tables are exact; a key is in exactly one of them.
constexpr int kInline = 24;
constexpr int kInlineWord0 = 8;
constexpr int kAxisBits = 24;
constexpr uint32_t kAxisBias = 1u << (kAxisBits - 1);
constexpr uint32_t kAxisMask = (1u << kAxisBits) - 1u;
constexpr uint32_t kMaxPackedWorld = (1u << 24) - 2u;  // world + 1 must fit 24 bits

struct __attribute__((aligned(128))) Record {
    uint64_t pk;       // low 64 bits of the packed key
    uint32_t count;    // peers subscribed to the cube
    uint32_t list_off; // list[list_off] = count, list[list_off+1 ..] = ascending peers
    uint64_t sig;      // OR of peer_sig over the cube's peers
    uint32_t cap;      // capacity (peers) of the cube's list block
    uint32_t ext;      // high 32 bits of the packed key; 0 = empty record
    uint32_t peers[kInline];  // the first min(count, kInline) peers, ascending; rest 0xFFFFFFFF
};
// Two of the 64 signature bits per peer (one multiply): with ~10 peers per cube about 7% of
// non-subscribed senders pass the test and are verified against the list; none is missed.
__host__ __device__ __forceinline__ uint64_t peer_sig(uint32_t peer) {
    const uint32_t h = peer * 0x9E3779B1u;
    return (1ull << (h >> 26)) | (1ull << ((h >> 20) & 63u));
}
static_assert(sizeof(Record) == 128, "Record must be one 128-byte line");
// Capacity (peers) a list gets when the table is built: 25% headroom plus 2, so the incremental
// update (wq_delta.hip) edits most churned lists in place.
__host__ __device__ __forceinline__ uint32_t list_capacity(uint32_t count) { return count + count / 4 + 2; }

__host__ __device__ __forceinline__ bool pack_key(uint32_t w, int64_t x, int64_t y, int64_t z, double sf,
                                                  uint64_t* pk, uint32_t* ext) {
    if (w > kMaxPackedWorld) return false;
    const int64_t k[3] = {x, y, z};
    uint64_t a[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        // |k| < 2^40: exact in f64; with |k/s| < 2^23 the quotient's ulp is <= 2^-29, far below the
        // >= 2^-16 distance of a non-multiple's k/s from an integer, so k/s is an integer iff the
        // rounded quotient is
        if (k[d] <= -(1ll << 40) || k[d] >= (1ll << 40)) return false;
        const double q = (double)k[d] / sf;
        if (q != trunc(q) || q < -(double)kAxisBias || q >= (double)kAxisBias) return false;
        a[d] = (uint64_t)((int64_t)q + (int64_t)kAxisBias);
    }
    *pk = (a[0] << 48) | (a[1] << 24) | a[2];
    *ext = ((w + 1u) << 8) | (uint32_t)(a[0] >> 16);
    return true;
}

// coord_clamp_dev on the three coordinates and pack_key on the key, in one pass, with the same
// results for every input (tests/test_quantize_pack.py checks it against the two functions). For a
// finite coordinate with n = |c| / s (an exact multiple) or ceil(|c| / s) [+ 1] at most 2^23 + 2
// and a cube size below 2^29, every product is exact and the key is n s with the sign of c: the key
// and pack_key's biased axis n + 2^23 come from n in integer arithmetic, and k / s = n exactly is
// pack_key's integer test. That skips, per axis, the saturating f64 -> i64 conversion, pack_key's
// second division and its conversion. Anything else (NaN, inf, huge coordinates or cube sizes)
// takes coord_clamp_dev and pack_key themselves. Used by the slot grouping (wq_shard.hip), whose
// quantisation is VALU-bound; in the route tick's count it made C2 slower.
__host__ __device__ __forceinline__ bool quantize_pack(uint32_t w, const double (&c)[3], double sf, int64_t si,
                                                       int64_t (&k)[3], uint64_t* pk, uint32_t* ext) {
    bool fast = si >= 1 && si < (1ll << 29), ok = w <= kMaxPackedWorld;
    uint64_t a[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const double x = c[d], ax = fabs(x), q = ax / sf;
        const bool is_mult = (q == trunc(q)) && (fma(q, sf, -ax) == 0.0) && (x != 0.0);
        const double cq = (ax == 0.0) ? 1.0 : ceil(q);
        const bool add = !is_mult & !(cq * sf > x);
        const double nd = is_mult ? q : cq + (add ? 1.0 : 0.0);
        const bool f = nd <= 8388610.0;  // 2^23 + 2; false for NaN
        fast = fast && f;
        const int64_t n_abs = (int64_t)(int32_t)(f ? nd : 0.0);
        const int64_t n = x < 0.0 ? -n_abs : n_abs;
        k[d] = n * si;
        ok = ok && n >= -(int64_t)kAxisBias && n < (int64_t)kAxisBias && k[d] > -(1ll << 40) && k[d] < (1ll << 40);
        a[d] = (uint64_t)(n + (int64_t)kAxisBias);
    }
    if (!fast) {
#pragma unroll
        for (int d = 0; d < 3; ++d) k[d] = coord_clamp_dev(c[d], sf, si);
        return pack_key(w, k[0], k[1], k[2], sf, pk, ext);
    }
    if (ok) {  // (pack_key writes nothing for an irregular key either)
        *pk = (a[0] << 48) | (a[1] << 24) | a[2];
        *ext = ((w + 1u) << 8) | (uint32_t)(a[0] >> 16);
    }
    return ok;
}

// The packed key's world and biased axes (a_d = k_d / s + 2^23).
__host__ __device__ __forceinline__ void unpack_key(uint64_t pk, uint32_t ext, uint32_t* w, uint32_t* a) {
    *w = (ext >> 8) - 1u;
    a[0] = ((ext & 0xFFu) << 16) | (uint32_t)(pk >> 48);
    a[1] = (uint32_t)(pk >> 24) & kAxisMask;
    a[2] = (uint32_t)pk & kAxisMask;
}

__host__ __device__ __forceinline__ uint64_t rec_hash(uint64_t pk, uint32_t ext) {
    uint64_t h = pk ^ ((uint64_t)ext * 0xD6E8FEB86659FD93ull);
    h ^= h >> 31;
    h *= 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h;
}

// Slot index from the hash's high bits. shift = 64 - log2(capacity), capacity >= 1024.
__device__ __forceinline__ uint64_t slot_of(uint64_t h, int shift) { return h >> shift; }

// Home slot of a cube in the compact header table. blk = 0: the cube's own hash. blk = 4 / 8: the
// cube's 2 x 2 (y, z) / 2 x 2 x 2 block hashes to a group of blk consecutive slots and the cube takes
// slot (x, y, z low bits) of it, so neighbouring cubes share header lines (4 32-B headers per line).
__device__ __forceinline__ uint64_t hdr_home(uint64_t pk, uint32_t ext, uint64_t hash_mask, int shift, uint32_t blk) {
    if (!blk) return slot_of(rec_hash(pk, ext) & hash_mask, shift);
    const uint64_t sub = ((pk >> 48) & 1ull) << 2 | ((pk >> 24) & 1ull) << 1 | (pk & 1ull);
    const uint64_t low = blk == 8 ? (1ull << 48) | (1ull << 24) | 1ull : (1ull << 24) | 1ull;
    return (slot_of(rec_hash(pk & ~low, ext) & hash_mask, shift) & ~(uint64_t)(blk - 1)) | (sub & (blk - 1));
}

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

struct TableView {
    const Record* recs;
    uint64_t rec_mask;
    int rec_shift;
    const Slot* slots;
    uint64_t slot_mask;
    int slot_shift;
    uint64_t hash_mask;
    const uint32_t* list;
    double sf;
    // C5 radius filter (wq_set_radius): peer positions (n_ppos x 3) and r^2; r2 < 0: off
    const double* ppos;
    const float4* ppos4;  // the same positions rounded to f32 {x, y, z, 0}: the second, exact-or-defer test
    // the first test: 4 bytes per peer (4 MB for C5's 1M entities, mostly L2-resident, where the f32
    // rows take 16 MB): x, y on 11 bits and z on 10 over the positions' bounding box (kQNone: no code)
    const uint32_t* pcode;
    const double* qbox;   // {lo x, lo y, lo z, step x, step y, step z} of the codes
    uint32_t n_ppos;
    double r2;
    // per-peer boxes of the record cubes each peer is subscribed to (PeerBox); nullptr: none
    const uint32_t* pbox;
    uint32_t n_pbox;            // peers [0, n_pbox) have a box; others hold no record cube
    const uint32_t* pbox_valid; // device word: 0 once an update could not keep the boxes
    const uint32_t* stale;      // device word: non-zero while an incremental batch awaits re-application
    // dense copy of every record's first 32 bytes (key, count, list offset, signature) at the same
    // slot index, 4 per 128-B line; nullptr: the count pass probes the records themselves
    const uint4* hdr = nullptr;
    // hdr_mask != 0: the headers are a COMPACT table of their own (load <= 1/2, 4 per line, so the hot
    // cubes of a tick share lines and the table is 1/8 of the records' size): a cube's header is found
    // by linear probing from slot_of(hash, hdr_shift), and its word 6 holds the cube's record slot
    // (the record's cap, which no tick reads). hdr_mask == 0: header i is record i's.
    uint64_t hdr_mask = 0;
    int hdr_shift = 64;
    uint32_t hdr_blk = 0;  // hdr_home's block grouping (0: per-cube hashing)
};

// ---- per-peer boxes: a fast "certainly not subscribed" for long lists ---------------------
// For every peer, the [min, max] world and the per-axis [min, max] of the packed axes (pack_key)
// of the record cubes it is subscribed to: 8 words {world_min, world_max, a0_min, a0_max | a1_min,
// a1_max, a2_min, a2_max} (empty: every min 0xFFFFFFFF, every max 0). A message whose cube lies
// outside its sender's box cannot have the sender among the cube's peers, so the count pass skips
// the binary search of a long list (C3: random senders in hotspot cubes of ~500 peers — ~0.8
// extra line per message). Built with the table; unsubscribes and disconnects leave boxes wider
// than needed, which is still exact ("maybe" -> the search decides); an incremental batch turns
// them off (valid word 0) until the next build. A peer with record cubes in several worlds gets
// the world-range test only. The test reads the box's first half (world, axis 0) and only then
// the second: few registers live in the count pass's probe loop.
constexpr int kBoxWords = 8;

__device__ __forceinline__ void box_add(uint32_t* box, uint64_t pk, uint32_t ext) {
    uint32_t w, a[3];
    unpack_key(pk, ext, &w, a);
    atomicMin(&box[0], w);
    atomicMax(&box[1], w);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        atomicMin(&box[2 + 2 * d], a[d]);
        atomicMax(&box[3 + 2 * d], a[d]);
    }
}

// false: `peer` is certainly not subscribed to the record cube (pk, ext).
__device__ __forceinline__ bool box_may_hold(const TableView& t, uint32_t peer, uint64_t pk, uint32_t ext) {
    if (peer >= t.n_pbox) return false;
    const uint4* b = reinterpret_cast<const uint4*>(t.pbox + (uint64_t)kBoxWords * peer);
    const uint4 lo = b[0];
    const uint32_t w = (ext >> 8) - 1u;
    if (w < lo.x || w > lo.y) return false;  // also: no record cube at all (min > max)
    if (lo.x != lo.y) return true;            // several worlds: the world range is all we know
    const uint32_t a0 = ((ext & 0xFFu) << 16) | (uint32_t)(pk >> 48);
    if (a0 < lo.z || a0 > lo.w) return false;
    const uint4 hi = b[1];
    const uint32_t a1 = (uint32_t)(pk >> 24) & kAxisMask, a2 = (uint32_t)pk & kAxisMask;
    return a1 >= hi.x && a1 <= hi.y && a2 >= hi.z && a2 <= hi.w;
}

// C5: is peer p within the radius of message position (mx, my, mz)? f64, left to right, no FMA
// (this file is compiled with contraction off), a peer without a position never is.
// First from the f32 copy of the position (one aligned 16-byte load instead of 24 bytes that
// straddle a cache line one time in five): with pf = (double)(float)p, |p - pf| <= |pf| 2^-23 (plus
// 2^-120 below f32's normal range), so the reference's dx = fl(mx - px) is within
// e = |pf| 2^-23 + 2^-120 + |ax| 2^-50 of ax = fl(mx - pf), its square within e (2|ax| + e) of ax^2,
// and its three roundings add at most 2^-50 (d2 + E1). Only when the exact d2 could lie on either
// side of r^2 (or a value is NaN / beyond f32) are the f64 coordinates read.
// The f32 test alone: 1 = certainly within, 0 = certainly not, -1 = read the f64 coordinates.
__device__ __forceinline__ int radius_f32_test(const float4 f, double mx, double my, double mz, double r2) {
    const double ax = mx - (double)f.x, ay = my - (double)f.y, az = mz - (double)f.z;
    const double d2f = ax * ax + ay * ay + az * az;
    const double ex = fabs((double)f.x) * 0x1p-23 + 0x1p-120 + fabs(ax) * 0x1p-50;
    const double ey = fabs((double)f.y) * 0x1p-23 + 0x1p-120 + fabs(ay) * 0x1p-50;
    const double ez = fabs((double)f.z) * 0x1p-23 + 0x1p-120 + fabs(az) * 0x1p-50;
    const double E1 = ex * (2.0 * fabs(ax) + ex) + ey * (2.0 * fabs(ay) + ey) + ez * (2.0 * fabs(az) + ez);
    const double E = E1 * 1.001 + d2f * 0x1p-40 + 0x1p-1000;
    if (d2f + E <= r2) return 1;   // NaN: false
    if (d2f - E > r2) return 0;    // NaN: false
    return -1;
}

// The reference's f64 predicate itself (peer p has a position).
__device__ __forceinline__ bool radius_f64(const TableView& t, double mx, double my, double mz, uint32_t p) {
    const double* q = t.ppos + 3ull * p;
    const double dx = mx - q[0];
    const double dy = my - q[1];
    const double dz = mz - q[2];
    const double d2 = dx * dx + dy * dy + dz * dz;
    return d2 <= t.r2;
}

// ---- the 4-byte position codes (the radius filter's first test) ----
// code = ux | uy << 11 | uz << 22 with u_d = rint((p_d - lo_d) / step_d), steps = extent / 2047
// (x, y) and / 1022 (z, so no code is all ones): the decoded q_d = lo_d + u_d * step_d (f64) lies
// within e_d = step_d / 2 (1 + 2^-40) + (|lo_d| + |q_d| + u_d step_d) 2^-49 of p_d — the rounding of
// the division, of rint's argument and of the decode are all inside that margin. Peers without a
// finite position get kQNone and go to the f32 / f64 tests.
constexpr uint32_t kQNone = 0xFFFFFFFFu;
constexpr uint32_t kQMaxXY = 2047u, kQMaxZ = 1022u;

__device__ __forceinline__ uint32_t pos_code(double x, double y, double z, const double* box) {
    if (!(isfinite(x) && isfinite(y) && isfinite(z))) return kQNone;
    const double u[3] = {rint((x - box[0]) / box[3]), rint((y - box[1]) / box[4]), rint((z - box[2]) / box[5])};
    const double mx[3] = {(double)kQMaxXY, (double)kQMaxXY, (double)kQMaxZ};
    uint32_t q[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const double c = u[d] < 0.0 ? 0.0 : (u[d] > mx[d] ? mx[d] : u[d]);
        q[d] = (uint32_t)c;
    }
    return q[0] | (q[1] << 11) | (q[2] << 22);
}

// The code test: 1 = certainly within r, 0 = certainly not, -1 = ask the f32 / f64 tests. With
// the decoded q, a = m - q is within e of the reference's dx = fl(m - p) (plus that subtraction's
// rounding), so as in radius_f32_test the reference's f64 d2 lies within E of fl(a.a).
__device__ __forceinline__ int radius_code_test(uint32_t code, const double* box, double mx, double my, double mz,
                                                double r2) {
    if (code == kQNone) return -1;
    const uint32_t u[3] = {code & kQMaxXY, (code >> 11) & kQMaxXY, code >> 22};
    const double m[3] = {mx, my, mz};
    double d2 = 0.0, E1 = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const double ud = (double)u[d];
        const double q = box[d] + ud * box[3 + d];
        const double a = m[d] - q;
        const double e = box[3 + d] * 0.5 * (1.0 + 0x1p-40) + (fabs(box[d]) + fabs(q) + ud * box[3 + d]) * 0x1p-49 +
                         fabs(a) * 0x1p-50 + 0x1p-1000;
        d2 += a * a;
        E1 += e * (2.0 * fabs(a) + e);
    }
    const double E = E1 * 1.001 + d2 * 0x1p-40 + 0x1p-1000;
    if (d2 + E <= r2) return 1;  // NaN (a message without a finite position): false
    if (d2 - E > r2) return 0;
    return -1;
}

__device__ __forceinline__ bool within_radius(const TableView& t, double mx, double my, double mz, uint32_t p) {
    if (p >= t.n_ppos) return false;
    if (t.pcode) {
        const int c = radius_code_test(t.pcode[p], t.qbox, mx, my, mz, t.r2);
        if (c >= 0) return c > 0;
    }
    const int d = radius_f32_test(t.ppos4[p], mx, my, mz, t.r2);
    return d >= 0 ? d > 0 : radius_f64(t, mx, my, mz, p);
}

// Header (chunks 0-1) of the record probe sequence for (pk, ext): walks while the slot holds
// another key; an empty record (ext == 0) ends it.
__device__ __forceinline__ uint64_t find_record(const TableView& t, uint64_t pk, uint32_t ext, uint4* h0, uint4* h1) {
    uint64_t i = slot_of(rec_hash(pk, ext) & t.hash_mask, t.rec_shift);
    for (;;) {
        const uint4 a = *reinterpret_cast<const uint4*>(t.recs + i);
        const uint4 b = *(reinterpret_cast<const uint4*>(t.recs + i) + 1);
        const uint64_t k = ((uint64_t)a.y << 32) | a.x;
        if (b.w == 0 || (k == pk && b.w == ext)) {
            *h0 = a;
            *h1 = b;
            return i;
        }
        i = (i + 1) & t.rec_mask;
    }
}

// The cube's peers, ascending: a record cube with <= kInline peers keeps them only in its
// record's inline words (its `list` block, if any, is stale: wq_delta.hip); longer record lists
// and slot-table cubes are in `list`. *n = 0 when the cube has no peers.
__device__ __forceinline__ const uint32_t* find_peers(const TableView& t, uint32_t w, int64_t x, int64_t y, int64_t z,
                                                      uint32_t* n) {
    uint64_t pk;
    uint32_t ext;
    *n = 0;
    if (pack_key(w, x, y, z, t.sf, &pk, &ext)) {
        uint4 h0, h1;
        const uint64_t i = find_record(t, pk, ext, &h0, &h1);
        if (!h1.w || !h0.z) return t.list;
        *n = h0.z;
        return h0.z <= (uint32_t)kInline ? t.recs[i].peers : t.list + h0.w + 1;
    }
    const uint32_t off = probe(t.slots, t.slot_mask, t.slot_shift, cube_hash(w, x, y, z) & t.hash_mask, w, x, y, z);
    if (off == kNone) return t.list;
    *n = t.list[off];
    return t.list + off + 1;
}

// Offset of the cube's list in t.list, or kNone (both tables).
__device__ __forceinline__ uint32_t find_list(const TableView& t, uint32_t w, int64_t x, int64_t y, int64_t z) {
    uint64_t pk;
    uint32_t ext;
    if (pack_key(w, x, y, z, t.sf, &pk, &ext)) {
        uint4 h0, h1;
        find_record(t, pk, ext, &h0, &h1);
        return h1.w ? h0.w : kNone;
    }
    return probe(t.slots, t.slot_mask, t.slot_shift, cube_hash(w, x, y, z) & t.hash_mask, w, x, y, z);
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
