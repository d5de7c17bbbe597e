// wq_delta.hip — incremental subscribe / unsubscribe batches (SURVEY.md §8(d) C4 churn) and
// REMOVE_PEER in place (§8(f) F3).
//
// Same semantics as the full rebuild in wq_table.hip — per (world, cube, peer) the last op of the
// batch wins (AreaMap::add_subscription / remove_subscription, area_map.rs:72-119, applied in
// order by thread.rs:122-146) — but the work is proportional to the batch and the cubes it
// touches, not to the whole table. The group path (default):
//   events   each op -> packed cube key and its record slot (a new cube claims its record here by
//            CAS on the probe path, count 0), and a value kind << 32 | peer
//   sort     one stable radix sort of the values by slot over log2(capacity) bits: every cube's
//            ops are contiguous and in op order
//   plan     one lane per touched cube reads the record header and reserves relocation space for
//            old count + subscribes beyond the list's capacity (one host read-back of the totals)
//   apply    16 lanes per cube merge the cube's ops (16 at a time, sorted by (peer, op) in
//            registers, last op of a peer wins) into its list staged in LDS, then write the list
//            (in place, or relocated past the used part of `list` with 50% headroom) and the whole
//            record line (count, offset, capacity, Bloom signature, inline peers)
// Cubes beyond the group bounds (old count + ops > 128) send the batch to the per-lane path:
// sort by (slot, peer), one lane per cube, in-place forward compaction then backward merge.
// A cube that empties keeps its record (count 0, key kept), so every probe sequence stays intact.
// The sorted state `st` and the any-keys are left stale and regenerated from the records only
// when something needs them (table_materialize / table_ensure_any). A batch falls back to the full
// rebuild (no list changed) when an op is not regular, relocations would overflow `list`, or the
// record table would pass load 1/4.
#include <algorithm>

#include "table_prims.hpp"

namespace wq {

namespace {

struct DeltaSummary {
    uint64_t d_entries;    // two's complement: adds - removes
    uint64_t d_live;       // two's complement: cubes that became non-empty - cubes that emptied
    uint64_t n_big;        // touched cubes too large for the wave path (lists > kWaveOld, > kWaveCh changes)
    uint64_t reloc_words;  // list words to bump-allocate
    uint64_t new_recs;     // records claimed by this batch's new cubes
    uint32_t irregular;    // 1: an op without a packed key; 2: an invalid op (device batches)
    uint32_t n_dc;         // touched cubes
};

struct DeltaTable {
    Record* recs;
    uint32_t* rclaim;
    uint64_t rmask;
    int rshift;
    uint64_t hmask;
    uint32_t* list;
};

__device__ __forceinline__ void op_key(const wq_op& o, double sf, int64_t si, int64_t* k) {
    if (o.key_is_raw) {  // impl ToCubeArea for CubeArea: identity (cube_area.rs:65-70)
        k[0] = o.u.key[0];
        k[1] = o.u.key[1];
        k[2] = o.u.key[2];
    } else {  // CubeArea::from_vector3 (cube_area.rs:50-56)
        k[0] = coord_clamp_dev(o.u.pos[0], sf, si);
        k[1] = coord_clamp_dev(o.u.pos[1], sf, si);
        k[2] = coord_clamp_dev(o.u.pos[2], sf, si);
    }
}

// Per op: packed key, and the record slot of its cube — a cube the table does not hold yet gets
// its record here (key claimed by compare-and-swap on the probe path, count 0), so the batch can
// be grouped by slot with a short radix sort. The caller guarantees free slots (load <= 1/2).
// Claim words (rclaim, one per record slot): 0 free, kClaiming while an op writes a new cube's key,
// otherwise the slot holds a key — builds write the cube index + 2 (< 2^31), a delta batch writes
// its tag (kBatchTag | batch number). The 96-bit key spans two words of the record, so a slot is
// claimed through its claim word: the winner writes the key, then publishes the tag (release). A
// key published before this launch is read with plain loads; only a slot tagged by this very
// batch takes an acquire fence first (the one case where the key may still be in flight). An op
// that finds a slot being claimed looks again (the winner's wave progresses meanwhile).
constexpr uint32_t kClaiming = 1u, kBatchTag = 0x80000000u;

__global__ void k_delta_events(const wq_op* __restrict__ ops, uint32_t n, double sf, int64_t si, Record* recs,
                               uint32_t* rclaim, uint32_t tag, uint64_t rmask, int rshift, uint64_t hmask,
                               uint32_t* slot, uint32_t* peer, uint8_t* kind, uint64_t* sv, DeltaSummary* sum) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const wq_op o = ops[i];
    int64_t k[3];
    op_key(o, sf, si, k);
    uint64_t p = 0;
    uint32_t x = 0;
    uint32_t sl = 0;  // ops without a record (the batch then falls back): slot 0, an in-bounds dummy
    if (o.kind > WQ_OP_UNSUBSCRIBE || o.world == WQ_WORLD_INVALID) {
        atomicOr(&sum->irregular, 2u);  // bad op
    } else if (!pack_key(o.world, k[0], k[1], k[2], sf, &p, &x)) {
        atomicOr(&sum->irregular, 1u);
    } else {
        uint64_t j = slot_of(rec_hash(p, x) & hmask, rshift);
        for (;;) {
            uint32_t c = __hip_atomic_load(&rclaim[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c == 0) {
                c = atomicCAS(&rclaim[j], 0u, kClaiming);
                if (c == 0) {  // won: a new cube (count 0) with this key
                    recs[j].pk = p;
                    recs[j].ext = x;
                    __hip_atomic_store(&rclaim[j], tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    atomicAdd(reinterpret_cast<unsigned long long*>(&sum->new_recs), 1ull);
                    break;
                }
            }
            if (c == kClaiming) continue;  // being claimed: look again
            uint64_t rp;
            uint32_t rx;
            if (c == tag) {  // claimed by this batch: order the key loads after the tag
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                rp = __hip_atomic_load(&recs[j].pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                rx = __hip_atomic_load(&recs[j].ext, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                rp = recs[j].pk;
                rx = recs[j].ext;
            }
            if (rp == p && rx == x) break;
            j = (j + 1) & rmask;
        }
        sl = (uint32_t)j;
    }
    const uint32_t kd = o.kind == WQ_OP_SUBSCRIBE ? 1u : 0u;
    slot[i] = sl;
    peer[i] = o.peer;
    kind[i] = (uint8_t)kd;
    sv[i] = ((uint64_t)kd << 32) | o.peer;  // sorted along with the slot: no gather afterwards
}

// Sorted order -> peer / kind columns and cube heads.
__global__ void k_delta_mark(const uint32_t* __restrict__ order, const uint32_t* __restrict__ spk,
                             const uint32_t* __restrict__ peer, const uint8_t* __restrict__ kind, uint32_t n,
                             uint32_t* sp, uint8_t* skd, uint32_t* head) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = order[i];
    sp[i] = peer[a];
    skd[i] = kind[a];
    head[i] = (i == 0 || spk[i] != spk[i - 1]) ? 1u : 0u;
}

__global__ void k_delta_cubes(const uint32_t* __restrict__ head, const uint32_t* __restrict__ cid, uint32_t n,
                              uint32_t* cube_start, DeltaSummary* sum) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (head[i]) cube_start[cid[i] - 1] = i;
    if (i == n - 1) {
        sum->n_dc = cid[i];
        cube_start[cid[i]] = n;
    }
}

// Last index of the (cube, peer) run starting at t.
__device__ __forceinline__ uint32_t run_last(const uint32_t* sp, uint32_t t, uint32_t s1) {
    while (t + 1 < s1 && sp[t + 1] == sp[t]) ++t;
    return t;
}

__device__ __forceinline__ uint32_t grown(uint32_t n) { return n + n / 2 + 4; }

__global__ __launch_bounds__(kBlock) void k_delta_plan(DeltaTable tb, const uint32_t* __restrict__ cube_start,
                                                       const uint32_t* __restrict__ sslot,
                                                       const uint32_t* __restrict__ sp,
                                                       const uint8_t* __restrict__ skd, const DeltaSummary* sum,
                                                       uint32_t n, uint4* plan, uint32_t* reloc, uint64_t* part) {
    __shared__ unsigned long long acc[4];
    if (threadIdx.x < 4) acc[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t n_dc = sum->n_dc;
    uint32_t rw = 0;
    if (c < n_dc) {
        const uint32_t s0 = cube_start[c], s1 = cube_start[c + 1];
        const uint32_t slot = sslot[s0];  // k_delta_events gave every cube of the batch its record
        const Record& r = tb.recs[slot];
        const uint32_t oc = r.count, off = r.list_off, cap = r.cap;
        const uint32_t* old = tb.list + off + 1;
        uint32_t adds = 0, rms = 0, j = 0;
        for (uint32_t t = s0; t < s1;) {
            const uint32_t l = run_last(sp, t, s1);
            const uint32_t q = sp[l];
            while (j < oc && old[j] < q) ++j;
            const bool present = j < oc && old[j] == q;
            if (skd[l])
                adds += present ? 0u : 1u;
            else
                rms += present ? 1u : 0u;
            t = l + 1;
        }
        const uint32_t nc = oc + adds - rms;
        const bool changed = (adds | rms) != 0;
        if (changed && nc > cap) rw = 1 + grown(nc);
        plan[c] = make_uint4(slot, nc, changed ? 1u : 0u, oc);
        const int64_t de = (int64_t)adds - (int64_t)rms;
        const int64_t dl = (int64_t)(oc == 0 && nc > 0) - (int64_t)(oc > 0 && nc == 0);
        if (de) atomicAdd(&acc[0], (unsigned long long)de);
        if (dl) atomicAdd(&acc[1], (unsigned long long)dl);
        if (rw) atomicAdd(&acc[3], (unsigned long long)rw);
    }
    if (c < n) reloc[c] = rw;
    __syncthreads();
    if (threadIdx.x < 4) part[4ull * blockIdx.x + threadIdx.x] = acc[threadIdx.x];
}

__global__ __launch_bounds__(kBlock) void k_delta_reduce(const uint64_t* __restrict__ part, uint32_t nb,
                                                         DeltaSummary* sum) {
    __shared__ unsigned long long acc[4];
    if (threadIdx.x < 4) acc[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long v[4] = {0, 0, 0, 0};
    for (uint32_t b = threadIdx.x; b < nb; b += kBlock)
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += part[4ull * b + k];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (v[k]) atomicAdd(&acc[k], v[k]);
    __syncthreads();
    if (threadIdx.x == 0) {
        sum->d_entries = acc[0];
        sum->d_live = acc[1];
        sum->n_big = acc[2];
        sum->reloc_words = acc[3];
    }
}

__global__ __launch_bounds__(kBlock) void k_delta_apply(DeltaTable tb, const uint32_t* __restrict__ cube_start,
                                                        const uint32_t* __restrict__ sp,
                                                        const uint8_t* __restrict__ skd, const DeltaSummary* sum,
                                                        const uint4* __restrict__ plan,
                                                        const uint32_t* __restrict__ reloc,
                                                        const uint32_t* __restrict__ reloc_off, uint64_t list_base) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= sum->n_dc) return;
    const uint4 pl = plan[c];
    if (!pl.z) return;
    const uint32_t s0 = cube_start[c], s1 = cube_start[c + 1];
    const uint32_t nc = pl.y, oc = pl.w;
    uint64_t slot = pl.x;
    uint32_t off = 0, cap = 0;
    if (pl.x == kNone) return;  // unreachable: k_delta_events gave every cube of the batch a record
    off = tb.recs[slot].list_off;
    cap = tb.recs[slot].cap;
    uint32_t* L = tb.list;
    if (reloc[c]) {  // forward merge of the old list and the changes into new space
        const uint32_t dst = (uint32_t)(list_base + reloc_off[c]);
        const uint32_t* old = L + off + 1;
        uint32_t* out = L + dst + 1;
        uint32_t i = 0, w = 0, t = s0;
        while (i < oc || t < s1) {
            if (t < s1) {
                const uint32_t l = run_last(sp, t, s1);
                const uint32_t q = sp[l];
                while (i < oc && old[i] < q) out[w++] = old[i++];
                const bool present = i < oc && old[i] == q;
                if (present) ++i;
                if (skd[l]) out[w++] = q;  // subscribed after the batch (kept or added)
                t = l + 1;
            } else {
                out[w++] = old[i++];
            }
        }
        off = dst;
        cap = reloc[c] - 1;
    } else {  // in place: compact the removals forward, then merge the adds backward
        uint32_t* a = L + off + 1;
        uint32_t w = 0, t = s0;
        for (uint32_t i = 0; i < oc; ++i) {
            const uint32_t x = a[i];
            while (t < s1 && sp[t] < x) t = run_last(sp, t, s1) + 1;
            bool rm = false;
            if (t < s1 && sp[t] == x) rm = skd[run_last(sp, t, s1)] == 0;
            if (!rm) a[w++] = x;
        }
        int64_t i = (int64_t)w - 1;
        uint32_t k = nc;
        for (int64_t u = (int64_t)s1 - 1; u >= (int64_t)s0;) {
            const uint32_t q = sp[u];
            const bool sub = skd[u] != 0;  // u is the last op of its run
            while (u >= (int64_t)s0 && sp[u] == q) --u;
            if (!sub) continue;
            while (i >= 0 && a[i] > q) a[--k] = a[i--];
            if (i >= 0 && a[i] == q) continue;  // already subscribed
            a[--k] = q;
        }
    }
    L[off] = nc;
    const uint32_t* a = L + off + 1;
    uint64_t sig = 0;
    for (uint32_t j = 0; j < nc; ++j) sig |= peer_sig(a[j]);
    Record& r = tb.recs[slot];  // the key (pk, ext) stays as claimed
    r.count = nc;
    r.list_off = off;
    r.sig = sig;
    r.cap = cap;
#pragma unroll 4
    for (int j = 0; j < kInline; ++j) r.peers[j] = (uint32_t)j < nc ? a[j] : kNone;
}

// ---- the group path: 16 lanes per touched cube ------------------------------------------------
// The batch is grouped by record slot (one radix sort over log2(capacity) bits). A light plan reads
// only each touched cube's record header and reserves relocation space for an upper bound (old
// count + changes). Then a group of 16 lanes per cube stages the list in LDS (old count + changes
// <= kGroupList), takes the cube's changes in op order 16 at a time, sorts each chunk by (peer, op)
// with a bitonic network in registers (the last op of a peer wins within the chunk, chunks apply in
// order), merges adds and removes into the other LDS buffer by rank, and finally writes the list
// and the record line with coalesced stores. A batch holding a cube beyond the bound takes the
// per-lane path above.
constexpr int kG = 16;
constexpr int kGroups = kBlock / kG;
constexpr uint32_t kGroupList = 128;
constexpr uint32_t kGroupGrid = 2048;

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lds_lower_bound(const uint32_t* a, uint32_t n, uint32_t v) {
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

__global__ void k_slot_heads(const uint32_t* __restrict__ sslot, uint32_t n, uint32_t* head) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) head[i] = (i == 0 || sslot[i] != sslot[i - 1]) ? 1u : 0u;
}

// One lane per touched cube: {slot, first op, ops, old count} and the relocation reserve.
__global__ __launch_bounds__(kBlock) void k_delta_plan_light(const Record* __restrict__ recs,
                                                             const uint32_t* __restrict__ cube_start,
                                                             const uint32_t* __restrict__ sslot,
                                                             const uint64_t* __restrict__ svs,
                                                             const DeltaSummary* sum, uint32_t n, uint4* cinfo,
                                                             uint32_t* reloc, uint64_t* part) {
    __shared__ unsigned long long acc[4];
    if (threadIdx.x < 4) acc[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    uint32_t rw = 0;
    if (c < sum->n_dc) {
        const uint32_t s0 = cube_start[c], nch = cube_start[c + 1] - s0;
        const uint32_t slot = sslot[s0];
        const uint4* line = reinterpret_cast<const uint4*>(recs + slot);
        const uint32_t oc = line[0].z, cap = line[1].z;
        uint32_t subs = 0;  // only subscribes can grow the list
        for (uint32_t t = s0; t < s0 + nch; ++t) subs += (uint32_t)(svs[t] >> 32);
        if ((uint64_t)oc + nch > kGroupList) atomicAdd(&acc[2], 1ull);
        const uint64_t ub = (uint64_t)oc + subs;
        if (ub > cap) rw = 1 + grown((uint32_t)std::min<uint64_t>(ub, 0x7FFFFFFFull));
        cinfo[c] = make_uint4(slot, s0, nch, oc);
        if (rw) atomicAdd(&acc[3], (unsigned long long)rw);
    }
    if (c < n) reloc[c] = rw;
    __syncthreads();
    if (threadIdx.x < 4) part[4ull * blockIdx.x + threadIdx.x] = acc[threadIdx.x];
}

struct GroupLds {
    uint32_t buf[kGroups][2][kGroupList];
    uint32_t add[kGroups][kG];
    uint32_t rem[kGroups][kG];
};

__global__ __launch_bounds__(kBlock) void k_delta_apply_group(DeltaTable tb, const uint4* __restrict__ cinfo,
                                                              const uint64_t* __restrict__ svs,
                                                              const DeltaSummary* sum,
                                                              const uint32_t* __restrict__ reloc,
                                                              const uint32_t* __restrict__ reloc_off,
                                                              uint64_t list_base, uint64_t* part) {
    __shared__ GroupLds sm;
    __shared__ unsigned long long acc[2];
    if (threadIdx.x < 2) acc[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, gl = threadIdx.x & (kG - 1), grp = threadIdx.x / kG;
    const int gshift = lane & ~(kG - 1);
    const uint32_t lt = (1u << gl) - 1u;
    const uint32_t n_dc = sum->n_dc;
    int64_t de = 0, dl = 0;
    uint32_t* add = sm.add[grp];
    uint32_t* rem = sm.rem[grp];
    const uint32_t stride = gridDim.x * kGroups;
    const uint4* recs4 = reinterpret_cast<const uint4*>(tb.recs);
    uint32_t c = blockIdx.x * kGroups + grp;
    // Software pipeline over the group's cubes c, c + stride, ...: while cube c merges, the next
    // cube's list (<= kGroupList words: kPref per lane) is in flight in registers and the header
    // of the one after it is being fetched, so a cube's list latency is paid once per group, not
    // once per cube. (Lists of different cubes are disjoint, and a relocated list moves to fresh
    // space, so prefetching never reads words this group or another is about to write.)
    constexpr int kPref = (int)(kGroupList / kG);
    uint4 ci = make_uint4(0, 0, 0, 0), h0 = ci, h1 = ci, ci_n = ci, h0_n = ci, h1_n = ci;
    uint32_t pref[kPref];
    if (c < n_dc) {
        ci = cinfo[c];
        if (c + stride < n_dc) ci_n = cinfo[c + stride];
        h0 = recs4[8ull * ci.x];
        h1 = recs4[8ull * ci.x + 1];
        if (c + stride < n_dc) {
            h0_n = recs4[8ull * ci_n.x];
            h1_n = recs4[8ull * ci_n.x + 1];
        }
#pragma unroll
        for (int k = 0; k < kPref; ++k) {
            const uint32_t i = (uint32_t)(gl + k * kG);
            pref[k] = i < ci.w ? tb.list[h0.w + 1 + i] : 0u;
        }
    }
    for (; c < n_dc; c += stride) {
        const uint32_t cn = c + stride, cnn = c + 2 * stride;
        uint4 ci_nn = ci_n;
        if (cnn < n_dc) ci_nn = cinfo[cnn];
        const uint32_t slot = ci.x, s0 = ci.y, nch = ci.z, oc = ci.w;
        Record* rec = tb.recs + slot;
        const uint32_t off = h0.w, cap0 = h1.z;
        uint32_t* cur = sm.buf[grp][0];
        uint32_t* nxt = sm.buf[grp][1];
        wave_lds_sync();  // the previous cube's LDS reads are done
#pragma unroll
        for (int k = 0; k < kPref; ++k) {
            const uint32_t i = (uint32_t)(gl + k * kG);
            if (i < oc) cur[i] = pref[k];
        }
        if (cn < n_dc) {  // the next cube's list (its header arrived during the previous cube)
#pragma unroll
            for (int k = 0; k < kPref; ++k) {
                const uint32_t i = (uint32_t)(gl + k * kG);
                pref[k] = i < ci_n.w ? tb.list[h0_n.w + 1 + i] : 0u;
            }
        }
        uint4 h0_nn = h0_n, h1_nn = h1_n;
        if (cnn < n_dc) {
            h0_nn = recs4[8ull * ci_nn.x];
            h1_nn = recs4[8ull * ci_nn.x + 1];
        }
        wave_lds_sync();
        uint32_t n = oc;
        bool changed = false;
        for (uint32_t t0 = 0; t0 < nch; t0 += kG) {
            const uint32_t m = std::min<uint32_t>(kG, nch - t0);
            const bool has = (uint32_t)gl < m;
            const uint64_t v = has ? svs[s0 + t0 + gl] : 0ull;
            uint64_t key = has ? ((v << 32) | (uint32_t)gl) : ~0ull;
            const uint32_t kd = (uint32_t)(v >> 32);
#pragma unroll
            for (int k = 2; k <= kG; k <<= 1) {
#pragma unroll
                for (int j = k >> 1; j > 0; j >>= 1) {
                    const uint64_t o = __shfl_xor(key, j, kG);
                    const bool keep_min = ((gl & j) == 0) == ((gl & k) == 0);
                    key = keep_min ? (o < key ? o : key) : (o > key ? o : key);
                }
            }
            const uint32_t q = (uint32_t)(key >> 32);
            const bool sub = __shfl(kd, (int)((uint32_t)key & (kG - 1)), kG) != 0;
            const uint32_t qn = __shfl(q, (gl + 1) & (kG - 1), kG);
            const bool last = has && ((uint32_t)gl == m - 1 || qn != q);
            const uint32_t at = last ? lds_lower_bound(cur, n, q) : 0u;
            const bool present = last && at < n && cur[at] == q;
            const bool is_add = last && sub && !present, is_rm = last && !sub && present;
            const uint32_t ga = (uint32_t)(__ballot(is_add) >> gshift) & 0xFFFFu;
            const uint32_t gr = (uint32_t)(__ballot(is_rm) >> gshift) & 0xFFFFu;
            const uint32_t nadd = (uint32_t)__popc(ga), nrm = (uint32_t)__popc(gr);
            if (!(nadd | nrm)) continue;
            changed = true;
            const uint32_t add_rank = (uint32_t)__popc(ga & lt);
            if (is_add) add[add_rank] = q;
            if (is_rm) rem[__popc(gr & lt)] = q;
            wave_lds_sync();
            for (uint32_t k = gl; k < n; k += kG) {  // kept peers shift by the removals / adds below them
                const uint32_t x = cur[k];
                const uint32_t r = lds_lower_bound(rem, nrm, x);
                if (r < nrm && rem[r] == x) continue;
                nxt[k - r + lds_lower_bound(add, nadd, x)] = x;
            }
            if (is_add) nxt[add_rank + at - lds_lower_bound(rem, nrm, q)] = q;
            wave_lds_sync();
            uint32_t* t = cur;
            cur = nxt;
            nxt = t;
            n = n + nadd - nrm;
        }
        if (changed) {
        uint32_t dst = off, cap = cap0;
        const uint32_t rl = reloc[c];
        if (rl) {
            dst = (uint32_t)(list_base + reloc_off[c]);
            cap = rl - 1;
        }
        uint32_t* L = tb.list + dst;
        uint64_t sig = 0;
        for (uint32_t k = gl; k < n; k += kG) {
            const uint32_t v = cur[k];
            L[1 + k] = v;
            sig |= peer_sig(v);
        }
#pragma unroll
        for (int d = kG / 2; d >= 1; d >>= 1) sig |= __shfl_xor(sig, d, kG);
        if (gl == 0) L[0] = n;
        uint32_t* rw = reinterpret_cast<uint32_t*>(rec);  // the record line: 32 words, two per lane
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int w = gl + h * kG;
            uint32_t v;
            switch (w) {
                case 0: v = h0.x; break;
                case 1: v = h0.y; break;
                case 2: v = n; break;
                case 3: v = dst; break;
                case 4: v = (uint32_t)sig; break;
                case 5: v = (uint32_t)(sig >> 32); break;
                case 6: v = cap; break;
                case 7: v = h1.w; break;  // ext: the key's high word
                default: v = (uint32_t)(w - kInlineWord0) < n ? cur[w - kInlineWord0] : kNone; break;
            }
            rw[w] = v;
        }
        if (gl == 0) {
            de += (int64_t)n - (int64_t)oc;
            dl += (int64_t)(oc == 0 && n > 0) - (int64_t)(oc > 0 && n == 0);
        }
        }  // changed
        ci = ci_n;
        h0 = h0_n;
        h1 = h1_n;
        ci_n = ci_nn;
        h0_n = h0_nn;
        h1_n = h1_nn;
    }
    if (de) atomicAdd(&acc[0], (unsigned long long)de);
    if (dl) atomicAdd(&acc[1], (unsigned long long)dl);
    __syncthreads();
    if (threadIdx.x < 2) part[2ull * blockIdx.x + threadIdx.x] = acc[threadIdx.x];
}

// Adds the group path's per-block entry / live-cube deltas into the running totals.
__global__ __launch_bounds__(kBlock) void k_delta_stats(const uint64_t* __restrict__ part, uint32_t nb,
                                                        uint64_t* dstat) {
    __shared__ unsigned long long acc[2];
    if (threadIdx.x < 2) acc[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long v0 = 0, v1 = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += kBlock) {
        v0 += part[2ull * b];
        v1 += part[2ull * b + 1];
    }
    if (v0) atomicAdd(&acc[0], v0);
    if (v1) atomicAdd(&acc[1], v1);
    __syncthreads();
    if (threadIdx.x == 0) {
        dstat[0] += acc[0];
        dstat[1] += acc[1];
    }
}

// ---- REMOVE_PEER in place (§8(f) F3) -------------------------------------------------------------
// WorldMap::remove_peer / AreaMap::remove_peer (world_map.rs:41-61, area_map.rs:124-135) for a
// batch of peers: one pass over every cube of both tables, 16 lanes per cube, removing the peers
// from each list in place (a chunk's kept peers move only to lower positions, so a forward
// compaction by group ballots is safe) and rewriting the record's count, signature and inline
// peers where something moved. Peers removed from every world are a bitmap test; removals from
// one world a binary search in the sorted (world << 32 | peer) keys. Empty cubes keep their record.
struct RemoveSet {
    const uint32_t* all_bits;  // peers removed from every world (bitmap), nullptr if none
    uint32_t all_n;            // bitmap length in peers
    const uint64_t* keys;      // sorted (world << 32 | peer) removed from one world
    uint32_t n_keys;
};

__device__ __forceinline__ bool removed(const RemoveSet& rs, uint32_t w, uint32_t p) {
    if (rs.all_bits && p < rs.all_n && ((rs.all_bits[p >> 5] >> (p & 31)) & 1u)) return true;
    if (!rs.n_keys) return false;
    const uint64_t v = ((uint64_t)w << 32) | p;
    uint32_t lo = 0, hi = rs.n_keys;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rs.keys[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo < rs.n_keys && rs.keys[lo] == v;
}

__global__ __launch_bounds__(kBlock) void k_remove_peers(DeltaTable tb, const Slot* __restrict__ slots,
                                                         uint64_t scap, RemoveSet rs, uint64_t* part) {
    __shared__ unsigned long long acc[2];
    if (threadIdx.x < 2) acc[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, gl = threadIdx.x & (kG - 1), grp = threadIdx.x / kG;
    const int gshift = lane & ~(kG - 1);
    const uint32_t lt = (1u << gl) - 1u;
    const uint64_t rcap = tb.rmask + 1, D = rcap + scap;
    int64_t de = 0, dl = 0;
    for (uint64_t e = (uint64_t)blockIdx.x * kGroups + grp; e < D; e += (uint64_t)gridDim.x * kGroups) {
        const bool is_rec = e < rcap;
        uint32_t w, off, n;
        if (is_rec) {
            const uint4 h0 = reinterpret_cast<const uint4*>(tb.recs + e)[0];
            const uint32_t ext = reinterpret_cast<const uint32_t*>(tb.recs + e)[7];
            if (!ext || !h0.z) continue;
            w = (ext >> 8) - 1u;
            n = h0.z;
            off = h0.w;
        } else {
            const SlotView v = load_slot(slots, e - rcap);
            if (v.world == kWorldEmpty) continue;
            w = v.world;
            off = v.off;
            n = tb.list[off];
        }
        uint32_t* L = tb.list + off + 1;
        uint32_t* rw = reinterpret_cast<uint32_t*>(tb.recs + e);
        uint32_t kept = 0;
        uint64_t sig = 0;
        for (uint32_t c0 = 0; c0 < n; c0 += kG) {
            const uint32_t k = c0 + gl;
            const uint32_t x = k < n ? L[k] : 0u;
            const bool keep = k < n && !removed(rs, w, x);
            const uint32_t mk = (uint32_t)(__ballot(keep) >> gshift) & 0xFFFFu;
            if (keep) {
                const uint32_t pos = kept + (uint32_t)__popc(mk & lt);
                sig |= peer_sig(x);
                if (pos != k) {  // shifted by an earlier removal
                    L[pos] = x;
                    if (is_rec && pos < (uint32_t)kInline) rw[kInlineWord0 + pos] = x;
                }
            }
            kept += (uint32_t)__popc(mk);
        }
        if (kept == n) continue;  // group-uniform: nothing removed here
#pragma unroll
        for (int d = kG / 2; d >= 1; d >>= 1) sig |= __shfl_xor(sig, d, kG);
        if (gl == 0) L[-1] = kept;
        if (is_rec) {
            for (uint32_t k = kept + gl; k < n && k < (uint32_t)kInline; k += kG) rw[kInlineWord0 + k] = kNone;
            if (gl == 0) {
                rw[2] = kept;
                rw[4] = (uint32_t)sig;
                rw[5] = (uint32_t)(sig >> 32);
            }
        }
        if (gl == 0) {
            de -= (int64_t)(n - kept);
            dl -= kept == 0 ? 1 : 0;
        }
    }
    if (de) atomicAdd(&acc[0], (unsigned long long)de);
    if (dl) atomicAdd(&acc[1], (unsigned long long)dl);
    __syncthreads();
    if (threadIdx.x < 2) part[2ull * blockIdx.x + threadIdx.x] = acc[threadIdx.x];
}

// ---- materialize: the sorted-state arrays from the records and slots ---------------------------

__device__ __forceinline__ void record_key(const Record& r, int64_t s, uint32_t* w, int64_t* k) {
    uint32_t a[3];
    unpack_key(r.pk, r.ext, w, a);
#pragma unroll
    for (int d = 0; d < 3; ++d) k[d] = ((int64_t)a[d] - (int64_t)kAxisBias) * s;
}

__global__ void k_mat_count(const Record* __restrict__ recs, uint64_t rcap, const Slot* __restrict__ slots,
                            uint64_t scap, const uint32_t* __restrict__ list, uint32_t* cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < rcap) {
        cnt[i] = recs[i].ext ? recs[i].count : 0u;
    } else if (i < rcap + scap) {
        const SlotView s = load_slot(slots, i - rcap);
        cnt[i] = s.world == kWorldEmpty ? 0u : list[s.off];
    }
}

__global__ void k_mat_write(const Record* __restrict__ recs, uint64_t rcap, const Slot* __restrict__ slots,
                            uint64_t scap, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                            const uint32_t* __restrict__ pos, int64_t s, uint64_t hmask, uint64_t* st_h,
                            uint32_t* st_w, int64_t* st_kx, int64_t* st_ky, int64_t* st_kz, uint32_t* st_p) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= rcap + scap) return;
    const uint32_t n = cnt[i];
    if (!n) return;
    uint32_t w, off;
    int64_t k[3];
    if (i < rcap) {
        const Record& r = recs[i];
        record_key(r, s, &w, k);
        off = r.list_off;
    } else {
        const SlotView v = load_slot(slots, i - rcap);
        w = v.world;
        k[0] = v.k0;
        k[1] = v.k1;
        k[2] = v.k2;
        off = v.off;
    }
    const uint64_t hh = cube_hash(w, k[0], k[1], k[2]) & hmask;
    const uint32_t o = pos[i];
    for (uint32_t j = 0; j < n; ++j) {
        st_h[o + j] = hh;
        st_w[o + j] = w;
        st_kx[o + j] = k[0];
        st_ky[o + j] = k[1];
        st_kz[o + j] = k[2];
        st_p[o + j] = list[off + 1 + j];
    }
}

}  // namespace

int table_sync_delta_stats(wq_router* h) {
    if (!h->dstat_pending) {
        WQ_HIP(h, hipStreamSynchronize(h->stream));
        return WQ_OK;
    }
    uint64_t v[2];
    WQ_HIP(h, hipMemcpyAsync(v, h->dws.dstat.p, 16, hipMemcpyDeviceToHost, h->stream));
    WQ_HIP(h, hipMemsetAsync(h->dws.dstat.p, 0, 16, h->stream));
    WQ_HIP(h, hipStreamSynchronize(h->stream));
    h->st.n = (uint64_t)((int64_t)h->st.n + (int64_t)v[0]);
    h->tab.n_cubes = (uint64_t)((int64_t)h->tab.n_cubes + (int64_t)v[1]);
    h->dstat_pending = false;
    return WQ_OK;
}

namespace {

// The per-lane path (any cube size): sort by (slot, peer), one lane per touched cube.
int delta_plan_lanes(wq_router* h, uint32_t n, DeltaTable tb, DeltaSummary* sum) {
    DeltaWs& d = h->dws;
    hipStream_t s = h->stream;
    const uint32_t nb = grid_for(n);
    int bits = 1;
    while ((1ull << bits) < h->tab.rec_cap) bits++;
    uint32_t* idx_a = h->idx_a.as<uint32_t>();
    uint32_t* idx_b = h->idx_b.as<uint32_t>();
    hipLaunchKernelGGL(k_iota, dim3(nb), dim3(kBlock), 0, s, idx_a, (uint64_t)n);
    int rc = sort_pairs<uint32_t>(h, d.peer.as<uint32_t>(), h->key32_a.as<uint32_t>(), idx_a, idx_b, n, 32);
    if (rc) return rc;
    uint32_t* key_a = h->key64_a.as<uint32_t>();  // 32-bit slot columns in the 64-bit scratch
    uint32_t* key_b = h->key64_b.as<uint32_t>();
    hipLaunchKernelGGL(k_gather<uint32_t>, dim3(nb), dim3(kBlock), 0, s, d.slot.as<uint32_t>(), idx_b, key_a,
                       (uint64_t)n);
    if ((rc = sort_pairs<uint32_t>(h, key_a, key_b, idx_b, idx_a, n, bits))) return rc;
    const uint32_t* spk = key_b;
    uint32_t* head = h->flags.as<uint32_t>();
    uint32_t* cid = h->scan.as<uint32_t>();
    hipLaunchKernelGGL(k_delta_mark, dim3(nb), dim3(kBlock), 0, s, idx_a, spk, d.peer.as<uint32_t>(),
                       d.kind.as<uint8_t>(), n, d.sp.as<uint32_t>(), d.skd.as<uint8_t>(), head);
    if ((rc = scan_u32(h, head, cid, n, true))) return rc;
    uint32_t* cube_start = h->cube_start.as<uint32_t>();
    hipLaunchKernelGGL(k_delta_cubes, dim3(nb), dim3(kBlock), 0, s, head, cid, n, cube_start, sum);
    hipLaunchKernelGGL(k_delta_plan, dim3(nb), dim3(kBlock), 0, s, tb, cube_start, spk, d.sp.as<uint32_t>(),
                       d.skd.as<uint8_t>(), sum, n, d.plan.as<uint4>(), d.reloc.as<uint32_t>(),
                       d.part.as<uint64_t>());
    hipLaunchKernelGGL(k_delta_reduce, dim3(1), dim3(kBlock), 0, s, d.part.as<uint64_t>(), nb, sum);
    return scan_u32(h, d.reloc.as<uint32_t>(), d.reloc_off.as<uint32_t>(), n, false);
}

// The group path's plan: sort by record slot, light plan per touched cube.
int delta_plan_groups(wq_router* h, uint32_t n, DeltaSummary* sum) {
    DeltaWs& d = h->dws;
    Table& t = h->tab;
    hipStream_t s = h->stream;
    const uint32_t nb = grid_for(n);
    int bits = 1;
    while ((1ull << bits) < t.rec_cap) bits++;
    // (slot, kind << 32 | peer) sorted by slot, stable: each cube's ops stay in op order
    int rc = sort_pairs<uint32_t, uint64_t>(h, d.slot.as<uint32_t>(), h->key32_a.as<uint32_t>(), d.sv.as<uint64_t>(),
                                            d.svs.as<uint64_t>(), n, bits);
    if (rc) return rc;
    const uint32_t* sslot = h->key32_a.as<uint32_t>();
    uint32_t* head = h->flags.as<uint32_t>();
    uint32_t* cid = h->scan.as<uint32_t>();
    hipLaunchKernelGGL(k_slot_heads, dim3(nb), dim3(kBlock), 0, s, sslot, n, head);
    if ((rc = scan_u32(h, head, cid, n, true))) return rc;
    uint32_t* cube_start = h->cube_start.as<uint32_t>();
    hipLaunchKernelGGL(k_delta_cubes, dim3(nb), dim3(kBlock), 0, s, head, cid, n, cube_start, sum);
    hipLaunchKernelGGL(k_delta_plan_light, dim3(nb), dim3(kBlock), 0, s, t.recs.as<Record>(), cube_start, sslot,
                       d.svs.as<uint64_t>(), sum, n, d.plan.as<uint4>(), d.reloc.as<uint32_t>(), d.part.as<uint64_t>());
    hipLaunchKernelGGL(k_delta_reduce, dim3(1), dim3(kBlock), 0, s, d.part.as<uint64_t>(), nb, sum);
    return scan_u32(h, d.reloc.as<uint32_t>(), d.reloc_off.as<uint32_t>(), n, false);
}

int read_summary(wq_router* h, const DeltaSummary* sum, DeltaSummary* hs) {
    WQ_HIP(h, hipGetLastError());
    WQ_HIP(h, hipMemcpyAsync(hs, sum, sizeof(*hs), hipMemcpyDeviceToHost, h->stream));
    return table_sync_delta_stats(h);  // synchronises the stream
}

}  // namespace

int table_apply_delta(wq_router* h, size_t n_ops, bool* applied) {
    *applied = false;
    if (n_ops == 0) {
        *applied = true;
        return WQ_OK;
    }
    const uint32_t n = (uint32_t)n_ops;
    DeltaWs& d = h->dws;
    Table& t = h->tab;
    hipStream_t s = h->stream;
    // every op may bring a new cube: keep the record table at load <= 1/2 through the claims
    if (2 * (t.n_recs + n) > t.rec_cap) {
        h->n_delta_fallbacks++;
        return WQ_OK;
    }
    const uint32_t nb = grid_for(n);
    WQ_ALLOC(h, d.slot, (uint64_t)n * 4);
    WQ_ALLOC(h, d.peer, (uint64_t)n * 4);
    WQ_ALLOC(h, d.kind, n);
    WQ_ALLOC(h, d.sp, (uint64_t)n * 4);
    WQ_ALLOC(h, d.sv, (uint64_t)n * 8);
    WQ_ALLOC(h, d.svs, (uint64_t)n * 8);
    WQ_ALLOC(h, d.skd, n);
    WQ_ALLOC(h, d.plan, (uint64_t)n * 16);
    WQ_ALLOC(h, d.reloc, (uint64_t)n * 4);
    WQ_ALLOC(h, d.reloc_off, (uint64_t)n * 4);
    WQ_ALLOC(h, d.part, ((uint64_t)nb + kGroupGrid) * 32);
    WQ_ALLOC(h, d.summ, sizeof(DeltaSummary));
    if (!d.dstat.p) {
        WQ_ALLOC(h, d.dstat, 16);
        WQ_HIP(h, hipMemsetAsync(d.dstat.p, 0, 16, s));
    }
    WQ_ALLOC(h, h->idx_a, (uint64_t)n * 4);
    WQ_ALLOC(h, h->idx_b, (uint64_t)n * 4);
    WQ_ALLOC(h, h->key32_a, (uint64_t)n * 4);
    WQ_ALLOC(h, h->key64_a, (uint64_t)n * 8);
    WQ_ALLOC(h, h->key64_b, (uint64_t)n * 8);
    WQ_ALLOC(h, h->flags, (uint64_t)n * 4);
    WQ_ALLOC(h, h->scan, (uint64_t)n * 4);
    WQ_ALLOC(h, h->cube_start, ((uint64_t)n + 1) * 4);
    DeltaSummary* sum = d.summ.as<DeltaSummary>();
    WQ_HIP(h, hipMemsetAsync(sum, 0, sizeof(DeltaSummary), s));
    hipLaunchKernelGGL(k_delta_events, dim3(nb), dim3(kBlock), 0, s, h->cur_ops, n, (double)h->cube_size,
                       (int64_t)h->cube_size, t.recs.as<Record>(), t.rclaim.as<uint32_t>(),
                       kBatchTag | (uint32_t)(++h->n_delta_batches & 0x7FFFFFFFu), t.rec_cap - 1,
                       t.rec_shift, h->hash_mask, d.slot.as<uint32_t>(), d.peer.as<uint32_t>(),
                       d.kind.as<uint8_t>(), d.sv.as<uint64_t>(), sum);
    DeltaTable tb{t.recs.as<Record>(), t.rclaim.as<uint32_t>(), t.rec_cap - 1, t.rec_shift, h->hash_mask,
                  t.list.as<uint32_t>()};
    int rc = delta_plan_groups(h, n, sum);
    if (rc) return rc;
    DeltaSummary hs;
    if ((rc = read_summary(h, sum, &hs))) return rc;
    // the claims of a batch that falls back stay as empty records (count 0): invisible to every
    // query, dropped by the rebuild
    t.n_recs += hs.new_recs;
    if (hs.irregular & 2u) return set_error(h, WQ_E_INVALID, "bad op (kind or reserved world id)");
    const bool groups = hs.n_big == 0 && !hs.irregular;
    if (!groups && !hs.irregular) {  // a cube past the wave path's bounds: plan the batch per lane
        if ((rc = delta_plan_lanes(h, n, tb, sum))) return rc;
        if ((rc = read_summary(h, sum, &hs))) return rc;
    }
    const uint64_t list_limit = std::min<uint64_t>(t.list_cap, 0xFFFFFFFFull);
    if (hs.irregular || t.list_used + hs.reloc_words > list_limit || 4 * t.n_recs > t.rec_cap) {
        h->n_delta_fallbacks++;
        return WQ_OK;  // no list or count changed: the caller rebuilds
    }
    if (groups) {
        const uint32_t ng = std::min<uint32_t>((n + kGroups - 1) / kGroups, kGroupGrid);
        hipLaunchKernelGGL(k_delta_apply_group, dim3(ng), dim3(kBlock), 0, s, tb, d.plan.as<uint4>(),
                           d.svs.as<uint64_t>(), sum, d.reloc.as<uint32_t>(),
                           d.reloc_off.as<uint32_t>(), t.list_used, d.part.as<uint64_t>());
        // entry / live-cube deltas stay on the device until the next read-back (table_sync_delta_stats)
        hipLaunchKernelGGL(k_delta_stats, dim3(1), dim3(kBlock), 0, s, d.part.as<uint64_t>(), ng,
                           d.dstat.as<uint64_t>());
        h->dstat_pending = true;
    } else {
        hipLaunchKernelGGL(k_delta_apply, dim3(nb), dim3(kBlock), 0, s, tb, h->cube_start.as<uint32_t>(),
                           d.sp.as<uint32_t>(), d.skd.as<uint8_t>(), sum,
                           d.plan.as<uint4>(), d.reloc.as<uint32_t>(), d.reloc_off.as<uint32_t>(), t.list_used);
        h->st.n = (uint64_t)((int64_t)h->st.n + (int64_t)hs.d_entries);
        t.n_cubes = (uint64_t)((int64_t)t.n_cubes + (int64_t)hs.d_live);
    }
    WQ_HIP(h, hipGetLastError());
    // subscribes may widen peer boxes: switch the boxes off until the next full build (the count
    // pass then searches every long list); per-op box atomics here cost more than they save
    if (t.n_pbox) WQ_HIP(h, hipMemsetAsync(t.pbox.as<uint32_t>() + (uint64_t)kBoxWords * t.n_pbox, 0, 4, s));
    t.list_used += hs.reloc_words;
    h->st_stale = true;
    h->any_stale = true;
    h->n_delta_applies++;
    if (!groups) h->n_delta_lane_batches++;
    *applied = true;
    return WQ_OK;
}

int table_remove_peers_inplace(wq_router* h, const uint64_t* keys, size_t n_rm) {
    DeltaWs& d = h->dws;
    Table& t = h->tab;
    hipStream_t s = h->stream;
    // split: (WQ_WORLD_INVALID, peer) = every world -> bitmap; the rest stay sorted keys
    size_t n_all = 0;
    uint32_t max_all = 0;
    while (n_all < n_rm && (keys[n_rm - 1 - n_all] >> 32) == WQ_WORLD_INVALID) {
        max_all = std::max<uint32_t>(max_all, (uint32_t)keys[n_rm - 1 - n_all]);
        ++n_all;
    }
    const size_t n_one = n_rm - n_all;  // keys sort by world first: the every-world ones are last
    RemoveSet rs{nullptr, 0, nullptr, (uint32_t)n_one};
    if (n_all) {
        const uint32_t words = max_all / 32 + 1;
        std::vector<uint32_t> bits(words, 0u);
        for (size_t i = n_one; i < n_rm; ++i) {
            const uint32_t p = (uint32_t)keys[i];
            bits[p >> 5] |= 1u << (p & 31);
        }
        WQ_ALLOC(h, d.rm_bits, (uint64_t)words * 4);
        WQ_HIP(h, hipMemcpyAsync(d.rm_bits.p, bits.data(), (size_t)words * 4, hipMemcpyHostToDevice, s));
        rs.all_bits = d.rm_bits.as<uint32_t>();
        rs.all_n = words * 32;
    }
    if (n_one) {
        WQ_ALLOC(h, h->key32_b, n_one * 8);
        WQ_HIP(h, hipMemcpyAsync(h->key32_b.p, keys, n_one * 8, hipMemcpyHostToDevice, s));
        rs.keys = h->key32_b.as<uint64_t>();
    }
    WQ_ALLOC(h, d.part, (uint64_t)kGroupGrid * 32);
    if (!d.dstat.p) {
        WQ_ALLOC(h, d.dstat, 16);
        WQ_HIP(h, hipMemsetAsync(d.dstat.p, 0, 16, s));
    }
    DeltaTable tb{t.recs.as<Record>(), t.rclaim.as<uint32_t>(), t.rec_cap - 1, t.rec_shift, h->hash_mask,
                  t.list.as<uint32_t>()};
    const uint64_t D = t.rec_cap + t.cap;
    const uint32_t ng = (uint32_t)std::min<uint64_t>((D + kGroups - 1) / kGroups, kGroupGrid);
    hipLaunchKernelGGL(k_remove_peers, dim3(ng), dim3(kBlock), 0, s, tb, t.slots.as<Slot>(), t.cap, rs,
                       d.part.as<uint64_t>());
    hipLaunchKernelGGL(k_delta_stats, dim3(1), dim3(kBlock), 0, s, d.part.as<uint64_t>(), ng, d.dstat.as<uint64_t>());
    WQ_HIP(h, hipGetLastError());
    h->dstat_pending = true;
    h->st_stale = true;
    h->any_stale = true;
    // the host arrays above are read by copies still in flight
    WQ_HIP(h, hipStreamSynchronize(s));
    return WQ_OK;
}

int table_materialize(wq_router* h) {
    if (!h->st_stale) return WQ_OK;
    int rc0 = table_sync_delta_stats(h);
    if (rc0) return rc0;
    Table& t = h->tab;
    hipStream_t s = h->stream;
    const uint64_t D = t.rec_cap + t.cap;
    if (D >= 0xFFFFFFFFull) return set_error(h, WQ_E_INVALID, "table too large to materialize");
    WQ_ALLOC(h, h->flags, D * 4);
    WQ_ALLOC(h, h->scan, D * 4);
    uint32_t* cnt = h->flags.as<uint32_t>();
    uint32_t* pos = h->scan.as<uint32_t>();
    hipLaunchKernelGGL(k_mat_count, dim3(grid_for(D)), dim3(kBlock), 0, s, t.recs.as<Record>(), t.rec_cap,
                       t.slots.as<Slot>(), t.cap, t.list.as<uint32_t>(), cnt);
    int rc = scan_u32(h, cnt, pos, D, false);
    if (rc) return rc;
    uint32_t lp = 0, lc = 0;
    if ((rc = read_u32(h, pos, D - 1, &lp))) return rc;
    if ((rc = read_u32(h, cnt, D - 1, &lc))) return rc;
    const uint64_t S = (uint64_t)lp + lc;
    if (S != h->st.n) return set_error(h, WQ_E_HIP, "materialize: entry count disagrees with the table");
    if ((rc = ensure_state(h, h->st, S))) return rc;
    hipLaunchKernelGGL(k_mat_write, dim3(grid_for(D)), dim3(kBlock), 0, s, t.recs.as<Record>(), t.rec_cap,
                       t.slots.as<Slot>(), t.cap, t.list.as<uint32_t>(), cnt, pos, (int64_t)h->cube_size,
                       h->hash_mask, h->st.h.as<uint64_t>(), h->st.w.as<uint32_t>(), h->st.kx.as<int64_t>(),
                       h->st.ky.as<int64_t>(), h->st.kz.as<int64_t>(), h->st.p.as<uint32_t>());
    WQ_HIP(h, hipGetLastError());
    h->st_stale = false;
    return WQ_OK;
}

}  // namespace wq
