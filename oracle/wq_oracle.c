/*
 * wq_oracle.c — CPU restatement of the WorldQL subscription table and LocalMessage routing.
 * TEST INFRASTRUCTURE ONLY (see wq_oracle.h). Also the `cpu_baseline` ("port") of bench.py:
 * it keeps the reference's shape — hash map world -> hash map cube(3 x i64) -> hash set of
 * peers, one message at a time on one core (worldql_server/src/processing/thread.rs:113-148).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no -ffast-math: the f64 op sequence of
 * coord_clamp must be reproduced exactly).
 */
#include "wq_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------
 * Quantisation
 * ------------------------------------------------------------------------------------------ */

/* Rust `f64 as i64` (saturating, NaN -> 0, truncation toward zero). */
static int64_t sat_i64(double x) {
    if (x != x) return 0;
    if (x >= 9223372036854775808.0) return INT64_MAX;
    if (x <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)x;
}

/* worldql_server/src/utils/round.rs:1-13 */
double wqo_round_by_multiple(double n, double multiple) {
    if (multiple == 0.0) return n;
    if (n == 0.0 || n == -0.0) return multiple; /* "0 should round up" (round.rs:6-9) */
    double c = ceil(n / multiple);
    return c * multiple;
}

/* worldql_server/src/subscriptions/cube_area.rs:23-44. Release build: i64 `+` and `*` wrap
 * (Cargo.toml:7-9 sets no overflow checks), hence the unsigned arithmetic. */
int64_t wqo_coord_clamp(double coord, uint16_t size) {
    double abs_coord = fabs(coord);
    int64_t mult = (coord < 0.0) ? -1 : 1; /* cube_area.rs:25-28: -0.0 and NaN give +1 */
    int64_t size_i = (int64_t)size;
    double size_f = (double)size;

    if (fmod(abs_coord, size_f) == 0.0 && coord != 0.0) /* cube_area.rs:33-35 */
        return sat_i64(coord);

    double rounded = wqo_round_by_multiple(abs_coord, size_f); /* cube_area.rs:37 */
    int64_t result;
    if (rounded > coord) /* compared with the SIGNED coordinate, cube_area.rs:38-41 */
        result = sat_i64(rounded);
    else
        result = (int64_t)((uint64_t)sat_i64(rounded) + (uint64_t)size_i);
    return (int64_t)((uint64_t)result * (uint64_t)mult); /* cube_area.rs:43 */
}

void wqo_quantize(const double* coords, size_t n, uint16_t size, int64_t* out) {
    for (size_t i = 0; i < n; ++i) out[i] = wqo_coord_clamp(coords[i], size);
}

/* ------------------------------------------------------------------------------------------
 * Containers. AHashSet<Uuid> -> u32 "peer set" (unordered array, O(n) membership like a small
 * set scan); AHashMap<CubeArea, set> -> open addressing with tombstones; AHashSet<Uuid>
 * subscribed_peers -> u32 open-addressing set; AHashMap<String, AreaMap> -> u32 world map.
 * ------------------------------------------------------------------------------------------ */

static uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xbf58476d1ce4e5b9ULL;
    z ^= z >> 27;
    z *= 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return z;
}

typedef struct {
    uint32_t* v;
    uint32_t n, cap;
} peer_set;

static int ps_find(const peer_set* s, uint32_t p) {
    for (uint32_t i = 0; i < s->n; ++i)
        if (s->v[i] == p) return (int)i;
    return -1;
}
static int ps_insert(peer_set* s, uint32_t p) {
    if (ps_find(s, p) >= 0) return 0;
    if (s->n == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 4;
        s->v = (uint32_t*)realloc(s->v, sizeof(uint32_t) * s->cap);
    }
    s->v[s->n++] = p;
    return 1;
}
static int ps_remove(peer_set* s, uint32_t p) {
    int i = ps_find(s, p);
    if (i < 0) return 0;
    s->v[i] = s->v[--s->n];
    return 1;
}

/* u32 hash set with tombstones (subscribed_peers) */
enum { SLOT_EMPTY = 0, SLOT_FULL = 1, SLOT_TOMB = 2 };
typedef struct {
    uint32_t* key;
    uint8_t* st;
    size_t cap, n_full, n_used; /* n_used counts full + tombstones */
} u32_set;

static void us_init(u32_set* s) {
    s->cap = 16;
    s->key = (uint32_t*)calloc(s->cap, sizeof(uint32_t));
    s->st = (uint8_t*)calloc(s->cap, 1);
    s->n_full = s->n_used = 0;
}
static void us_free(u32_set* s) {
    free(s->key);
    free(s->st);
}
static int us_contains(const u32_set* s, uint32_t k) {
    size_t m = s->cap - 1, i = mix64(k) & m;
    for (;;) {
        if (s->st[i] == SLOT_EMPTY) return 0;
        if (s->st[i] == SLOT_FULL && s->key[i] == k) return 1;
        i = (i + 1) & m;
    }
}
static int us_insert(u32_set* s, uint32_t k);
static void us_grow(u32_set* s) {
    u32_set old = *s;
    s->cap = old.cap * ((old.n_full * 2 >= old.cap / 2) ? 2 : 1);
    s->key = (uint32_t*)calloc(s->cap, sizeof(uint32_t));
    s->st = (uint8_t*)calloc(s->cap, 1);
    s->n_full = s->n_used = 0;
    for (size_t i = 0; i < old.cap; ++i)
        if (old.st[i] == SLOT_FULL) us_insert(s, old.key[i]);
    us_free(&old);
}
static int us_insert(u32_set* s, uint32_t k) {
    if ((s->n_used + 1) * 4 > s->cap * 3) us_grow(s);
    size_t m = s->cap - 1, i = mix64(k) & m, tomb = (size_t)-1;
    for (;;) {
        if (s->st[i] == SLOT_EMPTY) break;
        if (s->st[i] == SLOT_FULL && s->key[i] == k) return 0;
        if (s->st[i] == SLOT_TOMB && tomb == (size_t)-1) tomb = i;
        i = (i + 1) & m;
    }
    if (tomb != (size_t)-1) {
        i = tomb;
    } else {
        s->n_used++;
    }
    s->st[i] = SLOT_FULL;
    s->key[i] = k;
    s->n_full++;
    return 1;
}
static int us_remove(u32_set* s, uint32_t k) {
    size_t m = s->cap - 1, i = mix64(k) & m;
    for (;;) {
        if (s->st[i] == SLOT_EMPTY) return 0;
        if (s->st[i] == SLOT_FULL && s->key[i] == k) {
            s->st[i] = SLOT_TOMB;
            s->n_full--;
            return 1;
        }
        i = (i + 1) & m;
    }
}

/* cube map: CubeArea -> peer_set, tombstones on removal (area_map.rs:108-110) */
typedef struct {
    int64_t k[3];
    uint8_t st;
    peer_set set;
} cube_slot;

typedef struct {
    cube_slot* s;
    size_t cap, n_full, n_used;
} cube_map;

static uint64_t cube_hash(const int64_t k[3]) {
    uint64_t h = mix64((uint64_t)k[0] ^ 0x9e3779b97f4a7c15ULL);
    h = mix64(h ^ (uint64_t)k[1]);
    return mix64(h ^ (uint64_t)k[2]);
}
static int key_eq(const int64_t a[3], const int64_t b[3]) {
    return a[0] == b[0] && a[1] == b[1] && a[2] == b[2];
}
static void cm_init(cube_map* m) {
    m->cap = 64;
    m->s = (cube_slot*)calloc(m->cap, sizeof(cube_slot));
    m->n_full = m->n_used = 0;
}
static void cm_free(cube_map* m) {
    for (size_t i = 0; i < m->cap; ++i)
        if (m->s[i].st == SLOT_FULL) free(m->s[i].set.v);
    free(m->s);
}
static cube_slot* cm_find(const cube_map* m, const int64_t k[3]) {
    size_t msk = m->cap - 1, i = cube_hash(k) & msk;
    for (;;) {
        cube_slot* c = &m->s[i];
        if (c->st == SLOT_EMPTY) return NULL;
        if (c->st == SLOT_FULL && key_eq(c->k, k)) return c;
        i = (i + 1) & msk;
    }
}
static cube_slot* cm_insert(cube_map* m, const int64_t k[3]);
static void cm_grow(cube_map* m) {
    cube_map old = *m;
    m->cap = old.cap * ((old.n_full * 2 >= old.cap / 2) ? 2 : 1);
    m->s = (cube_slot*)calloc(m->cap, sizeof(cube_slot));
    m->n_full = m->n_used = 0;
    for (size_t i = 0; i < old.cap; ++i)
        if (old.s[i].st == SLOT_FULL) {
            cube_slot* c = cm_insert(m, old.s[i].k);
            c->set = old.s[i].set; /* move */
        }
    free(old.s);
}
/* entry(cube).or_insert_with(Default::default) */
static cube_slot* cm_insert(cube_map* m, const int64_t k[3]) {
    cube_slot* f = cm_find(m, k);
    if (f) return f;
    if ((m->n_used + 1) * 4 > m->cap * 3) cm_grow(m);
    size_t msk = m->cap - 1, i = cube_hash(k) & msk, tomb = (size_t)-1;
    for (;;) {
        cube_slot* c = &m->s[i];
        if (c->st == SLOT_EMPTY) break;
        if (c->st == SLOT_TOMB && tomb == (size_t)-1) tomb = i;
        i = (i + 1) & msk;
    }
    if (tomb != (size_t)-1)
        i = tomb;
    else
        m->n_used++;
    cube_slot* c = &m->s[i];
    c->st = SLOT_FULL;
    memcpy(c->k, k, sizeof(c->k));
    memset(&c->set, 0, sizeof(c->set));
    m->n_full++;
    return c;
}
static void cm_remove(cube_map* m, cube_slot* c) {
    free(c->set.v);
    memset(&c->set, 0, sizeof(c->set));
    c->st = SLOT_TOMB;
    m->n_full--;
}

/* u32 -> u32 counter map (fast mode, below): open addressing, no deletion (a zero count stays) */
typedef struct {
    uint32_t* key;
    uint32_t* val;
    uint8_t* st;
    size_t cap, n;
} u32_count;

static void uc_init(u32_count* c) {
    c->cap = 16;
    c->key = (uint32_t*)calloc(c->cap, sizeof(uint32_t));
    c->val = (uint32_t*)calloc(c->cap, sizeof(uint32_t));
    c->st = (uint8_t*)calloc(c->cap, 1);
    c->n = 0;
}
static void uc_free(u32_count* c) {
    free(c->key);
    free(c->val);
    free(c->st);
}
static uint32_t* uc_slot(u32_count* c, uint32_t k) {
    if ((c->n + 1) * 2 > c->cap) {
        u32_count old = *c;
        c->cap *= 2;
        c->key = (uint32_t*)calloc(c->cap, sizeof(uint32_t));
        c->val = (uint32_t*)calloc(c->cap, sizeof(uint32_t));
        c->st = (uint8_t*)calloc(c->cap, 1);
        c->n = 0;
        for (size_t i = 0; i < old.cap; ++i)
            if (old.st[i]) *uc_slot(c, old.key[i]) = old.val[i];
        uc_free(&old);
    }
    size_t m = c->cap - 1, i = mix64(k) & m;
    while (c->st[i] && c->key[i] != k) i = (i + 1) & m;
    if (!c->st[i]) {
        c->st[i] = 1;
        c->key[i] = k;
        c->val[i] = 0;
        c->n++;
    }
    return &c->val[i];
}

/* AreaMap, worldql_server/src/subscriptions/area_map.rs:10-17. `cubes_of` is only kept in fast
 * mode (wqo_set_fast): the number of cubes of this world holding each peer. */
typedef struct {
    cube_map map;
    u32_set subscribed_peers;
    u32_count cubes_of;
} area_map;

/* WorldMap, world_map.rs:10-13 (world names are interned to u32 ids on the host) */
typedef struct {
    uint32_t world;
    area_map* am;
} world_slot;

struct wqo_world_map {
    uint16_t cube_size;
    int fast; /* wqo_set_fast */
    world_slot* w;
    size_t cap, n;
};

int wqo_set_fast(wqo_world_map* wm, int fast) {
    if (wm->n) return -1; /* only on an empty map: the per-peer cube counts start at zero */
    wm->fast = fast != 0;
    return 0;
}

wqo_world_map* wqo_create(uint16_t cube_size) {
    wqo_world_map* wm = (wqo_world_map*)calloc(1, sizeof(*wm));
    wm->cube_size = cube_size;
    wm->cap = 16;
    wm->w = (world_slot*)calloc(wm->cap, sizeof(world_slot));
    return wm;
}

void wqo_destroy(wqo_world_map* wm) {
    if (!wm) return;
    for (size_t i = 0; i < wm->cap; ++i)
        if (wm->w[i].am) {
            cm_free(&wm->w[i].am->map);
            us_free(&wm->w[i].am->subscribed_peers);
            uc_free(&wm->w[i].am->cubes_of);
            free(wm->w[i].am);
        }
    free(wm->w);
    free(wm);
}

/* world_map.rs:25-27 */
static area_map* wm_get(const wqo_world_map* wm, uint32_t world) {
    size_t m = wm->cap - 1, i = mix64(world) & m;
    for (;;) {
        if (!wm->w[i].am) return NULL;
        if (wm->w[i].world == world) return wm->w[i].am;
        i = (i + 1) & m;
    }
}
static void wm_put(wqo_world_map* wm, uint32_t world, area_map* am) {
    size_t m = wm->cap - 1, i = mix64(world) & m;
    while (wm->w[i].am) i = (i + 1) & m;
    wm->w[i].world = world;
    wm->w[i].am = am;
}
/* world_map.rs:31-36 */
static area_map* wm_get_mut(wqo_world_map* wm, uint32_t world) {
    area_map* am = wm_get(wm, world);
    if (am) return am;
    if ((wm->n + 1) * 2 > wm->cap) {
        world_slot* old = wm->w;
        size_t oc = wm->cap;
        wm->cap *= 2;
        wm->w = (world_slot*)calloc(wm->cap, sizeof(world_slot));
        for (size_t i = 0; i < oc; ++i)
            if (old[i].am) wm_put(wm, old[i].world, old[i].am);
        free(old);
    }
    am = (area_map*)calloc(1, sizeof(area_map));
    cm_init(&am->map);
    us_init(&am->subscribed_peers);
    uc_init(&am->cubes_of);
    wm_put(wm, world, am);
    wm->n++;
    return am;
}

/* ToCubeArea (cube_area.rs:61-77): raw CubeArea passes through, Vector3 is quantised. */
static void to_cube_area(int key_is_raw, const void* key_or_pos, uint16_t size, int64_t out[3]) {
    if (key_is_raw) {
        memcpy(out, key_or_pos, 3 * sizeof(int64_t));
    } else {
        const double* p = (const double*)key_or_pos;
        out[0] = wqo_coord_clamp(p[0], size);
        out[1] = wqo_coord_clamp(p[1], size);
        out[2] = wqo_coord_clamp(p[2], size);
    }
}

/* area_map.rs:72-85 */
static int am_add(area_map* am, uint32_t peer, const int64_t k[3], int fast) {
    cube_slot* c = cm_insert(&am->map, k);
    us_insert(&am->subscribed_peers, peer);
    const int added = ps_insert(&c->set, peer);
    if (fast && added) ++*uc_slot(&am->cubes_of, peer);
    return added;
}

/* area_map.rs:88-119, including the O(#cubes) scan at :113. Fast mode answers the scan's question
 * ("does any other cube still hold the peer?") from the per-peer cube count instead: the same
 * answer, because a peer is in subscribed_peers exactly when some cube set holds it (add inserts
 * into both, remove_peer removes from both, and this function keeps it) — for the test checker
 * only, never for the timed CPU baseline, which keeps the reference's scan. */
static int am_remove(area_map* am, uint32_t peer, const int64_t k[3], int fast) {
    cube_slot* c = cm_find(&am->map, k);
    if (!c) return 0; /* :92-94 */
    int removed = ps_remove(&c->set, peer);
    if (c->set.n == 0) cm_remove(&am->map, c); /* :108-110 */
    int has_other = 0;
    if (fast) {
        uint32_t* n = uc_slot(&am->cubes_of, peer);
        if (removed) --*n;
        has_other = *n > 0;
    } else {
        for (size_t i = 0; i < am->map.cap && !has_other; ++i)
            if (am->map.s[i].st == SLOT_FULL && ps_find(&am->map.s[i].set, peer) >= 0) has_other = 1;
    }
    if (!has_other) us_remove(&am->subscribed_peers, peer);
    return removed;
}

/* area_map.rs:124-135: empty sets are kept */
static int am_remove_peer(area_map* am, uint32_t peer) {
    us_remove(&am->subscribed_peers, peer);
    if (am->cubes_of.n) *uc_slot(&am->cubes_of, peer) = 0;
    int removed = 0;
    for (size_t i = 0; i < am->map.cap; ++i)
        if (am->map.s[i].st == SLOT_FULL && ps_remove(&am->map.s[i].set, peer)) removed = 1;
    return removed;
}

int wqo_add_subscription(wqo_world_map* wm, uint32_t world, uint32_t peer, int key_is_raw,
                         const void* key_or_pos) {
    int64_t k[3];
    to_cube_area(key_is_raw, key_or_pos, wm->cube_size, k);
    return am_add(wm_get_mut(wm, world), peer, k, wm->fast);
}

int wqo_remove_subscription(wqo_world_map* wm, uint32_t world, uint32_t peer, int key_is_raw,
                            const void* key_or_pos) {
    int64_t k[3];
    to_cube_area(key_is_raw, key_or_pos, wm->cube_size, k);
    return am_remove(wm_get_mut(wm, world), peer, k, wm->fast); /* get_mut creates (area_unsubscribe.rs:189) */
}

/* world_map.rs:41-61 */
int wqo_remove_peer(wqo_world_map* wm, uint32_t peer) {
    int removed = 0;
    for (size_t i = 0; i < wm->cap; ++i)
        if (wm->w[i].am && am_remove_peer(wm->w[i].am, peer)) removed = 1;
    return removed;
}

int wqo_is_subscribed(const wqo_world_map* wm, uint32_t world, uint32_t peer, int key_is_raw,
                      const void* key_or_pos) {
    const area_map* am = wm_get(wm, world);
    if (!am) return 0;
    int64_t k[3];
    to_cube_area(key_is_raw, key_or_pos, wm->cube_size, k);
    const cube_slot* c = cm_find(&am->map, k);
    return c ? (ps_find(&c->set, peer) >= 0) : 0;
}

int wqo_is_subscribed_any(const wqo_world_map* wm, uint32_t world, uint32_t peer) {
    const area_map* am = wm_get(wm, world);
    return am ? us_contains(&am->subscribed_peers, peer) : 0;
}

size_t wqo_world_peers(const wqo_world_map* wm, uint32_t world, uint32_t* out, size_t cap) {
    const area_map* am = wm_get(wm, world);
    if (!am) return 0;
    size_t n = 0;
    for (size_t i = 0; i < am->subscribed_peers.cap; ++i)
        if (am->subscribed_peers.st[i] == SLOT_FULL) {
            if (n < cap) out[n] = am->subscribed_peers.key[i];
            n++;
        }
    return n;
}

/* Same byte layout as wq_op (include/wq_router.h). */
typedef struct {
    uint32_t world, peer;
    uint8_t kind, key_is_raw, pad_[6];
    union {
        double pos[3];
        int64_t key[3];
    } u;
} oracle_op;

void wqo_apply_ops(wqo_world_map* wm, const void* ops_v, size_t n) {
    const oracle_op* ops = (const oracle_op*)ops_v;
    for (size_t i = 0; i < n; ++i) {
        const oracle_op* o = &ops[i];
        const void* kp = o->key_is_raw ? (const void*)o->u.key : (const void*)o->u.pos;
        if (o->kind == 0)
            wqo_add_subscription(wm, o->world, o->peer, o->key_is_raw, kp);
        else if (o->kind == 1)
            wqo_remove_subscription(wm, o->world, o->peer, o->key_is_raw, kp);
        else if (o->world == 0xFFFFFFFFu)
            wqo_remove_peer(wm, o->peer); /* WorldMap::remove_peer */
        else {
            area_map* am = wm_get(wm, o->world); /* AreaMap::remove_peer on one world */
            if (am) am_remove_peer(am, o->peer);
        }
    }
}

/* handle_local_message after validation, local_message.rs:52-86, plus the replication decode
 * fallback (replication.rs:34-43: unknown codes are ExceptSelf). */
size_t wqo_route(const wqo_world_map* wm, const double* pos, const int64_t* keys,
                 const uint32_t* world, const uint32_t* sender, const uint8_t* repl, size_t M,
                 uint32_t* offsets, uint32_t* peers, size_t cap, uint64_t* n_candidates) {
    size_t P = 0;
    uint64_t F = 0;
    for (size_t m = 0; m < M; ++m) {
        if (offsets) offsets[m] = (uint32_t)P;
        const area_map* am = wm_get(wm, world[m]);
        if (!am) continue; /* :52-56 no subscriptions in this world */
        int64_t k[3];
        if (keys)
            memcpy(k, keys + 3 * m, sizeof(k));
        else
            to_cube_area(0, pos + 3 * m, wm->cube_size, k);
        const cube_slot* c = cm_find(&am->map, k);
        if (!c) continue; /* get_subscribed_peers -> empty_set */
        uint32_t me = sender[m];
        uint8_t r = repl[m];
        F += c->set.n;
        for (uint32_t i = 0; i < c->set.n; ++i) {
            uint32_t p = c->set.v[i];
            int keep = (r == 1) ? 1 : (r == 2) ? (p == me) : (p != me);
            if (!keep) continue;
            if (peers && P < cap) peers[P] = p;
            P++;
        }
    }
    if (offsets) offsets[M] = (uint32_t)P;
    if (n_candidates) *n_candidates = F;
    return P;
}

/* cpu_server_faithful_1t: wqo_route per message, then what
 * PeerMap::broadcast_to does with the recipients (worldql_server/src/transport/peer_map.rs:151-163):
 * collect them into a new hash set (:156), then filter EVERY connected peer of the PeerMap against
 * it (:157-160, O(|PeerMap|) per message). connected[0 .. n_connected) is the PeerMap's iteration
 * order; the output per message is in that order. Returns P (pairs actually sent). */
size_t wqo_route_faithful(const wqo_world_map* wm, const double* pos, const uint32_t* world,
                          const uint32_t* sender, const uint8_t* repl, size_t M, const uint32_t* connected,
                          size_t n_connected, uint32_t* offsets, uint32_t* peers, size_t cap) {
    size_t P = 0;
    uint32_t* tmp = NULL;
    size_t tcap = 0;
    uint32_t* set = NULL; /* open addressing, 0xFFFFFFFF = empty; rebuilt per message like AHashSet::collect */
    size_t scap = 0;
    for (size_t m = 0; m < M; ++m) {
        if (offsets) offsets[m] = (uint32_t)P;
        const size_t n = wqo_route(wm, pos + 3 * m, NULL, world + m, sender + m, repl + m, 1, NULL, NULL, 0, NULL);
        if (!wm_get(wm, world[m])) continue; /* local_message.rs:52-56: no broadcast at all */
        /* otherwise broadcast_to runs even for an empty recipient set (:60-86), scanning the map */
        if (n > tcap) {
            tcap = 2 * n;
            tmp = (uint32_t*)realloc(tmp, tcap * sizeof(uint32_t));
        }
        if (n) wqo_route(wm, pos + 3 * m, NULL, world + m, sender + m, repl + m, 1, NULL, tmp, n, NULL);
        size_t need = 16;
        while (need < 2 * n) need <<= 1;
        if (need > scap) {
            scap = need;
            set = (uint32_t*)realloc(set, scap * sizeof(uint32_t));
        }
        memset(set, 0xFF, need * sizeof(uint32_t));
        for (size_t i = 0; i < n; ++i) {
            size_t h = (tmp[i] * 0x9E3779B1u) & (need - 1);
            while (set[h] != 0xFFFFFFFFu && set[h] != tmp[i]) h = (h + 1) & (need - 1);
            set[h] = tmp[i];
        }
        for (size_t j = 0; j < n_connected; ++j) {
            const uint32_t q = connected[j];
            size_t h = (q * 0x9E3779B1u) & (need - 1);
            while (set[h] != 0xFFFFFFFFu && set[h] != q) h = (h + 1) & (need - 1);
            if (set[h] == q) {
                if (peers && P < cap) peers[P] = q;
                P++;
            }
        }
    }
    if (offsets) offsets[M] = (uint32_t)P;
    free(tmp);
    free(set);
    return P;
}

/* C5 (an extension the reference does not have): handle_local_message's
 * recipients (wqo_route) intersected with the exact Euclidean radius predicate
 *   dx = mx - px; dy = my - py; dz = mz - pz; keep iff (dx*dx + dy*dy) + dz*dz <= r*r
 * evaluated left to right in f64 with no FMA contraction (this file is built -ffp-contract=off).
 * peer_pos holds n_pos peers x 3; a peer id >= n_pos (no known position) is never within range,
 * and NaN compares false. Messages carry positions (no raw keys). */
size_t wqo_route_radius(const wqo_world_map* wm, const double* pos, const uint32_t* world, const uint32_t* sender,
                        const uint8_t* repl, size_t M, const double* peer_pos, size_t n_pos, double radius,
                        uint32_t* offsets, uint32_t* peers, size_t cap, uint64_t* n_candidates) {
    size_t P = 0;
    uint64_t F = 0;
    const double r2 = radius * radius;
    for (size_t m = 0; m < M; ++m) {
        if (offsets) offsets[m] = (uint32_t)P;
        const area_map* am = wm_get(wm, world[m]);
        if (!am) continue;
        int64_t k[3];
        to_cube_area(0, pos + 3 * m, wm->cube_size, k);
        const cube_slot* c = cm_find(&am->map, k);
        if (!c) continue;
        const uint32_t me = sender[m];
        const uint8_t r = repl[m];
        F += c->set.n;
        for (uint32_t i = 0; i < c->set.n; ++i) {
            const uint32_t p = c->set.v[i];
            int keep = (r == 1) ? 1 : (r == 2) ? (p == me) : (p != me);
            if (!keep || p >= n_pos) continue;
            const double dx = pos[3 * m] - peer_pos[3 * (size_t)p];
            const double dy = pos[3 * m + 1] - peer_pos[3 * (size_t)p + 1];
            const double dz = pos[3 * m + 2] - peer_pos[3 * (size_t)p + 2];
            const double d2 = dx * dx + dy * dy + dz * dz;
            if (!(d2 <= r2)) continue;
            if (peers && P < cap) peers[P] = p;
            P++;
        }
    }
    if (offsets) offsets[M] = (uint32_t)P;
    if (n_candidates) *n_candidates = F;
    return P;
}

/* handle_global_message for a named world (global_message.rs:36-84): the recipients are
 * AreaMap::get_subscribed_any_peers (area_map.rs:65-67) of the world, if it exists, under the same
 * replication filter as a LocalMessage. (The "@global" broadcast to every connected peer,
 * global_message.rs:18-35, is a PeerMap operation outside the subscription table.) */
size_t wqo_route_global(const wqo_world_map* wm, const uint32_t* world, const uint32_t* sender, const uint8_t* repl,
                        size_t M, uint32_t* offsets, uint32_t* peers, size_t cap) {
    size_t P = 0;
    for (size_t m = 0; m < M; ++m) {
        if (offsets) offsets[m] = (uint32_t)P;
        const area_map* am = wm_get(wm, world[m]);
        if (!am) continue; /* :50-54 */
        const uint32_t me = sender[m];
        const uint8_t r = repl[m];
        for (size_t i = 0; i < am->subscribed_peers.cap; ++i) {
            if (am->subscribed_peers.st[i] != SLOT_FULL) continue;
            const uint32_t p = am->subscribed_peers.key[i];
            int keep = (r == 1) ? 1 : (r == 2) ? (p == me) : (p != me);
            if (!keep) continue;
            if (peers && P < cap) peers[P] = p;
            P++;
        }
    }
    if (offsets) offsets[M] = (uint32_t)P;
    return P;
}

void wqo_counts(const wqo_world_map* wm, uint64_t* n_entries, uint64_t* n_cubes) {
    uint64_t e = 0, c = 0;
    for (size_t i = 0; i < wm->cap; ++i) {
        const area_map* am = wm->w[i].am;
        if (!am) continue;
        for (size_t j = 0; j < am->map.cap; ++j)
            if (am->map.s[j].st == SLOT_FULL && am->map.s[j].set.n) {
                c++;
                e += am->map.s[j].set.n;
            }
    }
    *n_entries = e;
    *n_cubes = c;
}

/* Checker for large ticks: routes every message like wqo_route (or wqo_route_radius when
 * peer_pos != NULL), sorts its recipients ascending and compares them with the message's slice of
 * a candidate CSR (got_offsets[M+1], got_peers[], ascending per message, as the GPU path writes
 * it). Returns the number of messages that differ; *first_bad (nullable) gets the first one, or M. */
static int cmp_u32(const void* a, const void* b) {
    const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return (x > y) - (x < y);
}

size_t wqo_route_check(const wqo_world_map* wm, const double* pos, const int64_t* keys, const uint32_t* world,
                       const uint32_t* sender, const uint8_t* repl, size_t M, const double* peer_pos, size_t n_pos,
                       double radius, const uint32_t* got_offsets, const uint32_t* got_peers, size_t* first_bad) {
    size_t bad = 0, first = M, cap = 1024;
    uint32_t* buf = (uint32_t*)malloc(cap * sizeof(uint32_t));
    uint32_t off[2];
    for (size_t m = 0; m < M; ++m) {
        const double* pm = pos ? pos + 3 * m : NULL;
        const int64_t* km = keys ? keys + 3 * m : NULL;
        size_t n = peer_pos ? wqo_route_radius(wm, pm, world + m, sender + m, repl + m, 1, peer_pos, n_pos, radius,
                                               off, buf, cap, NULL)
                            : wqo_route(wm, pm, km, world + m, sender + m, repl + m, 1, off, buf, cap, NULL);
        if (n > cap) {
            while (cap < n) cap *= 2;
            buf = (uint32_t*)realloc(buf, cap * sizeof(uint32_t));
            n = peer_pos ? wqo_route_radius(wm, pm, world + m, sender + m, repl + m, 1, peer_pos, n_pos, radius, off,
                                            buf, cap, NULL)
                         : wqo_route(wm, pm, km, world + m, sender + m, repl + m, 1, off, buf, cap, NULL);
        }
        qsort(buf, n, sizeof(uint32_t), cmp_u32);
        const size_t g0 = got_offsets[m], g1 = got_offsets[m + 1];
        int same = g1 >= g0 && g1 - g0 == n && (n == 0 || memcmp(buf, got_peers + g0, n * sizeof(uint32_t)) == 0);
        if (!same) {
            if (first == M) first = m;
            bad++;
        }
    }
    free(buf);
    if (first_bad) *first_bad = first;
    return bad;
}
