/*
 * wq_oracle.h — CPU restatement of the reference routing path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline. The product path
 * (worldql_server_amd/) never links or calls it.
 *
 * Parity pin: the reference (Rust) cannot be built here (no cargo/rustc),
 * so this restatement is pinned by the reference's own unit-test vectors, committed in
 * tests/golden/reference_kats.json (cube_area.rs:102-175, round.rs:28-76,
 * area_map.rs:154-254, world_names.rs:127-171), plus an independent numpy restatement
 * (oracle/oracle.py) cross-checked on random f64 bit patterns.
 */
#ifndef WQ_ORACLE_H
#define WQ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* worldql_server/src/utils/round.rs:1-13 */
double wqo_round_by_multiple(double n, double multiple);
/* worldql_server/src/subscriptions/cube_area.rs:23-44 */
int64_t wqo_coord_clamp(double coord, uint16_t size);
/* cube_area.rs:50-56 applied to n coordinates (x,y,z interleaved or not: per coordinate) */
void wqo_quantize(const double* coords, size_t n, uint16_t size, int64_t* out);

typedef struct wqo_world_map wqo_world_map;

/* world_map.rs:17-22 */
wqo_world_map* wqo_create(uint16_t cube_size);
void wqo_destroy(wqo_world_map* wm);
/* world_map.rs:31-36 get_mut (creates the AreaMap lazily, also on unsubscribe) +
 * area_map.rs:72-85 add_subscription. Returns 1 if newly added. */
int wqo_add_subscription(wqo_world_map* wm, uint32_t world, uint32_t peer, int key_is_raw,
                         const void* key_or_pos);
/* world_map.rs:31-36 + area_map.rs:88-119 remove_subscription. Returns 1 if removed. */
int wqo_remove_subscription(wqo_world_map* wm, uint32_t world, uint32_t peer, int key_is_raw,
                            const void* key_or_pos);
/* world_map.rs:41-61 -> area_map.rs:124-135. Returns 1 if removed from any world. */
int wqo_remove_peer(wqo_world_map* wm, uint32_t peer);
/* area_map.rs:33-41; 0 if the world does not exist (world_map.rs:25-27 get -> None) */
int wqo_is_subscribed(const wqo_world_map* wm, uint32_t world, uint32_t peer, int key_is_raw,
                      const void* key_or_pos);
/* area_map.rs:46-48 */
int wqo_is_subscribed_any(const wqo_world_map* wm, uint32_t world, uint32_t peer);
/* area_map.rs:65-67 for one world; returns count, writes up to cap ids (unsorted). */
size_t wqo_world_peers(const wqo_world_map* wm, uint32_t world, uint32_t* out, size_t cap);

/* Apply an op array in order (same 40-byte layout as wq_op in include/wq_router.h). */
void wqo_apply_ops(wqo_world_map* wm, const void* ops, size_t n);

/* local_message.rs:52-86 for M messages (already validated on the host, as the ABI requires).
 * keys may be NULL (then pos is quantised). Writes message-major CSR: offsets[M+1],
 * peers[..] in the AHashSet-like iteration order of this restatement (unsorted).
 * Returns P; writes at most cap peers (P may exceed cap). n_candidates (nullable) gets F. */
size_t wqo_route(const wqo_world_map* wm, const double* pos, const int64_t* keys,
                 const uint32_t* world, const uint32_t* sender, const uint8_t* repl, size_t M,
                 uint32_t* offsets, uint32_t* peers, size_t cap, uint64_t* n_candidates);

/* cpu_server_faithful_1t: wqo_route + PeerMap::broadcast_to's per-message recipient set and
 * O(|PeerMap|) connected-peer scan (peer_map.rs:151-163); output per message in connected[] order. */
size_t wqo_route_faithful(const wqo_world_map* wm, const double* pos, const uint32_t* world,
                          const uint32_t* sender, const uint8_t* repl, size_t M, const uint32_t* connected,
                          size_t n_connected, uint32_t* offsets, uint32_t* peers, size_t cap);

/* C5 extension: wqo_route's recipients with the exact radius predicate
 * (dx*dx + dy*dy) + dz*dz <= r*r in f64, d = message position - peer position; peers >= n_pos
 * have no position and are dropped. */
size_t wqo_route_radius(const wqo_world_map* wm, const double* pos, const uint32_t* world, const uint32_t* sender,
                        const uint8_t* repl, size_t M, const double* peer_pos, size_t n_pos, double radius,
                        uint32_t* offsets, uint32_t* peers, size_t cap, uint64_t* n_candidates);
/* GlobalMessage to a named world, global_message.rs:36-84 (get_subscribed_any_peers + replication). */
size_t wqo_route_global(const wqo_world_map* wm, const uint32_t* world, const uint32_t* sender, const uint8_t* repl,
                        size_t M, uint32_t* offsets, uint32_t* peers, size_t cap);

/* Fast mode for the test checker (call on an empty map): remove_subscription answers its
 * O(#cubes) "any other cube?" scan (area_map.rs:113-116) from per-peer cube counts — the same
 * result (see wq_oracle.c), so full-size churn configs can be checked. Returns -1 if not empty.
 * The timed CPU baseline never sets it. */
int wqo_set_fast(wqo_world_map* wm, int fast);
/* Routes each message (wqo_route, or wqo_route_radius when peer_pos != NULL), sorts its recipients
 * and compares them with got_offsets / got_peers (ascending per message). Returns the number of
 * differing messages; *first_bad gets the first (or M). */
size_t wqo_route_check(const wqo_world_map* wm, const double* pos, const int64_t* keys, const uint32_t* world,
                       const uint32_t* sender, const uint8_t* repl, size_t M, const double* peer_pos, size_t n_pos,
                       double radius, const uint32_t* got_offsets, const uint32_t* got_peers, size_t* first_bad);
/* Stats for tests: number of live (world,cube,peer) entries and of non-empty cubes. */
void wqo_counts(const wqo_world_map* wm, uint64_t* n_entries, uint64_t* n_cubes);

#ifdef __cplusplus
}
#endif
#endif
