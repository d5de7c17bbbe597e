/*
 * wq_router.h — C ABI of the MI355X-native WorldQL spatial message-routing path.
 *
 * This is the drop-in boundary for the reference server's subscription table
 * (worldql_server/src/subscriptions/{world_map,area_map,cube_area}.rs) and the
 * LocalMessage / AreaSubscribe / AreaUnsubscribe handlers that drive it
 * (worldql_server/src/processing/{local_message,area_subscribe,area_unsubscribe}.rs).
 * The reference has no FFI for this path (it is plain Rust methods);
 * each entry point below names the Rust method(s) it replaces, and INTEGRATION.md shows
 * the `extern "C"` block a `worldql_gpu` crate would declare to bind them.
 *
 * Conventions
 *   - plain pointers and sizes only; every function returns an int status (WQ_OK = 0,
 *     negative WQ_E_* on failure). No exception or panic crosses the ABI.
 *   - peers are dense uint32 ids (the Rust side keeps the Uuid <-> u32 map);
 *     worlds are dense uint32 ids interned on the host from the *sanitized* world name
 *     (worldql_server/src/utils/world_names.rs:54-87). WQ_WORLD_INVALID is reserved.
 *   - a handle is owned by one thread (Send, not Sync), mirroring the single owner task of
 *     WorldMap in worldql_server/src/processing/thread.rs:113-148.
 *   - functions without the `_device` suffix take HOST pointers and are synchronous;
 *     `_device` variants take DEVICE pointers and are asynchronous on the handle's stream.
 */
#ifndef WQ_ROUTER_H
#define WQ_ROUTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define WQ_OK 0
#define WQ_E_INVALID (-1)  /* bad argument (null handle, cube_size 0, reserved world id ...) */
#define WQ_E_OOM (-2)      /* device allocation failed */
#define WQ_E_HIP (-3)      /* HIP runtime error (message in wq_last_error) */
#define WQ_E_RCCL (-4)     /* the multi-GPU exchange failed (RCCL, hub timeout, caller callback) */
#define WQ_E_CAPACITY (-5) /* caller's output buffer too small; required size reported */
#define WQ_E_NODEV (-6)    /* no usable gfx950 device: the path never falls back to the CPU */
#define WQ_E_TIMEOUT (-7)  /* a bounded in-kernel spin gave up (must never happen) */

/* ---- op kinds (wq_op.kind) ---- */
#define WQ_OP_SUBSCRIBE 0   /* AreaMap::add_subscription, area_map.rs:72-85 */
#define WQ_OP_UNSUBSCRIBE 1 /* AreaMap::remove_subscription, area_map.rs:88-119 */
#define WQ_OP_REMOVE_PEER 2 /* world == WQ_WORLD_INVALID: WorldMap::remove_peer (world_map.rs:41-61);
                             otherwise that world only: AreaMap::remove_peer (area_map.rs:124-135) */

/* ---- replication codes, wire values of WorldQLFB_generated.rs:176-188 ---- */
#define WQ_REPL_EXCEPT_SELF 0    /* default; also every unknown code (replication.rs:40) */
#define WQ_REPL_INCLUDING_SELF 1
#define WQ_REPL_ONLY_SELF 2

#define WQ_WORLD_INVALID 0xFFFFFFFFu

typedef struct wq_router wq_router;

/* One subscription-table op (40 bytes). key_is_raw = 1 means `key` is a CubeArea used as-is
 * (impl ToCubeArea for CubeArea, cube_area.rs:65-70); 0 means `pos` is a Vector3 quantised
 * by CubeArea::from_vector3 (cube_area.rs:50-56). */
typedef struct wq_op {
    uint32_t world;
    uint32_t peer;
    uint8_t kind;
    uint8_t key_is_raw;
    uint8_t pad_[6];
    union {
        double pos[3];
        int64_t key[3];
    } u;
} wq_op;

typedef struct wq_stats {
    uint64_t n_entries;     /* live (world, cube, peer) subscriptions */
    uint64_t n_cubes;       /* occupied (world, cube) buckets */
    uint64_t n_any;         /* distinct (world, peer) pairs = sum of |subscribed_peers| */
    uint64_t table_slots;   /* open-addressed slot count (power of two) */
    uint64_t hash_fallbacks;/* builds that hit a 64-bit hash collision and took the exact path */
    uint32_t cube_size;
    int32_t device;
} wq_stats;

/* Per-call route counters written by the route kernel (device memory, see wq_route_tick_device). */
typedef struct wq_route_counters {
    uint64_t n_pairs;      /* P: (message, peer) pairs after the replication filter */
    uint64_t n_candidates; /* F: peers read from the probed buckets before the filter */
    uint32_t overflow;     /* 1 if P exceeded the caller's capacity (outputs truncated) */
    uint32_t error;        /* 4: a bounded spin gave up (WQ_E_TIMEOUT); 2: P > 2^32-1 (WQ_E_CAPACITY);
                              8: the table is missing an incremental batch the device could not
                              apply (re-applied by the next wq_apply* / query call) */
} wq_route_counters;

/* ---- pinned host memory for the host-array entry points: buffers from wq_host_alloc move over
 * PCIe by DMA without a staging copy (pageable buffers work too, at a fraction of the rate). */
int wq_host_alloc(size_t bytes, void** out);
int wq_host_free(void* p);

/* ---- lifetime: replaces WorldMap::new (world_map.rs:17-22) ---- */
int wq_router_create(uint16_t cube_size, int device, wq_router** out);
/* The same table over n_gpus GPUs behind ONE handle (SURVEY.md §8(b) wq_router_create(cube_size,
 * n_gpus, devices, out)); the reference's single owner (thread.rs:119) keeps its one WorldMap.
 * Inside: one cube-hash shard per device (devices may repeat), attached to an in-process exchange,
 * driven by one worker thread each; every call below gives the one-table result:
 *   wq_apply_ops[_device], wq_remove_peers   the whole op stream to every shard (each keeps its cubes)
 *   wq_route_tick[_device]                   the sharded tick over G slices of the messages, CSR
 *                                            concatenated in message order (n_candidates = P)
 *   wq_is_subscribed[_any], wq_world_peers,  shard answers combined (any-keys merged on devices[0])
 *   wq_route_global[_device], wq_get_stats
 *   wq_set_radius, wq_set_peer_positions[_device], wq_set_fanout_hint, wq_route_health: every shard
 * Device-pointer calls take arrays on devices[0], ordered after the handle's stream (wq_set_stream),
 * and are synchronous on return — except wq_apply_ops_device, which keeps the single-GPU contract:
 * an invalid batch is not applied and shows as error bit 16 of wq_route_health (the call returns
 * WQ_OK); on the replicate layout it is also asynchronous. The cube-hash layout partitions a device
 * batch by owner on devices[0] (one read-back of the per-shard counts). The sharded entry points
 * (wq_shard_*, wq_sharded_*) and the instrumentation hooks are for single-device handles. */
int wq_router_create_multi(uint16_t cube_size, int n_gpus, const int* devices, wq_router** out);
/* The same with the layout chosen (wq_router_create_multi = WQ_MULTI_CUBE_HASH):
 *   WQ_MULTI_CUBE_HASH  the table partitioned by cube hash, as above (tables beyond one GPU's HBM);
 *   WQ_MULTI_REPLICATE  every device holds the WHOLE table and routes its own slice of a tick with
 *                       the single-GPU tick — no exchange at all (C3's table is ~10 GB of 288 GB).
 *                       Every op is applied on every device (the op stream is the only thing all
 *                       devices see); wq_apply_ops_device stays asynchronous; queries go to device 0.
 * Results are the one-table results either way. */
#define WQ_MULTI_CUBE_HASH 0
#define WQ_MULTI_REPLICATE 1
int wq_router_create_multi_mode(uint16_t cube_size, int n_gpus, const int* devices, int mode, wq_router** out);
/* Sub-handles behind a handle (1 for wq_router_create), and the layout (-1 for a single-GPU handle). */
int wq_multi_info(wq_router* h, uint32_t* n_gpus);
int wq_multi_mode(wq_router* h, int* mode);
/* The scaling form of a multi-GPU tick: every device routes the messages it ingested and keeps its
 * CSR (no pair crosses to devices[0]). in[g] = the messages on devices[g] (device pointers there,
 * complete before the call; keys or positions as wq_route_tick); out[g] = views into the handle's
 * workspace on devices[g] (a staging of their own), valid until the next wq_route_tick_slices_device
 * call on the handle or its destruction — every other call (routes, queries, op batches) leaves
 * them intact: offsets[n_msgs + 1] (from 0),
 * peers[n_pairs], msgs[n_pairs] (the index within the slice; NULL unless with_msgs). Per message
 * the recipients are exactly wq_route_tick's for the same message on one table. Synchronous. */
typedef struct wq_msg_slice {
    const double* d_pos;
    const int64_t* d_keys;
    const uint32_t* d_world;
    const uint32_t* d_sender;
    const uint8_t* d_repl;
    uint64_t n_msgs;
} wq_msg_slice;
typedef struct wq_slice_view {
    int32_t device;
    uint32_t pad_;
    uint64_t n_msgs;
    uint64_t n_pairs;
    const uint32_t* offsets;
    const uint32_t* peers;
    const uint32_t* msgs;
} wq_slice_view;
int wq_route_tick_slices_device(wq_router* h, const wq_msg_slice* in, int with_msgs, wq_slice_view* out);
int wq_router_destroy(wq_router* h);
const char* wq_last_error(const wq_router* h);
/* Use the caller's HIP stream (hipStream_t as void*); NULL restores the handle's own stream. */
int wq_set_stream(wq_router* h, void* hip_stream);
int wq_get_stats(wq_router* h, wq_stats* out);

/* ---- table mutation: AreaSubscribe / AreaUnsubscribe / disconnect ----
 * Ops are applied in ARRAY ORDER with the reference's sequential semantics
 * (processing/thread.rs:122-146): for each (world, cube, peer) the last op wins, and a
 * REMOVE_PEER op removes every subscription its peer holds at that point.
 * Replaces area_subscribe.rs:137-138 / area_unsubscribe.rs:189-190 -> AreaMap::{add,remove}_subscription
 * and thread.rs:124-125 -> WorldMap::remove_peer. */
int wq_apply_ops(wq_router* h, const wq_op* ops, size_t n);
/* The same for a batch already in device memory (e.g. assembled by the caller's own kernels):
 * subscribe / unsubscribe ops only — a REMOVE_PEER op or the reserved world id fails the whole
 * batch with WQ_E_INVALID before anything changes (use wq_remove_peers for disconnects).
 * Asynchronous: an incremental batch (up to 1/4 of the table's entries) is enqueued on the
 * handle's stream, before any later tick, and the call returns without waiting for the GPU; the
 * NEXT call on the handle folds its status in (waiting only for that batch, not for later work).
 * Keep d_ops unchanged until that next call has returned: a batch the device could not apply
 * (an op whose key has no packed form — NaN / huge coordinates, off-grid raw keys, world ids
 * >= 2^24 - 1 — or list space exhausted) is re-applied from it by the rebuild then, and routes
 * issued in between report error bit 8 (WQ stale table) in their counters and in
 * wq_route_health. A batch holding an invalid op (REMOVE_PEER kind, reserved world) is not applied at
 * all (the table stays as before it); the next call on the handle still does its own work in full
 * and leaves the rejection in wq_last_error and as error bit 16 of wq_route_health. */
int wq_apply_ops_device(wq_router* h, const wq_op* d_ops, size_t n);
/* WorldMap::remove_peer for n peers (every world), world_map.rs:41-61. */
int wq_remove_peers(wq_router* h, const uint32_t* peers, size_t n);

/* ---- the hot path: one tick of LocalMessages ----
 * Replaces the per-message body of handle_local_message (local_message.rs:52-86):
 * world lookup -> Vector3::to_cube_area -> AreaMap::get_subscribed_peers -> replication filter.
 * Validation (@global, missing position, bad world name: local_message.rs:17-50) stays on the
 * host, before the call. Output: message-major CSR, offsets[M+1] and peers[P]; msgs[P]
 * (nullable) repeats the message index of each pair. Pair order inside one message is
 * ascending peer id (the reference's AHashSet order is random per process: compare sets).
 * keys (nullable, M x 3 int64) replaces pos with raw CubeArea keys (ToCubeArea for CubeArea). */
int wq_route_tick(wq_router* h, const double* pos, const int64_t* keys, const uint32_t* world,
                  const uint32_t* sender, const uint8_t* repl, size_t n_msgs, uint32_t* offsets,
                  uint32_t* peers, uint32_t* msgs, size_t capacity, size_t* n_pairs);
/* Asynchronous form on device pointers; nothing is read back. counters (device pointer to a
 * wq_route_counters) receives P, F and the overflow / error flags (also kept sticky for
 * wq_route_health). Pairs beyond `capacity` are not written. */
int wq_route_tick_device(wq_router* h, const double* d_pos, const int64_t* d_keys,
                         const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                         size_t n_msgs, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs,
                         size_t capacity, wq_route_counters* d_counters);

/* ---- C5: exact radius filter after the cube broadphase ----
 * An extension the reference does not have (it stores no peer positions). With a radius > 0 set,
 * every subsequent tick keeps a (message, peer) pair only if additionally
 *     dx = mx - px; dy = my - py; dz = mz - pz;   (dx*dx + dy*dy) + dz*dz <= radius*radius
 * evaluated left to right in f64 without FMA contraction, m = the message position, p = the
 * peer's position from the latest wq_set_peer_positions; a peer id >= n_peers has no position and
 * is dropped. Ticks with the filter on take message positions (keys must be NULL).
 * radius <= 0 or NaN turns the filter off. The handle keeps the positions (24 B per peer) and an
 * f32 copy (16 B per peer) that decides every pair whose f64 result it can bound; the rest read
 * the f64 copy, so results are exactly the f64 predicate's. The _device form reads d_pos on the
 * handle's stream (asynchronous). */
int wq_set_peer_positions(wq_router* h, const double* pos, size_t n_peers);
int wq_set_peer_positions_device(wq_router* h, const double* d_pos, size_t n_peers);
int wq_set_radius(wq_router* h, double radius);

/* ---- tick shape: the caller's expected recipients per message (e.g. its previous tick's
 * n_pairs / M; no reference counterpart — the Rust loop routes one message at a time,
 * thread.rs:125-146). At >= WQ_HEAVY_FANOUT the tick runs as count / scan / emit launches, whose
 * emit writes each block's outputs straight to HBM without holding a block that waits on its
 * predecessors (C3: 2.18 -> 1.76 ms); below it, the single launch (C2). Results are identical
 * either way. Until the caller sets a hint, the host-array wq_route_tick sets it itself from each
 * tick's n_pairs / M (device-pointer ticks never read their counters back, so they keep the last
 * value; the initial one is the single launch). */
#define WQ_HEAVY_FANOUT 16.0
/* A negative or NaN hint hands the choice back to the automatic rule (host-array ticks of >= 256
 * messages set the next tick's shape from their own n_pairs / M). */
int wq_set_fanout_hint(wq_router* h, double pairs_per_message);

/* ---- F1: GlobalMessage to a named world (worldql_server/src/processing/global_message.rs:36-84)
 * Message m goes to every peer subscribed to at least one cube of world[m]
 * (AreaMap::get_subscribed_any_peers, area_map.rs:65-67), in ascending peer order, filtered by
 * repl[m] like LocalMessage: ExceptSelf drops sender[m], OnlySelf keeps only sender[m] (if it is
 * subscribed in that world), IncludingSelf keeps every peer. A world with no subscriptions yields
 * nothing (global_message.rs:50-54). Output, capacity and counters as wq_route_tick. The host-array
 * form rejects WQ_WORLD_INVALID (WQ_E_INVALID); the device form routes it to nobody. The "@global"
 * broadcast to every connected peer (global_message.rs:18-35) is a peer-map operation and has no
 * table entry point. */
int wq_route_global(wq_router* h, const uint32_t* world, const uint32_t* sender, const uint8_t* repl,
                    size_t n_msgs, uint32_t* offsets, uint32_t* peers, uint32_t* msgs, size_t capacity,
                    size_t* n_pairs);
int wq_route_global_device(wq_router* h, const uint32_t* d_world, const uint32_t* d_sender,
                           const uint8_t* d_repl, size_t n_msgs, uint32_t* d_offsets, uint32_t* d_peers,
                           uint32_t* d_msgs, size_t capacity, wq_route_counters* d_counters);

/* ---- queries (the reference uses these in its unit tests, area_map.rs:33-67) ---- */
/* AreaMap::is_peer_subscribed(uuid, cube), batched; key_or_pos is n x 3 (int64 if key_is_raw). */
int wq_is_subscribed(wq_router* h, size_t n, const uint32_t* world, const uint32_t* peer,
                     int key_is_raw, const void* key_or_pos, uint8_t* out);
/* AreaMap::is_peer_subscribed_any(uuid), batched. */
int wq_is_subscribed_any(wq_router* h, size_t n, const uint32_t* world, const uint32_t* peer,
                         uint8_t* out);
/* AreaMap::get_subscribed_any_peers() for one world (ascending ids). */
int wq_world_peers(wq_router* h, uint32_t world, uint32_t* out, size_t capacity, size_t* n_out);

/* ---- kernel (1) alone: CubeArea::coord_clamp over n coordinates (cube_area.rs:23-44) ---- */
int wq_quantize(const double* coords, size_t n, uint16_t cube_size, int64_t* out);
int wq_quantize_device(wq_router* h, const double* d_coords, size_t n, int64_t* d_out);

/* ---- multi-GPU: cube-hash ownership ----
 * The reference is single-process (one WorldMap owned by one task, thread.rs:113-148); these
 * entry points partition that one table over G GPUs without changing any result. Each (world,
 * cube) bucket has one owner shard in [0, G) computed from the QUANTISED key, so the owner
 * holds every subscription a message to that cube can reach. A sharded tick is
 *   wq_shard_messages_device -> all-to-all of the records (RCCL) -> wq_route_records_device on
 *   the owner -> all-to-all of per-message counts and peers back to the ingesting GPU.
 * These are the building blocks; the whole tick behind one call is wq_sharded_route_tick_device
 * (below), over RCCL, the in-process hub, or the caller's transport (wq_shard_attach_exchange;
 * tests/test_distributed.py and tests/test_gpu_sharded_native.py drive it over gloo). */
#define WQ_MAX_SHARDS 64
#define WQ_SHARD_ALL 0xFFFFFFFFu /* owner of a REMOVE_PEER op: every shard */

/* One message on the wire between GPUs (40 bytes): its quantised CubeArea (or, with flags &
 * WQ_REC_POS, the bits of its f64 position — what the owner's radius filter needs), world,
 * sender, index in the ingesting GPU's batch, and replication code. */
typedef struct wq_msg_rec {
    int64_t key[3];
    uint32_t world;
    uint32_t sender;
    uint32_t msg;
    uint8_t repl;
    uint8_t flags;
    uint8_t pad_[2];
} wq_msg_rec;
#define WQ_REC_POS 1u /* key[] holds the message position (double[3] bits); the owner quantises */

/* Owner shard of each op (host arrays); REMOVE_PEER ops get WQ_SHARD_ALL. Each shard applies,
 * in array order, the ops it owns plus every REMOVE_PEER (area_subscribe.rs / area_unsubscribe.rs
 * / thread.rs:124-125 on the owner). */
int wq_shard_ops(wq_router* h, const wq_op* ops, size_t n, uint32_t n_shards, uint32_t* owner);
/* Quantise (or take raw keys), compute owners and write the records grouped by owner, stable in
 * message order: d_out[M] and d_counts[n_shards] (device). Asynchronous on the handle's stream.
 * With the radius filter on (wq_set_radius) and positions given, the records carry the positions
 * (WQ_REC_POS) so the owner can filter; every shard then needs the peer positions. */
int wq_shard_messages_device(wq_router* h, const double* d_pos, const int64_t* d_keys,
                             const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                             size_t n_msgs, uint32_t n_shards, wq_msg_rec* d_out, uint32_t* d_counts);
/* wq_route_tick_device on received records (the owner side of a sharded tick). With the radius
 * filter on, records without WQ_REC_POS have no position and route to nobody. */
int wq_route_records_device(wq_router* h, const wq_msg_rec* d_recs, size_t n_msgs, uint32_t* d_offsets,
                            uint32_t* d_peers, uint32_t* d_msgs, size_t capacity,
                            wq_route_counters* d_counters);

/* ---- multi-GPU: sharded ticks behind the ABI ----
 * A handle becomes shard `rank` of G by attaching an exchange; afterwards
 *   wq_sharded_apply_ops            every shard is given the SAME op stream (the reference's one
 *                                   subscription task, thread.rs:122-146) and keeps the ops of the
 *                                   buckets it owns plus every REMOVE_PEER;
 *   wq_sharded_route_tick_device    every shard is given its OWN ingested messages; the call runs
 *                                   shard -> exchange -> route on the owners -> exchange back and
 *                                   returns, on each shard, exactly the CSR wq_route_tick_device would
 *                                   return for those messages on one GPU holding the whole table
 *                                   (offsets[M+1] and peers[P] in message order, msgs[P] optional).
 * The tick is collective: all G shards call it (M may be 0), each on its own thread or process.
 * Its exchanges are sized by budgets every shard derives from the previous tick's sizes (both ends
 * of a pair agree without a read-back), so it reads the device once, at its end, and is synchronous
 * on return; *n_pairs = P. The first tick, and a tick whose sizes outgrew a budget (every shard
 * learns it from the exchanged status words and all redo the tick), read the sizes back first. If
 * P > capacity the tick still completes (its peers are not left waiting), returns WQ_E_CAPACITY
 * with offsets written, and wq_sharded_copy_out re-copies the kept result into a larger buffer
 * without another exchange — as long as the table is unchanged since (WQ_E_INVALID otherwise).
 * Exchange failures return WQ_E_RCCL.
 * Exchanges: RCCL (one process per GPU, or several handles of one process), an in-process hub
 * (G handles of one process, peer copies over xGMI), or the caller's own all-to-all. */
#define WQ_RCCL_ID_BYTES 128
/* The caller's all-to-all: send_bytes[d] bytes to shard d from d_send (segments contiguous in
 * shard order), recv_bytes[s] bytes from shard s into d_recv (likewise); device pointers, ordered
 * after the work already queued on hip_stream. Returns 0 on success. */
typedef int (*wq_exchange_fn)(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv,
                              const size_t* recv_bytes, void* hip_stream);
typedef struct wq_hub wq_hub;
int wq_hub_create(uint32_t n_shards, wq_hub** out);
int wq_hub_destroy(wq_hub* hub);
int wq_shard_attach_hub(wq_router* h, wq_hub* hub, uint32_t rank);
/* RCCL: rank 0 makes the id (wq_rccl_unique_id), the caller distributes the 128 bytes, every rank
 * attaches (collective, blocks until all G have joined). librccl is loaded at run time. */
int wq_rccl_unique_id(uint8_t* id_out);
int wq_shard_attach_rccl(wq_router* h, uint32_t n_shards, uint32_t rank, const uint8_t* id);
int wq_shard_attach_exchange(wq_router* h, uint32_t n_shards, uint32_t rank, wq_exchange_fn fn, void* ctx);
int wq_shard_detach(wq_router* h);
int wq_shard_info(wq_router* h, uint32_t* n_shards, uint32_t* rank);
int wq_sharded_apply_ops(wq_router* h, const wq_op* ops, size_t n);
int wq_sharded_route_tick_device(wq_router* h, const double* d_pos, const int64_t* d_keys,
                                 const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                                 size_t n_msgs, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs,
                                 size_t capacity, size_t* n_pairs);
int wq_sharded_copy_out(wq_router* h, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs, size_t capacity);
/* The same tick without its end-of-tick read: it returns as soon as its work is enqueued (the GPU
 * never idles between back-to-back ticks) and writes its result to d_counters (device memory,
 * nullable) and the sticky wq_route_health words, as wq_route_tick_device does: n_pairs = P,
 * overflow = P > capacity (outputs truncated), error = the device bits of every shard's counters
 * and statuses (2, 4, 8 as for a single-GPU tick), 32 when some shard's local step failed, 64 when a
 * budget was too small — the tick's outputs are then NOT valid and the caller routes it again; every
 * shard sees the same bits. The budgets of a tick come from the tick two calls back: each call first
 * folds in the read-back of every earlier asynchronous tick but the latest (all shards fold the same
 * ticks, so both ends of every pair agree). A tick that must run exact (the first, or after a bit
 * 64) runs synchronously, as wq_sharded_route_tick_device does. A shard whose local step fails on a
 * budgeted tick still ends it asynchronously (its snapshot queued like every other shard's, so all
 * shards keep folding the same ticks) and returns its error code; the others see bit 32. Collective:
 * all G shards make the same sequence of sharded calls. wq_sharded_copy_out does not apply to an
 * asynchronous tick. The slot form only (not wq_debug_set_shard_form's expanded form). A result that
 * never arrives (60 s) returns WQ_E_TIMEOUT naming the tick, its ring slot and the sequence words. */
int wq_sharded_route_tick_async(wq_router* h, const double* d_pos, const int64_t* d_keys,
                                const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                                size_t n_msgs, uint32_t* d_offsets, uint32_t* d_peers, uint32_t* d_msgs,
                                size_t capacity, wq_route_counters* d_counters);
/* What crosses between GPUs in a sharded tick: each message as one 20-byte slot to its owner (two
 * for a key without a packed form), and back a 12-byte row reference per slot plus, per (owner,
 * ingesting shard), ONE copy of every cube list those messages hit — not the expanded (message,
 * peer) pairs (C3: a hotspot list of ~500 peers is hit by thousands of messages a tick). The
 * ingesting GPU expands the rows itself; with the radius filter on it also filters them there, where
 * the message positions are (every shard holds every peer position), so a hot cube costs its owner
 * one list copy per ingesting shard, however many messages hit it.
 * wq_shard_last_bytes: bytes this shard sent to / received from OTHER shards in its latest sharded
 * tick (the xGMI volume; the self segment is not counted). */
int wq_shard_last_bytes(wq_router* h, uint64_t* sent, uint64_t* received);
/* Slot ticks run exactly (the sizes read back twice: the first tick, or a redo after a tick outgrew
 * its budgets) and on budgets (one host read per tick, at its end), on this shard so far. */
int wq_shard_tick_stats(wq_router* h, uint64_t* exact, uint64_t* budgeted);
/* Test / tuning hook: 1 = the sharded tick sends 40-byte records and returns expanded pairs (the
 * earlier form; the owner filters by radius), 0 = slots, row references and pools (default).
 * Results are identical. */
int wq_debug_set_shard_form(wq_router* h, int expanded);
/* Test hook: the next sharded tick on this handle fails locally at step 1 (grouping its messages)
 * or 3 (routing what it owns) with WQ_E_INVALID, as a real local failure would: it still completes
 * every exchange of the tick, and every shard of the tick returns an error. 0 = off. */
int wq_debug_inject_shard_failure(wq_router* h, int step);

/* The owner-side form of the sharded tick ("pairs stay on the owner"):
 * the same collective shard -> exchange -> route, but the (message, peer) pairs are not sent back.
 * On return, *out describes what THIS shard routed — the R messages it owns, as the records it
 * received (recs[i].msg = the message's index in its ingesting shard's batch; records from source
 * shard s are recs[seg[s] .. seg[s+1])) with their recipients as a CSR (offsets[R + 1], peers[P]),
 * each message's peers ascending. Device pointers into the handle's workspace, valid until the
 * next sharded call on it. A transport that sends from the owner (or re-partitions by peer) needs
 * no return exchange: across the shards every message appears exactly once. */
typedef struct wq_owner_view {
    const wq_msg_rec* recs;
    const uint32_t* offsets;
    const uint32_t* peers;
    uint64_t n_recs;
    uint64_t n_pairs;
    uint32_t seg[WQ_MAX_SHARDS + 1];
} wq_owner_view;
int wq_sharded_route_owner_device(wq_router* h, const double* d_pos, const int64_t* d_keys,
                                  const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                                  size_t n_msgs, wq_owner_view* out);

/* The owner form on budgeted 20-byte slots (first option; the per-slot
 * lookup is area_map.rs:52-60 / local_message.rs:52-86): every message goes to the shard owning its
 * cube as one slot (two for a key without a packed form), this shard's own messages through the
 * self segment. The slot exchange is the tick's only collective step. Each owner routes the slots it
 * received and keeps the pairs. The exchange sizes are budgets from the previous tick (the first
 * tick, or one after a short budget anywhere, runs exact), so only the end of the tick reads back.
 * Collective: every shard calls it. Received segment of source s: slots [seg[s], seg[s+1]), in
 * the order of s's sent segment for this shard, [send_seg[me], send_seg[me+1]) on s. So slot
 * seg[s] + k carries the message send_perm[send_seg[me] + k] of shard s (UINT32_MAX: padding, or
 * the second slot of a wide key). Padding and second slots route to nobody. The pairs are a CSR
 * over the received slots: slot i's recipients are peers[offsets[i] .. offsets[i+1]). Device
 * pointers into the handle's workspace stay valid until the next sharded call. No radius filter
 * here (wq_sharded_route_owner_device has it). */
#define WQ_SLOT_WORDS 5
typedef struct wq_owner_slot_view {
    const uint32_t* slots;      /* n_slots x WQ_SLOT_WORDS words, as received */
    const uint32_t* offsets;    /* [n_slots + 1] */
    const uint32_t* peers;      /* [n_pairs] */
    const uint32_t* send_perm;  /* this shard's sent slots -> its message index */
    uint64_t n_slots;
    uint64_t n_pairs;
    uint32_t seg[WQ_MAX_SHARDS + 1];       /* received segments, per source shard */
    uint32_t send_seg[WQ_MAX_SHARDS + 1];  /* sent segments, per owner shard */
} wq_owner_slot_view;
int wq_sharded_route_owner_slots(wq_router* h, const double* d_pos, const int64_t* d_keys,
                                 const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                                 size_t n_msgs, wq_owner_slot_view* out);
/* The same without the end-of-tick read (as wq_sharded_route_tick_async): a budgeted tick returns
 * once enqueued, with out->n_pairs = UINT64_MAX; P and the status bits land in d_counters (device;
 * nullable) and the sticky health words (error bit 64: a budget was too small, the tick's outputs
 * are not valid and the next call runs exact; overflow: the handle's pair buffer was short, the
 * outputs are truncated and the buffer grows for the tick after next). A tick that must run exact
 * (the first, one after a short budget, one after the slot tick) runs synchronously and fills
 * n_pairs. A local failure on a budgeted tick ends it asynchronously all the same and returns the
 * error. The view's arrays are rewritten by the next tick on the handle's stream. */
int wq_sharded_route_owner_slots_async(wq_router* h, const double* d_pos, const int64_t* d_keys,
                                       const uint32_t* d_world, const uint32_t* d_sender, const uint8_t* d_repl,
                                       size_t n_msgs, wq_route_counters* d_counters, wq_owner_slot_view* out);

/* ---- F2: per-peer send lists (PeerMap::broadcast_to, worldql_server/src/transport/peer_map.rs:151-163)
 * The transpose of a tick's message-major CSR for a transport that batches per peer: for every
 * peer p < n_peers whose bit is set in d_connected (bit p % 32 of word p / 32; NULL = every peer
 * connected) the messages it must receive, ascending — the reference's "recipients intersected
 * with the connected peers". d_peer_offsets[n_peers + 1]; d_msgs_out[n_pairs] (the kept ones
 * first: d_peer_offsets[n_peers] of them). n_pairs = d_offsets[n_msgs]. Asynchronous. */
int wq_peer_major_device(wq_router* h, const uint32_t* d_offsets, const uint32_t* d_peers, size_t n_msgs,
                         size_t n_pairs, const uint32_t* d_connected, uint32_t n_peers,
                         uint32_t* d_peer_offsets, uint32_t* d_msgs_out);

/* ---- health of asynchronous ticks ----
 * OR of wq_route_counters.error (error_bits) and of .overflow over every route / global call since
 * the previous wq_route_health on this handle; reading clears them (synchronises the stream). A
 * normal tick never writes them, so a caller that runs many _device ticks without reading their
 * counters checks the whole run here: error bit 4 = a bounded spin gave up (WQ_E_TIMEOUT), 2 =
 * more than 2^32-1 pairs in one tick, 8 = a tick ran on a table still missing an incremental
 * batch (wq_apply_ops_device), 16 = a device op batch held an invalid op and was not applied;
 * overflow = some tick's pairs exceeded its capacity. */
int wq_route_health(wq_router* h, uint32_t* error_bits, uint32_t* overflow);

/* ---- instrumentation ----
 * When enabled, every route launch is bracketed by HIP events on the launch stream;
 * wq_profile_read returns the summed kernel-only milliseconds and launch count (and resets). */
int wq_profile_enable(wq_router* h, int enable);
int wq_profile_read(wq_router* h, double* kernel_ms, uint64_t* launches);
/* The same, plus per-kernel time of the launches that ran the three-launch shape (count / tile scan /
 * emit: events between the kernels): phase_ms[0..2] summed over those `phased` launches. */
int wq_profile_read_phases(wq_router* h, double* kernel_ms, uint64_t* launches, double* phase_ms,
                           uint64_t* phased);
/* The shader clock in MHz right now (a short all-CU spin: s_memtime cycles over s_memrealtime wall
 * time), so a bench line can say what clock its timed region ran at. Synchronises the stream. */
int wq_probe_sclk(wq_router* h, double* mhz);

/* ---- test hook: keep only the low `bits` bits of the 64-bit cube hash (64 = normal).
 * Forces bucket collisions so the exact-compare fallback paths are exercised. */
int wq_debug_set_hash_bits(wq_router* h, int bits);
/* ---- tuning hook: record slots per cube at the next full build (default 8: load <= 1/8). More
 * slots = fewer displaced keys (fewer second probe rounds) for more HBM. */
int wq_debug_set_record_slack(wq_router* h, uint32_t slots_per_cube);
/* ---- test hook: how many op batches took the incremental update (wq_delta.hip), how many
 * tried it but fell back to the full rebuild (irregular keys, list space, record load), and how
 * many incremental batches had a cube go through the wave path (a list longer than 48 peers;
 * shorter lists are merged one lane per cube). */
int wq_debug_update_counts(wq_router* h, uint64_t* incremental, uint64_t* rebuild_fallbacks,
                           uint64_t* wave_batches);
/* ---- tuning hook: select a compiled route-kernel shape (messages per thread, expansion chunk);
 * 0 is the default. Results are identical for every shape. */
int wq_debug_set_route_config(wq_router* h, int cfg);
/* ---- tuning hook: the heavy-fan-out tick (count / scan / emit) in `chunks` pipelined chunks — the
 * chunks' counts on a side stream, each chunk's scan and emit on the launch stream as soon as its
 * count is done (0 = the default; 1 = one chunk). Applies to ticks of >= 2 chunks of at most 8,192
 * count tiles each. Results are identical for every value. */
int wq_debug_set_route_chunks(wq_router* h, int chunks);
/* The tick shape the next default-config tick takes (heavy_fanout = count / scan / emit) and
 * whether it is still chosen automatically (no hint set, or reset by a negative hint). */
int wq_debug_route_shape(wq_router* h, int* heavy_fanout, int* fanout_auto);
/* Number of route kernel configurations (valid cfg values are 0 .. n-1). */
int wq_debug_route_config_count(void);
/* Diagnostics: when d_stamps is non-null, the single-launch tick writes four s_memrealtime stamps
 * (100 MHz) per block — start, counted, prefix known, done — to d_stamps[4*block ..]. */
int wq_debug_set_timeline(wq_router* h, uint64_t* d_stamps);

#ifdef __cplusplus
}
#endif

#endif /* WQ_ROUTER_H */
