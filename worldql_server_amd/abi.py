"""Host-side constants and record layouts of the C ABI (include/wq_router.h).

Pure data: importing this module loads no native code.
"""
from __future__ import annotations

import ctypes

import numpy as np

WQ_OK = 0
WQ_E_INVALID = -1
WQ_E_OOM = -2
WQ_E_HIP = -3
WQ_E_RCCL = -4
WQ_E_CAPACITY = -5
WQ_E_NODEV = -6
WQ_E_TIMEOUT = -7

OP_SUBSCRIBE = 0    # AreaMap::add_subscription (area_map.rs:72-85)
OP_UNSUBSCRIBE = 1  # AreaMap::remove_subscription (area_map.rs:88-119)
OP_REMOVE_PEER = 2  # WorldMap::remove_peer (world_map.rs:41-61)

REPL_EXCEPT_SELF = 0     # Replication wire codes, WorldQLFB_generated.rs:176-188
REPL_INCLUDING_SELF = 1
REPL_ONLY_SELF = 2

WORLD_INVALID = 0xFFFFFFFF

# struct wq_op: 40 bytes; `key` aliases `pos` (union).
OP_DTYPE = np.dtype({
    "names": ["world", "peer", "kind", "key_is_raw", "pos", "key"],
    "formats": [np.uint32, np.uint32, np.uint8, np.uint8, (np.float64, 3), (np.int64, 3)],
    "offsets": [0, 4, 8, 9, 16, 16],
    "itemsize": 40,
})

# struct wq_route_counters: 24 bytes
COUNTERS_DTYPE = np.dtype([("n_pairs", np.uint64), ("n_candidates", np.uint64),
                           ("overflow", np.uint32), ("error", np.uint32)])


def make_op(world: int, peer: int, kind: int, pos=None, key=None) -> np.void:
    """One wq_op record; give `pos` (Vector3, quantised) or `key` (raw CubeArea)."""
    o = np.zeros((), dtype=OP_DTYPE)
    o["world"] = world
    o["peer"] = peer
    o["kind"] = kind
    if key is not None:
        o["key_is_raw"] = 1
        o["key"] = np.asarray(key, dtype=np.int64)
    else:
        o["key_is_raw"] = 0
        o["pos"] = np.asarray(pos if pos is not None else (0.0, 0.0, 0.0), dtype=np.float64)
    return o[()]


def ops_array(world, peer, kind, pos=None, key=None) -> np.ndarray:
    """Vectorised op construction (all arguments broadcast over n ops)."""
    world = np.asarray(world, dtype=np.uint32)
    n = world.shape[0]
    ops = np.zeros(n, dtype=OP_DTYPE)
    ops["world"] = world
    ops["peer"] = np.asarray(peer, dtype=np.uint32)
    ops["kind"] = np.asarray(kind, dtype=np.uint8)
    if key is not None:
        ops["key_is_raw"] = 1
        ops["key"] = np.asarray(key, dtype=np.int64).reshape(n, 3)
    else:
        ops["pos"] = np.asarray(pos, dtype=np.float64).reshape(n, 3)
    return ops


def concat_ops(parts) -> np.ndarray:
    """np.concatenate drops the union layout of OP_DTYPE; join the raw 40-byte records instead."""
    return np.concatenate([np.ascontiguousarray(p, dtype=OP_DTYPE).view(np.uint8) for p in parts]).view(OP_DTYPE)


# ---- multi-GPU (include/wq_router.h, "cube-hash ownership") ----
MAX_SHARDS = 64
RCCL_ID_BYTES = 128  # WQ_RCCL_ID_BYTES
SHARD_ALL = 0xFFFFFFFF  # owner of a REMOVE_PEER op

# struct wq_owner_view (wq_sharded_route_owner_device): device pointers + counts + source segments
class OwnerView(ctypes.Structure):
    _fields_ = [("recs", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("peers", ctypes.c_void_p),
                ("n_recs", ctypes.c_uint64), ("n_pairs", ctypes.c_uint64), ("seg", ctypes.c_uint32 * (MAX_SHARDS + 1))]


SLOT_WORDS = 5  # WQ_SLOT_WORDS


class OwnerSlotView(ctypes.Structure):  # struct wq_owner_slot_view
    _fields_ = [("slots", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("peers", ctypes.c_void_p),
                ("send_perm", ctypes.c_void_p), ("n_slots", ctypes.c_uint64),
                ("n_pairs", ctypes.c_uint64), ("seg", ctypes.c_uint32 * (MAX_SHARDS + 1)),
                ("send_seg", ctypes.c_uint32 * (MAX_SHARDS + 1))]


# wq_router_create_multi_mode layouts
MULTI_CUBE_HASH = 0
MULTI_REPLICATE = 1


class MsgSlice(ctypes.Structure):  # struct wq_msg_slice: one device's ingested messages
    _fields_ = [("d_pos", ctypes.c_void_p), ("d_keys", ctypes.c_void_p), ("d_world", ctypes.c_void_p),
                ("d_sender", ctypes.c_void_p), ("d_repl", ctypes.c_void_p), ("n_msgs", ctypes.c_uint64)]


class SliceView(ctypes.Structure):  # struct wq_slice_view: one device's CSR, left on that device
    _fields_ = [("device", ctypes.c_int32), ("pad_", ctypes.c_uint32), ("n_msgs", ctypes.c_uint64),
                ("n_pairs", ctypes.c_uint64), ("offsets", ctypes.c_void_p), ("peers", ctypes.c_void_p),
                ("msgs", ctypes.c_void_p)]


# struct wq_msg_rec: 40 bytes on the wire between GPUs
REC_POS = 1  # wq_msg_rec.flags: key holds the f64 position bits (radius filter on)
MSG_REC_DTYPE = np.dtype({
    "names": ["key", "world", "sender", "msg", "repl", "flags"],
    "formats": [(np.int64, 3), np.uint32, np.uint32, np.uint32, np.uint8, np.uint8],
    "offsets": [0, 24, 28, 32, 36, 37],
    "itemsize": 40,
})
