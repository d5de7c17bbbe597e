"""Python restatement of the reference routing path — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module (or the C restatement it loads), and only as the checker / timed CPU baseline. The
product path in ``worldql_server_amd`` never imports it.

Two independent restatements live here:

* a numpy restatement of the quantiser (``coord_clamp_np``), following
  worldql_server/src/subscriptions/cube_area.rs:23-44 and worldql_server/src/utils/round.rs:1-13
  op for op (fabs, fmod == 0, divide, ceil, multiply, signed compare, Rust's saturating
  ``as i64``, wrapping ``+`` / ``*``);
* ``COracle``: ctypes binding of the C restatement (oracle/wq_oracle.c, built by
  oracle/Makefile into oracle/liboracle.so) of WorldMap / AreaMap / handle_local_message.

Parity pin: the reference is Rust and cannot be built here; both
restatements are checked against the reference's own unit-test vectors in
tests/golden/reference_kats.json, and against each other on random f64 bit patterns.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

I64_MAX = np.iinfo(np.int64).max
I64_MIN = np.iinfo(np.int64).min


def sat_i64_np(x: np.ndarray) -> np.ndarray:
    """Rust ``f64 as i64``: truncate toward zero, saturate, NaN -> 0."""
    x = np.asarray(x, dtype=np.float64)
    out = np.zeros(x.shape, dtype=np.int64)
    nan = np.isnan(x)
    hi = x >= 9223372036854775808.0
    lo = x <= -9223372036854775808.0
    mid = ~(nan | hi | lo)
    out[mid] = np.trunc(x[mid]).astype(np.int64)
    out[hi] = I64_MAX
    out[lo] = I64_MIN
    return out


def round_by_multiple_np(n: np.ndarray, multiple: float) -> np.ndarray:
    """worldql_server/src/utils/round.rs:1-13 (vectorised)."""
    n = np.asarray(n, dtype=np.float64)
    if multiple == 0.0:
        return n.copy()
    with np.errstate(all="ignore"):
        r = np.ceil(n / multiple) * multiple
    return np.where(n == 0.0, np.float64(multiple), r)


def coord_clamp_np(coord, size: int) -> np.ndarray:
    """worldql_server/src/subscriptions/cube_area.rs:23-44 (vectorised, release semantics)."""
    c = np.asarray(coord, dtype=np.float64)
    a = np.abs(c)
    sf = np.float64(size)
    with np.errstate(all="ignore"):
        is_mult = (np.fmod(a, sf) == 0.0) & (c != 0.0)
        rounded = round_by_multiple_np(a, float(size))
        r_i = sat_i64_np(rounded)
        res = np.where(rounded > c, r_i, (r_i.view(np.uint64) + np.uint64(size)).view(np.int64))
        neg = c < 0.0
        res = np.where(neg, (np.uint64(0) - res.view(np.uint64)).view(np.int64), res)
    return np.where(is_mult, sat_i64_np(c), res).astype(np.int64)


def quantize_np(pos, size: int) -> np.ndarray:
    """CubeArea::from_vector3 (cube_area.rs:50-56) over an (n, 3) array."""
    return coord_clamp_np(np.asarray(pos, dtype=np.float64), size)


# ------------------------------------------------------------------------------------------
# C restatement (WorldMap / AreaMap / handle_local_message)
# ------------------------------------------------------------------------------------------

_lib = None


def build_c_oracle() -> str:
    """Compile oracle/wq_oracle.c (gcc) if the .so is missing or stale."""
    src = os.path.join(HERE, "wq_oracle.c")
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB_PATH


def load_c_oracle():
    global _lib
    if _lib is not None:
        return _lib
    build_c_oracle()
    lib = ctypes.CDLL(LIB_PATH)
    vp, u32, u16, i32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int, ctypes.c_size_t
    lib.wqo_round_by_multiple.argtypes = [ctypes.c_double, ctypes.c_double]
    lib.wqo_round_by_multiple.restype = ctypes.c_double
    lib.wqo_coord_clamp.argtypes = [ctypes.c_double, u16]
    lib.wqo_coord_clamp.restype = ctypes.c_int64
    lib.wqo_quantize.argtypes = [vp, sz, u16, vp]
    lib.wqo_quantize.restype = None
    lib.wqo_create.argtypes = [u16]
    lib.wqo_create.restype = vp
    lib.wqo_destroy.argtypes = [vp]
    lib.wqo_destroy.restype = None
    for name in ("wqo_add_subscription", "wqo_remove_subscription", "wqo_is_subscribed"):
        f = getattr(lib, name)
        f.argtypes = [vp, u32, u32, i32, vp]
        f.restype = i32
    lib.wqo_remove_peer.argtypes = [vp, u32]
    lib.wqo_remove_peer.restype = i32
    lib.wqo_is_subscribed_any.argtypes = [vp, u32, u32]
    lib.wqo_is_subscribed_any.restype = i32
    lib.wqo_world_peers.argtypes = [vp, u32, vp, sz]
    lib.wqo_world_peers.restype = sz
    lib.wqo_apply_ops.argtypes = [vp, vp, sz]
    lib.wqo_apply_ops.restype = None
    lib.wqo_route.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, vp, sz, vp]
    lib.wqo_route.restype = sz
    lib.wqo_counts.argtypes = [vp, vp, vp]
    lib.wqo_counts.restype = None
    lib.wqo_route_radius.argtypes = [vp, vp, vp, vp, vp, sz, vp, sz, ctypes.c_double, vp, vp, sz, vp]
    lib.wqo_route_radius.restype = sz
    lib.wqo_route_global.argtypes = [vp, vp, vp, vp, sz, vp, vp, sz]
    lib.wqo_route_global.restype = sz
    lib.wqo_set_fast.argtypes = [vp, i32]
    lib.wqo_set_fast.restype = i32
    lib.wqo_route_check.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, sz, ctypes.c_double, vp, vp,
                                    ctypes.POINTER(sz)]
    lib.wqo_route_check.restype = sz
    lib.wqo_route_faithful.argtypes = [vp] * 5 + [sz, vp, sz, vp, vp, sz]
    lib.wqo_route_faithful.restype = sz
    _lib = lib
    return lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def c_coord_clamp(coords, size: int) -> np.ndarray:
    lib = load_c_oracle()
    c = np.ascontiguousarray(coords, dtype=np.float64)
    out = np.empty(c.shape, dtype=np.int64)
    lib.wqo_quantize(_ptr(c), c.size, size, _ptr(out))
    return out


class COracle:
    """WorldMap restated in C; same op / message encodings as the C ABI (include/wq_router.h)."""

    def __init__(self, cube_size: int):
        self.lib = load_c_oracle()
        self.cube_size = cube_size
        self.h = self.lib.wqo_create(cube_size)

    def close(self):
        if self.h:
            self.lib.wqo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _key(key_is_raw, v):
        a = np.ascontiguousarray(v, dtype=np.int64 if key_is_raw else np.float64)
        return a, _ptr(a)

    def add_subscription(self, world, peer, key_is_raw, v) -> bool:
        a, p = self._key(key_is_raw, v)
        return bool(self.lib.wqo_add_subscription(self.h, world, peer, int(key_is_raw), p))

    def remove_subscription(self, world, peer, key_is_raw, v) -> bool:
        a, p = self._key(key_is_raw, v)
        return bool(self.lib.wqo_remove_subscription(self.h, world, peer, int(key_is_raw), p))

    def remove_peer(self, peer) -> bool:
        return bool(self.lib.wqo_remove_peer(self.h, peer))

    def is_subscribed(self, world, peer, key_is_raw, v) -> bool:
        a, p = self._key(key_is_raw, v)
        return bool(self.lib.wqo_is_subscribed(self.h, world, peer, int(key_is_raw), p))

    def is_subscribed_any(self, world, peer) -> bool:
        return bool(self.lib.wqo_is_subscribed_any(self.h, world, peer))

    def world_peers(self, world) -> np.ndarray:
        n = self.lib.wqo_world_peers(self.h, world, None, 0)
        out = np.empty(n, dtype=np.uint32)
        self.lib.wqo_world_peers(self.h, world, _ptr(out), n)
        return np.sort(out)

    def apply_ops(self, ops: np.ndarray):
        """ops: structured array with dtype worldql_server_amd.router.OP_DTYPE (40 bytes)."""
        ops = np.ascontiguousarray(ops)
        assert ops.dtype.itemsize == 40 and ops.dtype.fields["key"][1] == 16, "pass OP_DTYPE records"
        self.lib.wqo_apply_ops(self.h, _ptr(ops), len(ops))

    def counts(self):
        e, c = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.wqo_counts(self.h, ctypes.byref(e), ctypes.byref(c))
        return e.value, c.value

    def route(self, pos, world, sender, repl, keys=None):
        """Returns (offsets[M+1] u32, peers[P] u32 sorted within each message, F)."""
        world = np.ascontiguousarray(world, dtype=np.uint32)
        M = len(world)
        sender = np.ascontiguousarray(sender, dtype=np.uint32)
        repl = np.ascontiguousarray(repl, dtype=np.uint8)
        pos_a = None if pos is None else np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
        keys_a = None if keys is None else np.ascontiguousarray(keys, dtype=np.int64).reshape(-1, 3)
        offsets = np.zeros(M + 1, dtype=np.uint32)
        F = ctypes.c_uint64()
        P = self.lib.wqo_route(self.h, _ptr(pos_a), _ptr(keys_a), _ptr(world), _ptr(sender), _ptr(repl), M,
                               _ptr(offsets), None, 0, ctypes.byref(F))
        peers = np.zeros(max(P, 1), dtype=np.uint32)
        self.lib.wqo_route(self.h, _ptr(pos_a), _ptr(keys_a), _ptr(world), _ptr(sender), _ptr(repl), M,
                           _ptr(offsets), _ptr(peers), P, None)
        peers = peers[:P]
        sort_within_segments(offsets, peers)
        return offsets, peers, F.value


    def set_fast(self, on: bool = True) -> None:
        """Checker mode for full-size churn (wqo_set_fast): same results, no O(#cubes) scan per
        unsubscribe. Only on an empty map; never for the timed CPU baseline."""
        if self.lib.wqo_set_fast(self.h, int(on)) != 0:
            raise ValueError("wqo_set_fast needs an empty map")

    def route_check(self, pos, world, sender, repl, got_offsets, got_peers, keys=None, peer_pos=None,
                    radius: float = 0.0):
        """(number of messages whose recipients differ from got_offsets / got_peers, first such
        message or M) — wqo_route_check, for ticks too large to sort in numpy."""
        world = np.ascontiguousarray(world, dtype=np.uint32)
        M = len(world)
        sender = np.ascontiguousarray(sender, dtype=np.uint32)
        repl = np.ascontiguousarray(repl, dtype=np.uint8)
        pos_a = None if pos is None else np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
        keys_a = None if keys is None else np.ascontiguousarray(keys, dtype=np.int64).reshape(-1, 3)
        pp = None if peer_pos is None else np.ascontiguousarray(peer_pos, dtype=np.float64).reshape(-1, 3)
        go = np.ascontiguousarray(got_offsets, dtype=np.uint32)
        gp = np.ascontiguousarray(got_peers, dtype=np.uint32)
        assert len(go) == M + 1
        first = ctypes.c_size_t()
        bad = self.lib.wqo_route_check(self.h, _ptr(pos_a), _ptr(keys_a), _ptr(world), _ptr(sender), _ptr(repl), M,
                                       _ptr(pp), 0 if pp is None else len(pp), float(radius), _ptr(go), _ptr(gp),
                                       ctypes.byref(first))
        return int(bad), int(first.value)

    def route_faithful(self, pos, world, sender, repl, connected):
        """cpu_server_faithful_1t (wqo_route_faithful): handle_local_message + PeerMap::broadcast_to
        (peer_map.rs:151-163) with the PeerMap iterating `connected` in order. Returns
        (offsets[M+1], peers in connected order per message)."""
        world = np.ascontiguousarray(world, dtype=np.uint32)
        M = len(world)
        args = (self.h, _ptr(np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)), _ptr(world),
                _ptr(np.ascontiguousarray(sender, dtype=np.uint32)), _ptr(np.ascontiguousarray(repl, dtype=np.uint8)), M)
        conn = np.ascontiguousarray(connected, dtype=np.uint32)
        offsets = np.zeros(M + 1, dtype=np.uint32)
        P = self.lib.wqo_route_faithful(*args, _ptr(conn), len(conn), _ptr(offsets), None, 0)
        peers = np.zeros(max(P, 1), dtype=np.uint32)
        self.lib.wqo_route_faithful(*args, _ptr(conn), len(conn), _ptr(offsets), _ptr(peers), P)
        return offsets, peers[:P]

    def route_radius(self, pos, world, sender, repl, peer_pos, radius: float):
        """C5: route() intersected with the exact radius predicate (wq_oracle.c wqo_route_radius)."""
        world = np.ascontiguousarray(world, dtype=np.uint32)
        M = len(world)
        sender = np.ascontiguousarray(sender, dtype=np.uint32)
        repl = np.ascontiguousarray(repl, dtype=np.uint8)
        pos_a = np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
        pp = np.ascontiguousarray(peer_pos, dtype=np.float64).reshape(-1, 3)
        offsets = np.zeros(M + 1, dtype=np.uint32)
        F = ctypes.c_uint64()
        args = (self.h, _ptr(pos_a), _ptr(world), _ptr(sender), _ptr(repl), M, _ptr(pp), len(pp), float(radius))
        P = self.lib.wqo_route_radius(*args, _ptr(offsets), None, 0, ctypes.byref(F))
        peers = np.zeros(max(P, 1), dtype=np.uint32)
        self.lib.wqo_route_radius(*args, _ptr(offsets), _ptr(peers), P, None)
        peers = peers[:P]
        sort_within_segments(offsets, peers)
        return offsets, peers, F.value

    def route_global(self, world, sender, repl):
        """GlobalMessage to named worlds (global_message.rs:36-84)."""
        world = np.ascontiguousarray(world, dtype=np.uint32)
        M = len(world)
        sender = np.ascontiguousarray(sender, dtype=np.uint32)
        repl = np.ascontiguousarray(repl, dtype=np.uint8)
        offsets = np.zeros(M + 1, dtype=np.uint32)
        P = self.lib.wqo_route_global(self.h, _ptr(world), _ptr(sender), _ptr(repl), M, _ptr(offsets), None, 0)
        peers = np.zeros(max(P, 1), dtype=np.uint32)
        self.lib.wqo_route_global(self.h, _ptr(world), _ptr(sender), _ptr(repl), M, _ptr(offsets), _ptr(peers), P)
        peers = peers[:P]
        sort_within_segments(offsets, peers)
        return offsets, peers


def sort_within_segments(offsets: np.ndarray, values: np.ndarray) -> None:
    """Sort each CSR segment in place (recipient order is a set in the reference)."""
    if len(values) == 0:
        return
    seg = np.repeat(np.arange(len(offsets) - 1, dtype=np.int64), np.diff(offsets.astype(np.int64)))
    order = np.lexsort((values, seg))
    values[:] = values[order]


# ---- cube-hash ownership (restates csrc/wq_device.hpp cube_hash + csrc/wq_shard.hip shard_of) ----
# Not a reference function (the reference is single-process); checked so the GPU owners and the
# CPU sharding tests agree on where every bucket lives.
def _as_u64(a) -> np.ndarray:
    a = np.asarray(a)
    return a if a.dtype == np.uint64 else a.astype(np.int64).view(np.uint64)


def cube_hash_np(w, x, y, z) -> np.ndarray:
    with np.errstate(over="ignore"):
        u = _as_u64
        h = u(x) * np.uint64(0x9E3779B97F4A7C15)
        h ^= u(y) * np.uint64(0xC2B2AE3D27D4EB4F)
        h ^= u(z) * np.uint64(0x165667B19E3779F9)
        h ^= (np.asarray(w, dtype=np.uint64) + np.uint64(0x27D4EB2F165667C5)) * np.uint64(0xD6E8FEB86659FD93)
        h ^= h >> np.uint64(32)
        h *= np.uint64(0xD6E8FEB86659FD93)
        h ^= h >> np.uint64(29)
        h *= np.uint64(0x94D049BB133111EB)
        h ^= h >> np.uint64(32)
    return h


def shard_of_np(w, x, y, z, n_shards: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        v = cube_hash_np(w, x, y, z)
        v ^= v >> np.uint64(31)
        v *= np.uint64(0xBF58476D1CE4E5B9)
        v ^= v >> np.uint64(29)
        return (((v >> np.uint64(32)) * np.uint64(n_shards)) >> np.uint64(32)).astype(np.uint32)
