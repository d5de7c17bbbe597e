"""Python binding of the C ABI (include/wq_router.h) — the HIP routing library, nothing else.

`Router` is a thin ctypes wrapper; every compute call runs the gfx950 kernels of
libwq_router.so. There is no CPU fallback: without the library or without a gfx950 device the
constructor raises `WQError`.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import abi

PKG = os.path.dirname(os.path.abspath(__file__))
# WQ_LIBRARY: another in-tree build of the same sources (A/B timing of a kernel variant on one box)
LIB_PATH = os.environ.get("WQ_LIBRARY") or os.path.join(PKG, "libwq_router.so")

_lib = None

# typedef int (*wq_exchange_fn)(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv,
#                               const size_t* recv_bytes, void* hip_stream)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                               ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p)


class WQError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"wq error {code}: {msg}")
        self.code = code


def load_library(build_if_missing: bool = True):
    """Load libwq_router.so (building it with hipcc if it is absent and hipcc exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not build_if_missing or not os.path.exists(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")):
            raise ImportError(f"{LIB_PATH} is missing: run `python -m worldql_server_amd.build`")
        from .build import build
        build()
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7. Loading torch
    # first makes this library's libamdhip64.so.7 dependency resolve to that same copy (two
    # runtimes in one process do not share devices). Without torch the system runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    vp, sz, u32, u16, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int
    sig = {
        "wq_router_create": ([u16, i32, ctypes.POINTER(vp)], i32),
        "wq_router_create_multi": ([u16, i32, vp, ctypes.POINTER(vp)], i32),
        "wq_multi_info": ([vp, ctypes.POINTER(u32)], i32),
        "wq_router_create_multi_mode": ([u16, i32, vp, i32, ctypes.POINTER(vp)], i32),
        "wq_multi_mode": ([vp, ctypes.POINTER(i32)], i32),
        "wq_route_tick_slices_device": ([vp, vp, i32, vp], i32),
        "wq_shard_tick_stats": ([vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], i32),
        "wq_router_destroy": ([vp], i32),
        "wq_last_error": ([vp], ctypes.c_char_p),
        "wq_set_stream": ([vp, vp], i32),
        "wq_get_stats": ([vp, vp], i32),
        "wq_apply_ops": ([vp, vp, sz], i32),
        "wq_host_alloc": ([sz, ctypes.POINTER(vp)], i32),
        "wq_host_free": ([vp], i32),
        "wq_apply_ops_device": ([vp, vp, sz], i32),
        "wq_remove_peers": ([vp, vp, sz], i32),
        "wq_route_tick": ([vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, sz, ctypes.POINTER(sz)], i32),
        "wq_route_tick_device": ([vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, sz, vp], i32),
        "wq_route_global": ([vp, vp, vp, vp, sz, vp, vp, vp, sz, ctypes.POINTER(sz)], i32),
        "wq_route_global_device": ([vp, vp, vp, vp, sz, vp, vp, vp, sz, vp], i32),
        "wq_peer_major_device": ([vp, vp, vp, sz, sz, vp, u32, vp, vp], i32),
        "wq_is_subscribed": ([vp, sz, vp, vp, i32, vp, vp], i32),
        "wq_is_subscribed_any": ([vp, sz, vp, vp, vp], i32),
        "wq_world_peers": ([vp, u32, vp, sz, ctypes.POINTER(sz)], i32),
        "wq_quantize": ([vp, sz, u16, vp], i32),
        "wq_quantize_device": ([vp, vp, sz, vp], i32),
        "wq_profile_enable": ([vp, i32], i32),
        "wq_profile_read": ([vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)], i32),
        "wq_profile_read_phases": ([vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)], i32),
        "wq_probe_sclk": ([vp, ctypes.POINTER(ctypes.c_double)], i32),
        "wq_debug_set_hash_bits": ([vp, i32], i32),
        "wq_debug_set_record_slack": ([vp, u32], i32),
        "wq_debug_set_route_config": ([vp, i32], i32),
        "wq_debug_set_route_chunks": ([vp, i32], i32),
        "wq_debug_route_config_count": ([], i32),
        "wq_debug_set_timeline": ([vp, vp], i32),
        "wq_debug_update_counts": ([vp] + [ctypes.POINTER(ctypes.c_uint64)] * 3, i32),
        "wq_set_peer_positions": ([vp, vp, sz], i32),
        "wq_set_peer_positions_device": ([vp, vp, sz], i32),
        "wq_set_radius": ([vp, ctypes.c_double], i32),
        "wq_set_fanout_hint": ([vp, ctypes.c_double], i32),
        "wq_debug_route_shape": ([vp, ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
        "wq_route_health": ([vp, ctypes.POINTER(u32), ctypes.POINTER(u32)], i32),
        "wq_shard_ops": ([vp, vp, sz, u32, vp], i32),
        "wq_shard_messages_device": ([vp, vp, vp, vp, vp, vp, sz, u32, vp, vp], i32),
        "wq_route_records_device": ([vp, vp, sz, vp, vp, vp, sz, vp], i32),
        "wq_hub_create": ([u32, ctypes.POINTER(vp)], i32),
        "wq_hub_destroy": ([vp], i32),
        "wq_shard_attach_hub": ([vp, vp, u32], i32),
        "wq_rccl_unique_id": ([vp], i32),
        "wq_shard_attach_rccl": ([vp, u32, u32, vp], i32),
        "wq_shard_attach_exchange": ([vp, u32, u32, EXCHANGE_FN, vp], i32),
        "wq_shard_detach": ([vp], i32),
        "wq_shard_info": ([vp, ctypes.POINTER(u32), ctypes.POINTER(u32)], i32),
        "wq_sharded_apply_ops": ([vp, vp, sz], i32),
        "wq_sharded_route_tick_device": ([vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, sz, ctypes.POINTER(sz)], i32),
        "wq_sharded_route_tick_async": ([vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, sz, vp], i32),
        "wq_sharded_copy_out": ([vp, vp, vp, vp, sz], i32),
        "wq_sharded_route_owner_device": ([vp, vp, vp, vp, vp, vp, sz, ctypes.POINTER(abi.OwnerView)], i32),
        "wq_sharded_route_owner_slots": ([vp, vp, vp, vp, vp, vp, sz, ctypes.POINTER(abi.OwnerSlotView)], i32),
        "wq_sharded_route_owner_slots_async": ([vp, vp, vp, vp, vp, vp, sz, vp, ctypes.POINTER(abi.OwnerSlotView)],
                                               i32),
        "wq_shard_last_bytes": ([vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], i32),
        "wq_debug_set_shard_form": ([vp, i32], i32),
        "wq_debug_inject_shard_failure": ([vp, i32], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    _lib = lib
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class PinnedArray:
    """A numpy array over pinned host memory (wq_host_alloc): DMA-able by the host-array ABI."""

    def __init__(self, shape, dtype):
        self.lib = load_library()
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        p = ctypes.c_void_p()
        rc = self.lib.wq_host_alloc(max(n, 1), ctypes.byref(p))
        if rc != 0:
            raise WQError(rc, "wq_host_alloc")
        self.ptr = p
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=np.uint8, count=n).view(dt).reshape(shape)

    def close(self):
        if self.ptr:
            self.array = None
            self.lib.wq_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WQStats(ctypes.Structure):
    _fields_ = [("n_entries", ctypes.c_uint64), ("n_cubes", ctypes.c_uint64), ("n_any", ctypes.c_uint64),
                ("table_slots", ctypes.c_uint64), ("hash_fallbacks", ctypes.c_uint64),
                ("cube_size", ctypes.c_uint32), ("device", ctypes.c_int32)]


def quantize(coords, cube_size: int) -> np.ndarray:
    """Kernel (1) on host arrays: CubeArea::coord_clamp per coordinate (cube_area.rs:23-44)."""
    lib = load_library()
    c = np.ascontiguousarray(coords, dtype=np.float64)
    out = np.empty(c.shape, dtype=np.int64)
    rc = lib.wq_quantize(_p(c), c.size, cube_size, _p(out))
    if rc != 0:
        raise WQError(rc, lib.wq_last_error(None).decode())
    return out


class Router:
    """One subscription table on one GPU (`WorldMap` of worldql_server/src/subscriptions/world_map.rs)."""

    def __init__(self, cube_size: int = 16, device: int = 0, hash_bits: int = 64):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.wq_router_create(cube_size, device, ctypes.byref(h))
        if rc != 0:
            raise WQError(rc, self.lib.wq_last_error(None).decode())
        self.h = h
        self.cube_size = cube_size
        self.device = device
        if hash_bits != 64:
            self._check(self.lib.wq_debug_set_hash_bits(self.h, hash_bits))

    @classmethod
    def multi(cls, cube_size: int = 16, devices=(0,), mode: str = "cube") -> "Router":
        """One handle over len(devices) GPUs (wq_router_create_multi_mode): the same API, the one-table
        result; mode "cube" = the table sharded by cube hash over the devices (they may repeat),
        "replicate" = every device holds the whole table and routes its own slice."""
        self = cls.__new__(cls)
        self.lib = load_library()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        m = {"cube": abi.MULTI_CUBE_HASH, "replicate": abi.MULTI_REPLICATE}[mode]
        rc = self.lib.wq_router_create_multi_mode(cube_size, len(devices), devs, m, ctypes.byref(h))
        if rc != 0:
            raise WQError(rc, self.lib.wq_last_error(None).decode())
        self.h = h
        self.cube_size = cube_size
        self.device = devices[0]
        return self

    def n_gpus(self) -> int:
        n = ctypes.c_uint32()
        self._check(self.lib.wq_multi_info(self.h, ctypes.byref(n)))
        return n.value

    def multi_mode(self) -> int:
        m = ctypes.c_int()
        self._check(self.lib.wq_multi_mode(self.h, ctypes.byref(m)))
        return m.value

    def route_slices_device(self, slices, with_msgs: bool = False):
        """wq_route_tick_slices_device: slices = one (pos_ptr, world_ptr, sender_ptr, repl_ptr, n_msgs
        [, keys_ptr]) per device of the handle, on that device. Returns a list of abi.SliceView (device
        pointers into the handle's workspace, valid until its next route_slices_device call)."""
        G = len(slices)
        ins = (abi.MsgSlice * G)()
        for g, sl in enumerate(slices):
            pos, wo, se, rp, n = sl[:5]
            keys = sl[5] if len(sl) > 5 else None
            ins[g] = abi.MsgSlice(None if keys else (pos or None), keys or None, wo or None, se or None, rp or None, n)
        outs = (abi.SliceView * G)()
        self._check(self.lib.wq_route_tick_slices_device(self.h, ins, int(with_msgs), outs))
        return [outs[g] for g in range(G)]

    def shard_tick_stats(self):
        """(exact, budgeted) slot ticks run on this shard (wq_shard_tick_stats)."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.wq_shard_tick_stats(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def _check(self, rc: int):
        if rc != 0:
            raise WQError(rc, self.lib.wq_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.wq_router_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- table ----
    def apply_ops(self, ops: np.ndarray) -> None:
        ops = np.ascontiguousarray(ops, dtype=abi.OP_DTYPE)
        self._check(self.lib.wq_apply_ops(self.h, _p(ops), len(ops)))

    def apply_ops_device(self, ops_ptr: int, n: int) -> None:
        """A subscribe / unsubscribe batch already on the device (40-byte wq_op records)."""
        self._check(self.lib.wq_apply_ops_device(self.h, ops_ptr or None, n))

    def remove_peers(self, peers) -> None:
        a = np.ascontiguousarray(peers, dtype=np.uint32)
        self._check(self.lib.wq_remove_peers(self.h, _p(a), len(a)))

    def stats(self) -> dict:
        s = WQStats()
        self._check(self.lib.wq_get_stats(self.h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in WQStats._fields_}

    # ---- hot path ----
    def route(self, pos, world, sender, repl, keys=None, with_msgs: bool = False, capacity: int | None = None):
        """One tick on host arrays. Returns (offsets[M+1], peers[P], msgs[P] or None)."""
        world = np.ascontiguousarray(world, dtype=np.uint32)
        M = len(world)
        sender = np.ascontiguousarray(sender, dtype=np.uint32)
        repl = np.ascontiguousarray(repl, dtype=np.uint8)
        pos_a = None if pos is None else np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
        keys_a = None if keys is None else np.ascontiguousarray(keys, dtype=np.int64).reshape(-1, 3)
        cap = capacity if capacity is not None else max(1024, 16 * M)
        while True:
            offsets = np.empty(M + 1, dtype=np.uint32)
            peers = np.empty(max(cap, 1), dtype=np.uint32)
            msgs = np.empty(max(cap, 1), dtype=np.uint32) if with_msgs else None
            n = ctypes.c_size_t()
            rc = self.lib.wq_route_tick(self.h, _p(pos_a), _p(keys_a), _p(world), _p(sender), _p(repl), M,
                                        _p(offsets), _p(peers), _p(msgs), cap, ctypes.byref(n))
            if rc == abi.WQ_E_CAPACITY and n.value > cap and capacity is None:
                cap = n.value
                continue
            self._check(rc)
            P = n.value
            return offsets, peers[:P], (msgs[:P] if with_msgs else None)

    def route_device(self, pos_ptr: int, world_ptr: int, sender_ptr: int, repl_ptr: int, n_msgs: int,
                     offsets_ptr: int, peers_ptr: int, msgs_ptr: int | None, capacity: int,
                     counters_ptr: int | None = None, keys_ptr: int | None = None) -> None:
        """Asynchronous tick on device pointers (e.g. torch tensors' data_ptr())."""
        self._check(self.lib.wq_route_tick_device(self.h, pos_ptr or None, keys_ptr or None, world_ptr, sender_ptr,
                                                  repl_ptr, n_msgs, offsets_ptr, peers_ptr or None,
                                                  msgs_ptr or None, capacity, counters_ptr or None))

    def route_global(self, world, sender, repl, with_msgs: bool = False, capacity: int | None = None):
        """A tick of GlobalMessages to named worlds (global_message.rs:36-84) on host arrays.
        Returns (offsets[M+1], peers[P], msgs[P] or None); peers per message ascending."""
        world = np.ascontiguousarray(world, dtype=np.uint32)
        M = len(world)
        sender = np.ascontiguousarray(sender, dtype=np.uint32)
        repl = np.ascontiguousarray(repl, dtype=np.uint8)
        cap = capacity if capacity is not None else max(1024, 16 * M)
        while True:
            offsets = np.empty(M + 1, dtype=np.uint32)
            peers = np.empty(max(cap, 1), dtype=np.uint32)
            msgs = np.empty(max(cap, 1), dtype=np.uint32) if with_msgs else None
            n = ctypes.c_size_t()
            rc = self.lib.wq_route_global(self.h, _p(world), _p(sender), _p(repl), M, _p(offsets), _p(peers),
                                          _p(msgs), cap, ctypes.byref(n))
            if rc == abi.WQ_E_CAPACITY and n.value > cap and capacity is None:
                cap = n.value
                continue
            self._check(rc)
            P = n.value
            return offsets, peers[:P], (msgs[:P] if with_msgs else None)

    def route_global_device(self, world_ptr: int, sender_ptr: int, repl_ptr: int, n_msgs: int, offsets_ptr: int,
                            peers_ptr: int | None, msgs_ptr: int | None, capacity: int,
                            counters_ptr: int | None = None) -> None:
        self._check(self.lib.wq_route_global_device(self.h, world_ptr, sender_ptr, repl_ptr, n_msgs, offsets_ptr,
                                                    peers_ptr or None, msgs_ptr or None, capacity,
                                                    counters_ptr or None))

    def peer_major_device(self, offsets_ptr: int, peers_ptr: int | None, n_msgs: int, n_pairs: int,
                          connected_ptr: int | None, n_peers: int, peer_offsets_ptr: int, msgs_out_ptr: int | None):
        """Per-peer send lists of a tick's CSR, disconnected peers dropped (peer_map.rs:151-163)."""
        self._check(self.lib.wq_peer_major_device(self.h, offsets_ptr or None, peers_ptr or None, n_msgs, n_pairs,
                                                  connected_ptr or None, n_peers, peer_offsets_ptr,
                                                  msgs_out_ptr or None))

    # ---- multi-GPU (cube-hash ownership: wq_sharded.hip) ----
    def shard_ops(self, ops: np.ndarray, n_shards: int) -> np.ndarray:
        """Owner shard of each op (abi.SHARD_ALL for REMOVE_PEER)."""
        ops = np.ascontiguousarray(ops, dtype=abi.OP_DTYPE)
        out = np.empty(len(ops), dtype=np.uint32)
        self._check(self.lib.wq_shard_ops(self.h, _p(ops), len(ops), n_shards, _p(out)))
        return out

    def shard_messages_device(self, pos_ptr: int | None, keys_ptr: int | None, world_ptr: int, sender_ptr: int,
                              repl_ptr: int, n_msgs: int, n_shards: int, recs_ptr: int, counts_ptr: int) -> None:
        """Group a tick's messages by owner shard into 40-byte records (asynchronous)."""
        self._check(self.lib.wq_shard_messages_device(self.h, pos_ptr or None, keys_ptr or None, world_ptr or None,
                                                      sender_ptr or None, repl_ptr or None, n_msgs, n_shards,
                                                      recs_ptr or None, counts_ptr))

    def route_records_device(self, recs_ptr: int | None, n_msgs: int, offsets_ptr: int, peers_ptr: int | None,
                             msgs_ptr: int | None, capacity: int, counters_ptr: int | None = None) -> None:
        """Route received records on this shard (asynchronous)."""
        self._check(self.lib.wq_route_records_device(self.h, recs_ptr or None, n_msgs, offsets_ptr,
                                                     peers_ptr or None, msgs_ptr or None, capacity,
                                                     counters_ptr or None))

    # ---- multi-GPU behind the ABI: this handle as one shard of G (include/wq_router.h) ----
    def attach_hub(self, hub: "Hub", rank: int) -> None:
        self._check(self.lib.wq_shard_attach_hub(self.h, hub.h, rank))
        self._hub = hub  # keep it alive while attached

    def attach_rccl(self, n_shards: int, rank: int, uid: bytes) -> None:
        assert len(uid) == abi.RCCL_ID_BYTES
        buf = ctypes.create_string_buffer(bytes(uid), abi.RCCL_ID_BYTES)
        self._check(self.lib.wq_shard_attach_rccl(self.h, n_shards, rank, buf))

    def attach_exchange(self, n_shards: int, rank: int, fn) -> None:
        """fn(d_send, send_bytes[G], d_recv, recv_bytes[G], stream) -> None: the caller's all-to-all
        (device pointers as ints, byte counts as lists). Exceptions count as failures."""
        G = n_shards

        def tramp(_ctx, send, sb, recv, rb, stream):
            try:
                fn(send or 0, [sb[i] for i in range(G)], recv or 0, [rb[i] for i in range(G)], stream or 0)
                return 0
            except Exception:  # noqa: BLE001 — reported through the C status
                import traceback
                traceback.print_exc()
                return 1
        self._xfn = EXCHANGE_FN(tramp)  # keep the trampoline alive
        self._check(self.lib.wq_shard_attach_exchange(self.h, n_shards, rank, self._xfn, None))

    def detach_shard(self) -> None:
        self._check(self.lib.wq_shard_detach(self.h))

    def shard_info(self):
        g, r = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.wq_shard_info(self.h, ctypes.byref(g), ctypes.byref(r)))
        return g.value, r.value

    def sharded_apply_ops(self, ops: np.ndarray) -> None:
        """The tick's whole op stream (every shard gets the same); this shard keeps what it owns."""
        ops = np.ascontiguousarray(ops, dtype=abi.OP_DTYPE)
        self._check(self.lib.wq_sharded_apply_ops(self.h, _p(ops), len(ops)))

    def sharded_route_device(self, pos_ptr, world_ptr, sender_ptr, repl_ptr, n_msgs, offsets_ptr, peers_ptr,
                             msgs_ptr, capacity, keys_ptr=None):
        """One collective sharded tick on this shard's ingested messages (device pointers).
        Returns (rc, P): rc is WQ_OK or WQ_E_CAPACITY (then sharded_copy_out with room for P)."""
        n = ctypes.c_size_t()
        rc = self.lib.wq_sharded_route_tick_device(self.h, pos_ptr or None, keys_ptr or None, world_ptr or None,
                                                   sender_ptr or None, repl_ptr or None, n_msgs, offsets_ptr,
                                                   peers_ptr or None, msgs_ptr or None, capacity, ctypes.byref(n))
        if rc not in (0, abi.WQ_E_CAPACITY):
            self._check(rc)
        return rc, n.value

    def sharded_route_async(self, pos_ptr, world_ptr, sender_ptr, repl_ptr, n_msgs, offsets_ptr, peers_ptr,
                            msgs_ptr, capacity, counters_ptr=None, keys_ptr=None) -> None:
        """wq_sharded_route_tick_async: the collective tick without its end-of-tick read; P and the
        status bits (64: a budget was too small, route the tick again) land in counters_ptr."""
        self._check(self.lib.wq_sharded_route_tick_async(self.h, pos_ptr or None, keys_ptr or None, world_ptr or None,
                                                         sender_ptr or None, repl_ptr or None, n_msgs, offsets_ptr,
                                                         peers_ptr or None, msgs_ptr or None, capacity,
                                                         counters_ptr or None))

    def sharded_route_owner_device(self, pos_ptr, world_ptr, sender_ptr, repl_ptr, n_msgs, keys_ptr=None):
        """The owner-side form of the collective sharded tick: the pairs stay on the shard that routed
        them. Returns an abi.OwnerView of device pointers valid until the next sharded call."""
        v = abi.OwnerView()
        self._check(self.lib.wq_sharded_route_owner_device(self.h, pos_ptr or None, keys_ptr or None, world_ptr or None,
                                                           sender_ptr or None, repl_ptr or None, n_msgs,
                                                           ctypes.byref(v)))
        return v

    def sharded_route_owner_slots(self, pos_ptr, world_ptr, sender_ptr, repl_ptr, n_msgs, keys_ptr=None):
        """wq_sharded_route_owner_slots: the owner form on budgeted 20-byte slots (one exchange per
        tick; the pairs stay on the owner). Returns an abi.OwnerSlotView of device pointers valid
        until the next sharded call."""
        v = abi.OwnerSlotView()
        self._check(self.lib.wq_sharded_route_owner_slots(self.h, pos_ptr or None, keys_ptr or None, world_ptr or None,
                                                          sender_ptr or None, repl_ptr or None, n_msgs,
                                                          ctypes.byref(v)))
        return v

    def sharded_route_owner_slots_async(self, pos_ptr, world_ptr, sender_ptr, repl_ptr, n_msgs, counters_ptr=None,
                                        keys_ptr=None):
        """wq_sharded_route_owner_slots_async: the owner-slot tick without its end-of-tick read; P and the
        status bits land in counters_ptr (view.n_pairs is 2^64-1 when the tick ran asynchronously)."""
        v = abi.OwnerSlotView()
        self._check(self.lib.wq_sharded_route_owner_slots_async(self.h, pos_ptr or None, keys_ptr or None,
                                                                world_ptr or None, sender_ptr or None, repl_ptr or None,
                                                                n_msgs, counters_ptr or None, ctypes.byref(v)))
        return v

    def sharded_copy_out(self, offsets_ptr, peers_ptr, msgs_ptr, capacity) -> None:
        self._check(self.lib.wq_sharded_copy_out(self.h, offsets_ptr, peers_ptr or None, msgs_ptr or None, capacity))

    def shard_last_bytes(self):
        """(bytes sent to, bytes received from) OTHER shards in this shard's latest sharded tick."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.wq_shard_last_bytes(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def inject_shard_failure(self, step: int) -> None:
        """Test hook: the next sharded tick fails locally at step 1 or 3 (wq_debug_inject_shard_failure)."""
        self._check(self.lib.wq_debug_inject_shard_failure(self.h, step))

    def set_shard_form(self, expanded: bool) -> None:
        """True: the sharded tick returns expanded (message, peer) pairs (the radius filter's form);
        False (default): row references + one pool of cube lists per destination."""
        self._check(self.lib.wq_debug_set_shard_form(self.h, int(expanded)))

    # ---- C5 radius filter (include/wq_router.h) ----
    def set_peer_positions(self, pos) -> None:
        p = np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
        self._check(self.lib.wq_set_peer_positions(self.h, _p(p), len(p)))

    def set_peer_positions_device(self, pos_ptr: int, n_peers: int) -> None:
        self._check(self.lib.wq_set_peer_positions_device(self.h, pos_ptr or None, n_peers))

    def set_radius(self, radius: float) -> None:
        self._check(self.lib.wq_set_radius(self.h, float(radius)))

    def set_fanout_hint(self, pairs_per_message: float) -> None:
        """Expected recipients per message (e.g. the previous tick's P / M): >= 16 selects the
        count / scan / emit tick shape (wq_set_fanout_hint)."""
        self._check(self.lib.wq_set_fanout_hint(self.h, float(pairs_per_message)))

    def route_shape(self):
        """(heavy_fanout, fanout_auto) of the next default-config tick (wq_debug_route_shape)."""
        a, b = ctypes.c_int(), ctypes.c_int()
        self._check(self.lib.wq_debug_route_shape(self.h, ctypes.byref(a), ctypes.byref(b)))
        return bool(a.value), bool(b.value)

    def route_health(self):
        """(error bits OR, overflow OR) over every route / global call since the last read
        (wq_route_health; clears them)."""
        e, o = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.wq_route_health(self.h, ctypes.byref(e), ctypes.byref(o)))
        return e.value, o.value

    def check_health(self) -> None:
        """Raises WQError when any tick since the last check reported an error or an overflow."""
        e, o = self.route_health()
        if e & 16:
            raise WQError(abi.WQ_E_INVALID, f"a device op batch held an invalid op and was not applied "
                                            f"(error bits {e:#x})")
        if e & 8:
            raise WQError(abi.WQ_E_INVALID, f"a tick ran on a table still missing an incremental batch the "
                                            f"device could not apply (error bits {e:#x})")
        if e & 4:
            raise WQError(abi.WQ_E_TIMEOUT, f"a route look-back spin gave up (error bits {e:#x})")
        if e or o:
            raise WQError(abi.WQ_E_CAPACITY, f"route error bits {e:#x}, overflow {o}")

    def set_stream(self, stream_ptr: int | None) -> None:
        self._check(self.lib.wq_set_stream(self.h, stream_ptr or None))

    # ---- queries ----
    def is_subscribed(self, world, peer, key_is_raw: bool, key_or_pos) -> np.ndarray:
        world = np.ascontiguousarray(world, dtype=np.uint32)
        peer = np.ascontiguousarray(peer, dtype=np.uint32)
        k = np.ascontiguousarray(key_or_pos, dtype=np.int64 if key_is_raw else np.float64).reshape(-1, 3)
        out = np.zeros(len(world), dtype=np.uint8)
        self._check(self.lib.wq_is_subscribed(self.h, len(world), _p(world), _p(peer), int(key_is_raw), _p(k),
                                              _p(out)))
        return out.astype(bool)

    def is_subscribed_any(self, world, peer) -> np.ndarray:
        world = np.ascontiguousarray(world, dtype=np.uint32)
        peer = np.ascontiguousarray(peer, dtype=np.uint32)
        out = np.zeros(len(world), dtype=np.uint8)
        self._check(self.lib.wq_is_subscribed_any(self.h, len(world), _p(world), _p(peer), _p(out)))
        return out.astype(bool)

    def world_peers(self, world: int) -> np.ndarray:
        n = ctypes.c_size_t()
        rc = self.lib.wq_world_peers(self.h, world, None, 0, ctypes.byref(n))
        if rc not in (0, abi.WQ_E_CAPACITY):
            self._check(rc)
        out = np.zeros(max(n.value, 1), dtype=np.uint32)
        self._check(self.lib.wq_world_peers(self.h, world, _p(out), n.value, ctypes.byref(n)))
        return out[: n.value]

    def update_counts(self, lanes: bool = False):
        """(batches applied incrementally, batches that fell back to the full rebuild)
        [+ incremental batches in which a cube took the wave path (list > 48 peers), lanes=True]."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.wq_debug_update_counts(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return (a.value, b.value, c.value) if lanes else (a.value, b.value)

    def set_record_slack(self, slots_per_cube: int) -> None:
        self._check(self.lib.wq_debug_set_record_slack(self.h, slots_per_cube))

    def route_config_count(self) -> int:
        return int(self.lib.wq_debug_route_config_count())

    def set_route_config(self, cfg: int) -> None:
        self._check(self.lib.wq_debug_set_route_config(self.h, cfg))

    def set_route_chunks(self, chunks: int) -> None:
        """Chunks of the pipelined heavy tick (wq_debug_set_route_chunks; 0 = default)."""
        self._check(self.lib.wq_debug_set_route_chunks(self.h, chunks))

    # ---- instrumentation ----
    def profile_enable(self, on: bool = True) -> None:
        self._check(self.lib.wq_profile_enable(self.h, int(on)))

    def profile_read(self):
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        self._check(self.lib.wq_profile_read(self.h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def profile_read_phases(self):
        """(kernel ms, launches, [count, tile_scan, emit] ms summed over the three-launch launches, their
        number) — wq_profile_read_phases; resets like profile_read."""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        ph, npz = (ctypes.c_double * 3)(), ctypes.c_uint64()
        self._check(self.lib.wq_profile_read_phases(self.h, ctypes.byref(ms), ctypes.byref(n), ph, ctypes.byref(npz)))
        return ms.value, n.value, list(ph), npz.value

    def probe_sclk(self) -> float:
        """The shader clock in MHz right now (wq_probe_sclk)."""
        mhz = ctypes.c_double()
        self._check(self.lib.wq_probe_sclk(self.h, ctypes.byref(mhz)))
        return mhz.value


class Hub:
    """An in-process exchange for G router handles of one process (wq_hub_create)."""

    def __init__(self, n_shards: int):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.wq_hub_create(n_shards, ctypes.byref(h))
        if rc != 0:
            raise WQError(rc, "wq_hub_create")
        self.h = h
        self.n_shards = n_shards

    def close(self):
        if getattr(self, "h", None):
            self.lib.wq_hub_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rccl_unique_id() -> bytes:
    """wq_rccl_unique_id: the 128-byte communicator id rank 0 hands to every rank."""
    lib = load_library()
    buf = ctypes.create_string_buffer(abi.RCCL_ID_BYTES)
    rc = lib.wq_rccl_unique_id(buf)
    if rc != 0:
        raise WQError(rc, "wq_rccl_unique_id (librccl not loadable?)")
    return buf.raw
