"""`WorldMap` / `AreaMap` / `CubeArea` / `Vector3` with the reference's method names and meaning,
backed by the GPU table (libwq_router.so through `Router`).

Mirrors worldql_server/src/subscriptions/{world_map.rs:10-62, area_map.rs:10-135,
cube_area.rs:8-77} so code (and tests) written against the reference API run unchanged in
shape. Peers are any hashable id (the reference uses `Uuid`); they are mapped to the dense u32
ids the C ABI takes. World names are the sanitized names (the handlers sanitize before calling
`get` / `get_mut`, see processing.py).

The single-op methods are convenience wrappers (one GPU round trip each); the throughput path
is `Router.apply_ops` / `Router.route` on batches, used by processing.py.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Hashable, Iterator, Optional, Union

import numpy as np

from . import abi
from .router import Router
from .world_names import WorldIds


@dataclass(frozen=True)
class Vector3:
    """worldql_server/src/structures/vector3.rs:11-15 (f64 x, y, z)."""
    x: float
    y: float
    z: float


@dataclass(frozen=True)
class CubeArea:
    """worldql_server/src/subscriptions/cube_area.rs:8-13 (i64 x, y, z). Passed to the table as-is
    (impl ToCubeArea for CubeArea is the identity, cube_area.rs:65-70)."""
    x: int
    y: int
    z: int


ToCubeArea = Union[Vector3, CubeArea]


def _key_args(cube: ToCubeArea):
    if isinstance(cube, CubeArea):
        return True, np.array([[cube.x, cube.y, cube.z]], dtype=np.int64)
    if isinstance(cube, Vector3):
        return False, np.array([[cube.x, cube.y, cube.z]], dtype=np.float64)
    raise TypeError("expected Vector3 or CubeArea")


class PeerIds:
    """Uuid (any hashable) <-> dense u32 peer id, with ids recycled after a disconnect.

    The reference keys peers by Uuid and forgets a peer when it disconnects (PeerMap::remove,
    worldql_server/src/transport/peer_map.rs:121-141, then WorldMap::remove_peer). `release` does
    the same here: the id goes on a free list once the table no longer holds the peer, so per-peer
    arrays on the device (F2 send lists, C5 positions) stay bounded by the peers connected at once
    (`high_water`), not by every peer that ever connected."""

    def __init__(self):
        self._ids: dict = {}
        self._peers: list = []
        self._free: list = []

    def id(self, peer: Hashable) -> int:
        pid = self._ids.get(peer)
        if pid is None:
            if self._free:
                pid = self._free.pop()
                self._peers[pid] = peer
            else:
                pid = len(self._peers)
                self._peers.append(peer)
            self._ids[peer] = pid
        return pid

    def lookup(self, peer: Hashable) -> Optional[int]:
        return self._ids.get(peer)

    def release(self, peer: Hashable) -> Optional[int]:
        """Forget `peer` (call after its REMOVE_PEER op is applied); returns its former id."""
        pid = self._ids.pop(peer, None)
        if pid is not None:
            self._peers[pid] = None
            self._free.append(pid)
        return pid

    @property
    def high_water(self) -> int:
        """Ids ever handed out at once: per-peer device arrays need this many entries."""
        return len(self._peers)

    def __len__(self) -> int:
        return len(self._ids)

    def peer(self, pid: int) -> Hashable:
        return self._peers[pid]

    def peers(self, pids) -> list:
        return [self._peers[int(p)] for p in pids]


class WorldMap:
    """world_map.rs:10-62. One GPU table holds every world; a world "exists" once `get_mut`
    has been called for it, exactly like the reference's lazily created AreaMap."""

    def __init__(self, cube_size: int = 16, device: int = 0, router: Optional[Router] = None):
        self.cube_size = cube_size
        self.router = router if router is not None else Router(cube_size, device)
        self.worlds = WorldIds()
        self.peer_ids = PeerIds()
        self._maps: dict[str, AreaMap] = {}

    def get(self, world_name: str) -> Optional["AreaMap"]:  # world_map.rs:25-27
        return self._maps.get(world_name)

    def get_mut(self, world_name: str) -> "AreaMap":  # world_map.rs:31-36
        am = self._maps.get(world_name)
        if am is None:
            am = AreaMap(self, world_name, self.worlds.intern(world_name))
            self._maps[world_name] = am
        return am

    def remove_peer(self, uuid: Hashable) -> bool:  # world_map.rs:41-61
        pid = self.peer_ids.lookup(uuid)
        if pid is None:
            return False
        if not self._maps:
            self.peer_ids.release(uuid)
            return False
        wids = np.array([am.world_id for am in self._maps.values()], dtype=np.uint32)
        removed = bool(self.router.is_subscribed_any(wids, np.full(len(wids), pid, np.uint32)).any())
        self.router.apply_ops(np.array([abi.make_op(abi.WORLD_INVALID, pid, abi.OP_REMOVE_PEER)], abi.OP_DTYPE))
        self.peer_ids.release(uuid)  # the peer is gone (peer_map.rs:121-141): its id is free again
        return removed


class AreaMap:
    """area_map.rs:10-135 for one world of the shared GPU table."""

    def __init__(self, world_map: WorldMap, world_name: str, world_id: int):
        self._wm = world_map
        self.world_name = world_name
        self.world_id = world_id
        self.cube_size = world_map.cube_size

    @property
    def _r(self) -> Router:
        return self._wm.router

    def _pid(self, uuid) -> int:
        return self._wm.peer_ids.id(uuid)

    def is_peer_subscribed(self, uuid: Hashable, cube: ToCubeArea) -> bool:  # :33-41
        raw, k = _key_args(cube)
        return bool(self._r.is_subscribed([self.world_id], [self._pid(uuid)], raw, k)[0])

    def is_peer_subscribed_any(self, uuid: Hashable) -> bool:  # :46-48
        return bool(self._r.is_subscribed_any([self.world_id], [self._pid(uuid)])[0])

    def get_subscribed_peers(self, cube: ToCubeArea) -> Iterator[Hashable]:  # :52-60
        raw, k = _key_args(cube)
        w = np.array([self.world_id], np.uint32)
        z = np.zeros(1, np.uint32)
        incl = np.array([abi.REPL_INCLUDING_SELF], np.uint8)
        if raw:
            _, peers, _ = self._r.route(None, w, z, incl, keys=k)
        else:
            _, peers, _ = self._r.route(k, w, z, incl)
        return iter(self._wm.peer_ids.peers(peers))

    def get_subscribed_any_peers(self) -> Iterator[Hashable]:  # :65-67
        return iter(self._wm.peer_ids.peers(self._r.world_peers(self.world_id)))

    def _op(self, uuid, cube, kind):
        raw, k = _key_args(cube)
        if raw:
            return abi.make_op(self.world_id, self._pid(uuid), kind, key=k[0])
        return abi.make_op(self.world_id, self._pid(uuid), kind, pos=k[0])

    def add_subscription(self, uuid: Hashable, cube: ToCubeArea) -> bool:  # :72-85
        was = self.is_peer_subscribed(uuid, cube)
        self._r.apply_ops(np.array([self._op(uuid, cube, abi.OP_SUBSCRIBE)], abi.OP_DTYPE))
        return not was

    def remove_subscription(self, uuid: Hashable, cube: ToCubeArea) -> bool:  # :88-119
        was = self.is_peer_subscribed(uuid, cube)
        self._r.apply_ops(np.array([self._op(uuid, cube, abi.OP_UNSUBSCRIBE)], abi.OP_DTYPE))
        return was

    def remove_peer(self, uuid: Hashable) -> bool:  # :124-135
        was = self.is_peer_subscribed_any(uuid)
        self._r.apply_ops(np.array([abi.make_op(self.world_id, self._pid(uuid), abi.OP_REMOVE_PEER)],
                                   abi.OP_DTYPE))
        return was
