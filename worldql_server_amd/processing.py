"""Host side of the hot path: message validation and tick batching around the GPU table.

Mirrors, at tick granularity, the reference's single subscription task
`handle_sub_messages` (worldql_server/src/processing/thread.rs:113-148) and the handlers it
calls: handle_local_message (local_message.rs:10-89), handle_global_message
(global_message.rs:10-88), handle_area_subscribe (area_subscribe.rs:10-52),
handle_area_unsubscribe (area_unsubscribe.rs:10-52) and the disconnect path
WorldMap::remove_peer (thread.rs:124-125).

Ordering contract ("flush-on-reorder"): a tick is the arrival-ordered list of
events. Consecutive table events (subscribe / unsubscribe / disconnect) form one op batch;
consecutive read events (LocalMessage and GlobalMessage, which never change the table) form one
read run, routed as one wq_route_tick plus one wq_route_global; runs execute in arrival order —
so every message sees exactly the table the sequential reference would have shown it, and the
broadcast callback fires in arrival order.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Hashable, List, Optional, Sequence, Union

import numpy as np

from . import abi
from .subscriptions import Vector3, WorldMap
from .world_names import GLOBAL_WORLD, SanitizeError, sanitize_world_name

LOCAL_MESSAGE = "LocalMessage"
GLOBAL_MESSAGE = "GlobalMessage"
AREA_SUBSCRIBE = "AreaSubscribe"
AREA_UNSUBSCRIBE = "AreaUnsubscribe"
DISCONNECT = "Disconnect"  # a uuid arriving on remove_rx (thread.rs:124-125)

NO_PEER = 0xFFFFFFFF  # sender id of a peer that holds no id (never a subscriber)
_TABLE_EVENTS = (AREA_SUBSCRIBE, AREA_UNSUBSCRIBE, DISCONNECT)
_READ_EVENTS = (LOCAL_MESSAGE, GLOBAL_MESSAGE)


@dataclass
class Message:
    """The fields of worldql_server/src/structures/message.rs:14-24 this path reads."""
    instruction: str
    sender_uuid: Hashable
    world_name: str = ""
    position: Optional[Vector3] = None
    replication: int = abi.REPL_EXCEPT_SELF  # wire code; unknown codes route as ExceptSelf


@dataclass(frozen=True)
class PeerMapBroadcast:
    """A GlobalMessage to "@global" (global_message.rs:18-35): a PeerMap operation with no table
    lookup — broadcast_except(sender) / broadcast_all / the sender alone, by `replication`."""
    replication: int
    sender_uuid: Hashable


Recipients = Union[List[Hashable], PeerMapBroadcast]


def _sanitized(name: str) -> Optional[str]:
    try:
        return sanitize_world_name(name)
    except SanitizeError:
        return None


class SubscriptionProcessor:
    """Owns a WorldMap and processes ticks of events in arrival order."""

    def __init__(self, world_map: WorldMap,
                 broadcast: Optional[Callable[[Message, Recipients], None]] = None):
        self.world_map = world_map
        self.broadcast = broadcast

    def process_tick(self, events: Sequence[Message]) -> List[Optional[Recipients]]:
        """For every event: the recipients of a Local/GlobalMessage (a list of peers, or a
        PeerMapBroadcast for "@global"), or None when nothing is broadcast — a table event, a
        message dropped by validation, or one to a world that does not exist (local_message.rs:52-56,
        global_message.rs:50-54)."""
        results: List[Optional[Recipients]] = [None] * len(events)
        i = 0
        while i < len(events):
            ins = events[i].instruction
            if ins not in _TABLE_EVENTS and ins not in _READ_EVENTS:
                raise ValueError(f"not a subscription-task event: {ins}")  # thread.rs:136 panics
            is_read = ins in _READ_EVENTS
            j = i
            while j < len(events) and (events[j].instruction in _READ_EVENTS) == is_read:
                if events[j].instruction not in _TABLE_EVENTS and events[j].instruction not in _READ_EVENTS:
                    break
                j += 1
            if is_read:
                self._read_run(events, i, j, results)
            else:
                self._apply_run(events[i:j])
            i = j
        return results

    # area_subscribe.rs:10-52 / area_unsubscribe.rs:10-52 / thread.rs:124-125
    def _apply_run(self, events: Sequence[Message]) -> None:
        wm = self.world_map
        ops, gone = [], {}
        for ev in events:
            if ev.instruction == DISCONNECT:
                pid = wm.peer_ids.lookup(ev.sender_uuid)
                if pid is not None:  # a peer the table never saw has nothing to remove
                    ops.append(abi.make_op(abi.WORLD_INVALID, pid, abi.OP_REMOVE_PEER))
                    gone[ev.sender_uuid] = True
                continue
            if ev.world_name == GLOBAL_WORLD:  # :18-20
                continue
            name = _sanitized(ev.world_name)  # :23-33
            if name is None or ev.position is None:  # :35-46
                continue
            am = wm.get_mut(name)  # creates the world, also on unsubscribe (:137 / :189)
            p = ev.position
            if ev.instruction == AREA_SUBSCRIBE:
                ops.append(abi.make_op(am.world_id, wm.peer_ids.id(ev.sender_uuid), abi.OP_SUBSCRIBE,
                                       pos=(p.x, p.y, p.z)))
                gone.pop(ev.sender_uuid, None)  # back in the same batch: it keeps its (live) id
            else:
                pid = wm.peer_ids.lookup(ev.sender_uuid)
                if pid is not None:  # a peer without an id holds no subscription to remove
                    ops.append(abi.make_op(am.world_id, pid, abi.OP_UNSUBSCRIBE, pos=(p.x, p.y, p.z)))
        if ops:
            wm.router.apply_ops(np.array(ops, dtype=abi.OP_DTYPE))
        for uuid in gone:  # the table holds nothing of these peers any more: recycle their ids
            wm.peer_ids.release(uuid)

    def _sender_id(self, uuid) -> int:
        """A sender the table never saw is subscribed nowhere: NO_PEER matches no peer (ids are
        < 2^32 - 1), so ExceptSelf keeps everyone and OnlySelf no one, as in the reference."""
        pid = self.world_map.peer_ids.lookup(uuid)
        return NO_PEER if pid is None else pid

    def _read_run(self, events, lo: int, hi: int, results) -> None:
        wm = self.world_map
        # local_message.rs:10-89
        l_idx, pos, l_world, l_sender, l_repl = [], [], [], [], []
        # global_message.rs:10-88
        g_idx, g_world, g_sender, g_repl = [], [], [], []
        for k in range(lo, hi):
            ev = events[k]
            if ev.instruction == GLOBAL_MESSAGE:
                if ev.world_name == GLOBAL_WORLD:  # :18-35, every connected peer
                    rp = int(ev.replication) & 0xFF
                    results[k] = PeerMapBroadcast(rp if rp <= abi.REPL_ONLY_SELF else abi.REPL_EXCEPT_SELF,
                                                  ev.sender_uuid)  # unknown codes: replication.rs:40
                    continue
                name = _sanitized(ev.world_name)  # :37-47
                am = wm.get(name) if name is not None else None
                if am is None:  # :50-54 no subscriptions in this world
                    continue
                g_idx.append(k)
                g_world.append(am.world_id)
                g_sender.append(self._sender_id(ev.sender_uuid))
                g_repl.append(int(ev.replication) & 0xFF)
                continue
            if ev.world_name == GLOBAL_WORLD or ev.position is None:  # :17-37
                continue
            name = _sanitized(ev.world_name)  # :40-50
            am = wm.get(name) if name is not None else None
            if am is None:  # :52-56 no subscriptions in this world: nothing is broadcast
                continue
            l_idx.append(k)
            pos.append((ev.position.x, ev.position.y, ev.position.z))
            l_world.append(am.world_id)
            l_sender.append(self._sender_id(ev.sender_uuid))
            l_repl.append(int(ev.replication) & 0xFF)
        if l_idx:
            offsets, peers, _ = wm.router.route(np.array(pos, np.float64), np.array(l_world, np.uint32),
                                                np.array(l_sender, np.uint32), np.array(l_repl, np.uint8))
            for n, k in enumerate(l_idx):
                results[k] = wm.peer_ids.peers(peers[offsets[n]:offsets[n + 1]])
        if g_idx:
            offsets, peers, _ = wm.router.route_global(np.array(g_world, np.uint32), np.array(g_sender, np.uint32),
                                                       np.array(g_repl, np.uint8))
            for n, k in enumerate(g_idx):
                results[k] = wm.peer_ids.peers(peers[offsets[n]:offsets[n + 1]])
        if self.broadcast is not None:
            for k in range(lo, hi):
                if results[k] is not None:
                    self.broadcast(events[k], results[k])
