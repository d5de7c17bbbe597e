"""Host side of the hot path: message validation and tick batching around the GPU table.

Mirrors, at tick granularity, the reference's single subscription task
`handle_sub_messages` (worldql_server/src/processing/thread.rs:113-148) and the handlers it
calls: handle_local_message (local_message.rs:10-89), handle_area_subscribe
(area_subscribe.rs:10-52), handle_area_unsubscribe (area_unsubscribe.rs:10-52) and the
disconnect path WorldMap::remove_peer (thread.rs:124-125).

Ordering contract ("flush-on-reorder"): a tick is the arrival-ordered list of
events. Consecutive table events (subscribe / unsubscribe / disconnect) form one op batch,
consecutive LocalMessages one route batch, and batches run in arrival order — so every message
sees exactly the table the sequential reference would have shown it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Hashable, List, Optional, Sequence

import numpy as np

from . import abi
from .subscriptions import Vector3, WorldMap
from .world_names import GLOBAL_WORLD, SanitizeError, sanitize_world_name

LOCAL_MESSAGE = "LocalMessage"
AREA_SUBSCRIBE = "AreaSubscribe"
AREA_UNSUBSCRIBE = "AreaUnsubscribe"
DISCONNECT = "Disconnect"  # a uuid arriving on remove_rx (thread.rs:124-125)


@dataclass
class Message:
    """The fields of worldql_server/src/structures/message.rs:14-24 this path reads."""
    instruction: str
    sender_uuid: Hashable
    world_name: str = ""
    position: Optional[Vector3] = None
    replication: int = abi.REPL_EXCEPT_SELF  # wire code; unknown codes route as ExceptSelf


def _sanitized(name: str) -> Optional[str]:
    try:
        return sanitize_world_name(name)
    except SanitizeError:
        return None


class SubscriptionProcessor:
    """Owns a WorldMap and processes ticks of events in arrival order."""

    def __init__(self, world_map: WorldMap,
                 broadcast: Optional[Callable[[Message, List[Hashable]], None]] = None):
        self.world_map = world_map
        self.broadcast = broadcast

    def process_tick(self, events: Sequence[Message]) -> List[Optional[List[Hashable]]]:
        """Returns, for every event, the recipients of a LocalMessage (None if dropped by
        validation or not a LocalMessage)."""
        results: List[Optional[List[Hashable]]] = [None] * len(events)
        i = 0
        while i < len(events):
            is_msg = events[i].instruction == LOCAL_MESSAGE
            j = i
            while j < len(events) and (events[j].instruction == LOCAL_MESSAGE) == is_msg:
                j += 1
            if is_msg:
                self._route_run(events, i, j, results)
            else:
                self._apply_run(events[i:j])
            i = j
        return results

    # area_subscribe.rs:10-52 / area_unsubscribe.rs:10-52 / thread.rs:124-125
    def _apply_run(self, events: Sequence[Message]) -> None:
        wm = self.world_map
        ops = []
        for ev in events:
            if ev.instruction == DISCONNECT:
                ops.append(abi.make_op(abi.WORLD_INVALID, wm.peer_ids.id(ev.sender_uuid), abi.OP_REMOVE_PEER))
                continue
            if ev.instruction not in (AREA_SUBSCRIBE, AREA_UNSUBSCRIBE):
                raise ValueError(f"not a subscription-table event: {ev.instruction}")
            if ev.world_name == GLOBAL_WORLD:  # :18-20
                continue
            name = _sanitized(ev.world_name)  # :23-33
            if name is None or ev.position is None:  # :35-46
                continue
            am = wm.get_mut(name)  # creates the world, also on unsubscribe (:137 / :189)
            kind = abi.OP_SUBSCRIBE if ev.instruction == AREA_SUBSCRIBE else abi.OP_UNSUBSCRIBE
            p = ev.position
            ops.append(abi.make_op(am.world_id, wm.peer_ids.id(ev.sender_uuid), kind, pos=(p.x, p.y, p.z)))
        if ops:
            wm.router.apply_ops(np.array(ops, dtype=abi.OP_DTYPE))

    # local_message.rs:10-89
    def _route_run(self, events, lo: int, hi: int, results) -> None:
        wm = self.world_map
        idx, pos, world, sender, repl = [], [], [], [], []
        for k in range(lo, hi):
            ev = events[k]
            if ev.world_name == GLOBAL_WORLD or ev.position is None:  # :17-37
                continue
            name = _sanitized(ev.world_name)  # :40-50
            if name is None:
                continue
            am = wm.get(name)
            results[k] = []
            if am is None:  # :52-56 no subscriptions in this world
                continue
            idx.append(k)
            pos.append((ev.position.x, ev.position.y, ev.position.z))
            world.append(am.world_id)
            sender.append(wm.peer_ids.id(ev.sender_uuid))
            repl.append(int(ev.replication) & 0xFF)
        if idx:
            offsets, peers, _ = wm.router.route(np.array(pos, np.float64), np.array(world, np.uint32),
                                                np.array(sender, np.uint32), np.array(repl, np.uint8))
            for n, k in enumerate(idx):
                results[k] = wm.peer_ids.peers(peers[offsets[n]:offsets[n + 1]])
        if self.broadcast is not None:
            for k in range(lo, hi):
                if results[k] is not None:
                    self.broadcast(events[k], results[k])
