"""Cube-hash sharded routing over G GPUs, one process per GPU.

The reference keeps one `WorldMap` in one task (worldql_server/src/processing/thread.rs:113-148).
Here the table is partitioned by the owner of each (world, cube) bucket (`shard_of` in
csrc/wq_shard.hip) and a tick of LocalMessages becomes

    shard      each GPU quantises the messages it ingested and groups them by owner (40-B records)
    exchange   all-to-all of the per-owner counts, then of the records          (RCCL over xGMI)
    route      the owner runs count / scan / emit on what it received (local_message.rs:52-86)
    return     all-to-all of per-message recipient counts, then of the peer ids

so every GPU ends with the recipients of exactly the messages it ingested. Two host syncs per
tick read the split sizes all_to_all_single needs. Subscription ops are host-partitioned on
ingest: every rank sees the op stream and applies, in order, the ops it owns plus every
REMOVE_PEER (`apply_ops`). Results are identical to one router holding the whole table.

`Exchange` implementations: `DistExchange` (torch.distributed: RCCL on GPUs, gloo on CPU) and
`ThreadExchange` (G shards as threads of one process — rehearses G > 1 on a single GPU).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass

import numpy as np
import torch

from . import abi


# ---------------------------------------------------------------------------------------------
# exchanges
# ---------------------------------------------------------------------------------------------
class DistExchange:
    """all_to_all_single over a torch.distributed process group (one rank per GPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits) -> None:
        self.dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=self.group)


class LocalExchange:
    """G = 1: no exchange (the single-GPU path)."""
    rank, size = 0, 1


class ThreadHub:
    """Shared mailbox of a ThreadExchange group."""

    def __init__(self, size: int):
        self.size = size
        self.barrier = threading.Barrier(size)
        self.box = [[None] * size for _ in range(size)]


class ThreadExchange:
    """all-to-all between G threads of one process (each thread drives one shard)."""

    def __init__(self, hub: ThreadHub, rank: int):
        self.hub = hub
        self.rank = rank
        self.size = hub.size

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits) -> None:
        if inp.is_cuda:
            torch.cuda.current_stream(inp.device).synchronize()
        chunks = torch.split(inp, list(in_splits))
        for d in range(self.size):
            self.hub.box[self.rank][d] = chunks[d]
        self.hub.barrier.wait()
        parts = [self.hub.box[s][self.rank] for s in range(self.size)]
        assert [int(p.shape[0]) for p in parts] == list(out_splits), "split sizes disagree"
        if out.shape[0]:
            torch.cat(parts, out=out)
        if out.is_cuda:
            torch.cuda.current_stream(out.device).synchronize()
        self.hub.barrier.wait()


# ---------------------------------------------------------------------------------------------
# per-GPU backend over the C ABI
# ---------------------------------------------------------------------------------------------
class DeviceShard:
    """One shard's table on one GPU (a Router) with torch-tensor inputs on `stream`."""

    def __init__(self, router, stream: torch.cuda.Stream):
        self.router = router
        self.stream = stream
        self.device = stream.device
        router.set_stream(stream.cuda_stream)
        self.cap = 0
        self._peers = None
        # wq_route_counters of the latest route call (P, F, overflow, error), device memory
        self.counters = torch.zeros(abi.COUNTERS_DTYPE.itemsize, dtype=torch.uint8, device=self.device)

    def shard_ops(self, ops: np.ndarray, n_shards: int) -> np.ndarray:
        return self.router.shard_ops(ops, n_shards)

    def apply_ops(self, ops: np.ndarray) -> None:
        self.router.apply_ops(ops)

    def set_radius(self, radius: float, peer_pos) -> None:
        """C5: every shard holds every peer's position; records then carry message positions."""
        self.router.set_peer_positions(peer_pos)
        self.router.set_radius(radius)

    def shard(self, pos, keys, world, sender, repl, n_shards: int):
        M = int(world.shape[0])
        recs = torch.empty((M, abi.MSG_REC_DTYPE.itemsize), dtype=torch.uint8, device=self.device)
        counts = torch.empty(n_shards, dtype=torch.int32, device=self.device)
        self.router.shard_messages_device(_ptr(pos), _ptr(keys), world.data_ptr(), sender.data_ptr(),
                                          repl.data_ptr(), M, n_shards, recs.data_ptr(), counts.data_ptr())
        return recs, counts

    def route_records(self, recs: torch.Tensor, n: int, P_hint: int | None = None):
        """CSR offsets (int32[n+1]) and the pair buffer (int32[cap]) of the received records.
        With P_hint > cap the buffer grows first (the caller re-runs after reading P)."""
        if P_hint is not None and P_hint > self.cap:
            self.cap = int(P_hint * 1.25) + 1024
            self._peers = None
        if self._peers is None:
            self._peers = torch.empty(max(self.cap, 1), dtype=torch.int32, device=self.device)
        offsets = torch.empty(n + 1, dtype=torch.int32, device=self.device)
        self.router.route_records_device(recs.data_ptr() if n else None, n, offsets.data_ptr(),
                                         self._peers.data_ptr() if self.cap else None, None, self.cap,
                                         self.counters.data_ptr())
        return offsets, self._peers

    def route_local(self, pos, keys, world, sender, repl, P_hint: int | None = None):
        M = int(world.shape[0])
        if P_hint is not None and P_hint > self.cap:
            self.cap = int(P_hint * 1.25) + 1024
            self._peers = None
        if self._peers is None:
            self._peers = torch.empty(max(self.cap, 1), dtype=torch.int32, device=self.device)
        offsets = torch.empty(M + 1, dtype=torch.int32, device=self.device)
        self.router.route_device(_ptr(pos), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                                 offsets.data_ptr(), self._peers.data_ptr() if self.cap else None, None,
                                 self.cap, self.counters.data_ptr(), keys_ptr=_ptr(keys))
        return offsets, self._peers

    def counters_i64(self) -> torch.Tensor:
        """The latest route call's wq_route_counters as 3 int64 words {P, F, overflow | error << 32}
        (device), so a host sync the tick already makes can carry them."""
        return self.counters.view(torch.int64)

    @staticmethod
    def check_counters(words) -> None:
        """Raises when a route call reported an error (host copy of counters_i64)."""
        err = (int(words[2]) >> 32) & 0xFFFFFFFF
        if err & 8:  # as Router.check_health: the table still misses a batch the device could not apply
            raise RuntimeError(f"wq error {abi.WQ_E_INVALID}: a tick ran on a table still missing an incremental "
                               f"batch the device could not apply (error bits {err:#x})")
        if err:
            code = abi.WQ_E_TIMEOUT if err & 4 else abi.WQ_E_CAPACITY
            raise RuntimeError(f"wq error {code}: route counters report error bits {err:#x}")

    def read_counters(self):
        """(P, F) of the latest route call (synchronises the stream)."""
        self.stream.synchronize()
        c = self.counters.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]
        assert c["error"] == 0, c
        return int(c["n_pairs"]), int(c["n_candidates"])


def _ptr(t):
    return None if t is None else t.data_ptr()


# ---------------------------------------------------------------------------------------------
# the sharded router
# ---------------------------------------------------------------------------------------------
@dataclass
class ShardedTick:
    """Recipients of this rank's ingested messages, as a CSR over `order` (row i is message
    order[i] of the batch): offsets int64[M+1], peers int32[P] (ascending per row)."""
    order: torch.Tensor
    offsets: torch.Tensor
    peers: torch.Tensor

    def per_message(self, n_msgs: int):
        """{message index: np.ndarray of peers} (host; for tests)."""
        order = self.order.cpu().numpy()
        off = self.offsets.cpu().numpy()
        peers = self.peers.cpu().numpy().astype(np.uint32)
        out = [np.empty(0, np.uint32)] * n_msgs
        for i, m in enumerate(order):
            out[int(m)] = peers[off[i]:off[i + 1]]
        return out


class ShardedRouter:
    """WorldMap partitioned by cube hash over `exchange.size` shards; this object is one shard."""

    def __init__(self, backend, exchange):
        self.be = backend
        self.ex = exchange
        self.G = exchange.size
        self.rank = exchange.rank
        self.last_recv = 0  # messages routed on this shard in the latest tick

    def apply_ops(self, ops: np.ndarray) -> None:
        """The full op stream of the tick (every rank sees it); keep what this shard owns."""
        ops = np.ascontiguousarray(ops, dtype=abi.OP_DTYPE)
        if self.G == 1:
            self.be.apply_ops(ops)
            return
        owner = self.be.shard_ops(ops, self.G)
        keep = (owner == self.rank) | (owner == abi.SHARD_ALL)
        if keep.any():
            self.be.apply_ops(np.ascontiguousarray(ops[keep]))

    def tick(self, world, sender, repl, pos=None, keys=None) -> ShardedTick:
        """Route this rank's ingested messages (device tensors) through their owner shards."""
        G, ex, be = self.G, self.ex, self.be
        M = int(world.shape[0])
        dev = world.device
        if G == 1:
            self.last_recv = M
            offsets, peers = be.route_local(pos, keys, world, sender, repl)
            P = 0
            if M:  # one host sync: P and the call's counters
                h = torch.cat([offsets[M:M + 1].to(torch.int64), be.counters_i64()]).cpu().tolist()
                be.check_counters(h[1:])
                P = h[0]
            if P > be.cap:
                offsets, peers = be.route_local(pos, keys, world, sender, repl, P_hint=P)
            return ShardedTick(torch.arange(M, device=dev), offsets.to(torch.int64), peers[:P])

        # 1. group by owner; exchange counts, then records
        recs, send_counts = be.shard(pos, keys, world, sender, repl, G)
        recv_counts = torch.empty_like(send_counts)
        ones = [1] * G
        ex.all_to_all(recv_counts, send_counts, ones, ones)
        sc_rc = torch.cat([send_counts, recv_counts]).cpu().tolist()  # host sync 1
        sc, rc = sc_rc[:G], sc_rc[G:]
        R = sum(rc)
        self.last_recv = R
        recv = torch.empty((R, recs.shape[1]), dtype=recs.dtype, device=dev)
        ex.all_to_all(recv, recs, rc, sc)

        # 2. route on the owner; per-source pair sums -> exchange
        offsets, peers = be.route_records(recv, R)
        bounds = torch.tensor(np.concatenate([[0], np.cumsum(rc)]), dtype=torch.int64, device=dev)
        off_b = offsets.index_select(0, bounds).to(torch.int64)
        pair_send = (off_b[1:] - off_b[:-1]).to(torch.int64)
        pair_recv = torch.empty_like(pair_send)
        ex.all_to_all(pair_recv, pair_send, ones, ones)
        ps_pr = torch.cat([pair_send, pair_recv, be.counters_i64()]).cpu().tolist()  # host sync 2
        be.check_counters(ps_pr[2 * G:])  # a route error must not hand back wrong pairs
        ps, pr = ps_pr[:G], ps_pr[G:2 * G]
        P = sum(ps)
        if P > be.cap:  # the pair buffer was too small: offsets are right, re-run with room
            offsets, peers = be.route_records(recv, R, P_hint=P)

        # 3. return per-message counts and the peers to the ingesting ranks
        counts_back = (offsets[1:] - offsets[:-1]) if R else torch.empty(0, dtype=torch.int32, device=dev)
        ret_counts = torch.empty(M, dtype=torch.int32, device=dev)
        ex.all_to_all(ret_counts, counts_back.contiguous(), sc, rc)
        ret_peers = torch.empty(sum(pr), dtype=torch.int32, device=dev)
        ex.all_to_all(ret_peers, peers[:P], pr, ps)
        out_off = torch.zeros(M + 1, dtype=torch.int64, device=dev)
        if M:
            torch.cumsum(ret_counts.to(torch.int64), 0, out=out_off[1:])
        order = recs.view(torch.int32)[:, 8].to(torch.int64) if M else torch.empty(0, dtype=torch.int64, device=dev)
        return ShardedTick(order, out_off, ret_peers)
