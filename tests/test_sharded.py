"""Cube-hash sharded routing (worldql_server_amd/sharded.py).

CPU: the exchange logic with gloo (world_size 2 and 3, one process per rank) and with the
thread exchange (4 shards in one process); the C restatement stands in for each shard's GPU
table (OracleShard below — test infrastructure). GPU: the same ShardedRouter on real kernels,
G shards as threads sharing cuda:0, against one oracle holding the whole table.
"""
import os
import socket
import threading

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import oracle as orc
from worldql_server_amd import abi, synth
from worldql_server_amd.sharded import DeviceShard, DistExchange, ShardedRouter, ThreadExchange, ThreadHub


# ---------------------------------------------------------------------------------------------
# workload: several worlds, 3x3x3 subscriptions, churn (unsubscribe + REMOVE_PEER), raw keys,
# mixed replication codes
# ---------------------------------------------------------------------------------------------
def make_tick(n_peers=400, n_msgs=3000, seed=11):
    w = synth.uniform_box(11, n_peers, n_msgs, 96.0, neighbourhood=True, n_worlds=3, repl_mode="mixed")
    rng = np.random.default_rng(seed)
    subs = w.ops
    unsub = subs[rng.choice(len(subs), len(subs) // 10, replace=False)].copy()
    unsub["kind"] = abi.OP_UNSUBSCRIBE
    rm = abi.ops_array(np.full(5, abi.WORLD_INVALID, np.uint32), rng.choice(n_peers, 5, replace=False),
                       np.full(5, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((5, 3)))
    rm1 = abi.ops_array(np.array([1], np.uint32), np.array([7], np.uint32),
                        np.array([abi.OP_REMOVE_PEER], np.uint8), pos=np.zeros((1, 3)))
    raw = abi.ops_array(np.zeros(50, np.uint32), rng.integers(0, n_peers, 50).astype(np.uint32),
                        np.zeros(50, np.uint8), key=rng.integers(-3, 3, (50, 3)) * 5)  # off-grid raw keys
    resub = subs[rng.choice(len(subs), 200, replace=False)].copy()
    ops = abi.concat_ops([subs, unsub, rm, rm1, raw, resub])
    return w, ops


def expected(w, ops, lo, hi):
    o = orc.COracle(w.cube_size)
    o.apply_ops(ops)
    offs, peers, _ = o.route(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])
    return [peers[offs[i]:offs[i + 1]] for i in range(hi - lo)]


class OracleShard:
    """DeviceShard's interface over the C restatement, on CPU tensors (tests only)."""

    def __init__(self, cube_size):
        self.o = orc.COracle(cube_size)
        self.cube_size = cube_size
        self.cap = 1 << 40
        self.radius, self.peer_pos = 0.0, None

    def set_radius(self, radius, peer_pos):
        self.radius, self.peer_pos = radius, np.asarray(peer_pos, np.float64)

    def counters_i64(self):
        return torch.zeros(3, dtype=torch.int64)  # the restatement never reports an error

    check_counters = staticmethod(DeviceShard.check_counters)

    def shard_ops(self, ops, G):
        k = np.where(ops["key_is_raw"][:, None] == 1, ops["key"],
                     orc.coord_clamp_np(ops["pos"], self.cube_size))
        own = orc.shard_of_np(ops["world"], k[:, 0], k[:, 1], k[:, 2], G)
        own[ops["kind"] == abi.OP_REMOVE_PEER] = abi.SHARD_ALL
        return own

    def apply_ops(self, ops):
        self.o.apply_ops(ops)

    def shard(self, pos, keys, world, sender, repl, G):
        world, sender, repl = world.numpy(), sender.numpy(), repl.numpy()
        k = keys.numpy() if keys is not None else orc.coord_clamp_np(pos.numpy(), self.cube_size)
        own = orc.shard_of_np(world, k[:, 0], k[:, 1], k[:, 2], G)
        order = np.argsort(own, kind="stable")
        recs = np.zeros(len(world), abi.MSG_REC_DTYPE)
        recs["key"], recs["world"], recs["sender"] = k[order], world[order], sender[order]
        recs["msg"], recs["repl"] = order, repl[order]
        if self.radius > 0 and pos is not None:  # the owner's radius filter needs the positions
            recs["key"] = np.ascontiguousarray(pos.numpy()[order]).view(np.int64)
            recs["flags"] = abi.REC_POS
        counts = np.bincount(own, minlength=G).astype(np.int32)
        return torch.from_numpy(recs.view(np.uint8).reshape(-1, 40).copy()), torch.from_numpy(counts)

    def route_records(self, recs, n, P_hint=None):
        r = recs.numpy().reshape(-1).view(abi.MSG_REC_DTYPE)
        if self.radius > 0:
            pos = np.where((r["flags"] & abi.REC_POS)[:, None] != 0, np.ascontiguousarray(r["key"]).view(np.float64),
                           np.nan)
            offs, peers = self.o.route_radius(pos, r["world"], r["sender"], r["repl"], self.peer_pos, self.radius)[:2]
            return torch.from_numpy(offs.astype(np.int32)), torch.from_numpy(peers.astype(np.int32))
        offs, peers, _ = self.o.route(None, r["world"], r["sender"], r["repl"], keys=r["key"])
        return torch.from_numpy(offs.astype(np.int32)), torch.from_numpy(peers.astype(np.int32))

    def route_local(self, pos, keys, world, sender, repl, P_hint=None):
        offs, peers, _ = self.o.route(None if pos is None else pos.numpy(), world.numpy(), sender.numpy(),
                                      repl.numpy(), keys=None if keys is None else keys.numpy())
        return torch.from_numpy(offs.astype(np.int32)), torch.from_numpy(peers.astype(np.int32))


def _slice(w, rank, G):
    M = len(w.world)
    lo, hi = rank * M // G, (rank + 1) * M // G
    return lo, hi


def _run_rank(be, ex, w, ops, rank, G, device):
    sr = ShardedRouter(be, ex)
    sr.apply_ops(ops)
    lo, hi = _slice(w, rank, G)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    tick = sr.tick(t(w.world[lo:hi]), t(w.sender[lo:hi]), t(w.repl[lo:hi]), pos=t(w.pos[lo:hi]))
    return lo, hi, tick.per_message(hi - lo)


def _check(w, ops, lo, hi, got):
    want = expected(w, ops, lo, hi)
    for m in range(hi - lo):
        assert np.array_equal(np.sort(got[m]), want[m]), (lo + m, got[m], want[m])


# ---------------------------------------------------------------------------------------------
# CPU
# ---------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, G, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    try:
        w, ops = make_tick()
        lo, hi, got = _run_rank(OracleShard(w.cube_size), DistExchange(), w, ops, rank, G, "cpu")
        _check(w, ops, lo, hi, got)
        out[rank] = sum(len(g) for g in got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("G", [2, 3])
def test_cube_sharded_tick_gloo(G):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_gloo_worker, args=(G, _free_port(), out), nprocs=G, start_method="spawn", join=True)
    assert all(out[r] > 0 for r in range(G))


def _thread_cluster(G, make_backend, device):
    w, ops = make_tick()
    hub = ThreadHub(G)
    res, errs = {}, []

    def body(rank):
        try:
            be = make_backend(rank)
            if device != "cpu":
                with torch.cuda.stream(be.stream):
                    res[rank] = _run_rank(be, ThreadExchange(hub, rank), w, ops, rank, G, device)
            else:
                res[rank] = _run_rank(be, ThreadExchange(hub, rank), w, ops, rank, G, device)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    for r in range(G):
        _check(w, ops, *res[r])
    return res


def test_cube_sharded_tick_threads_cpu():
    _thread_cluster(4, lambda r: OracleShard(16), "cpu")


def _radius_cluster(G, make_backend, device):
    """C5-shaped (scaled) moving entities with the radius filter, sharded by cube over G threads:
    every shard holds all peer positions; the records carry message positions to the owners."""
    from worldql_server_amd import synth_ext
    c5 = synth_ext.config_c5(scale=0.003)
    init = c5.initial_ops()
    c5.step()
    ops = abi.concat_ops([init, c5.step()])
    pos, world, sender, repl = c5.messages()
    repl = synth.stream(5, 77).below(3, len(world)).astype(np.uint8)
    o = orc.COracle(16)
    o.apply_ops(ops)
    offs, peers = o.route_radius(pos, world, sender, repl, c5.pos, c5.radius)[:2]
    want = [peers[offs[i]:offs[i + 1]] for i in range(len(world))]
    hub = ThreadHub(G)
    res, errs = {}, []

    def body(rank):
        try:
            be = make_backend(rank)
            be.set_radius(c5.radius, c5.pos)
            sr = ShardedRouter(be, ThreadExchange(hub, rank))
            sr.apply_ops(ops)
            lo, hi = rank * len(world) // G, (rank + 1) * len(world) // G
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
            if device != "cpu":
                with torch.cuda.stream(be.stream):
                    tick = sr.tick(t(world[lo:hi]), t(sender[lo:hi]), t(repl[lo:hi]), pos=t(pos[lo:hi]))
            else:
                tick = sr.tick(t(world[lo:hi]), t(sender[lo:hi]), t(repl[lo:hi]), pos=t(pos[lo:hi]))
            res[rank] = (lo, hi, tick.per_message(hi - lo))
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(G)]
    for t_ in th:
        t_.start()
    for t_ in th:
        t_.join()
    if errs:
        raise errs[0]
    total = 0
    for r in range(G):
        lo, hi, got = res[r]
        for m in range(hi - lo):
            assert np.array_equal(got[m], want[lo + m]), (lo + m, got[m], want[lo + m])
            total += len(got[m])
    assert total > 0


def test_radius_sharded_tick_threads_cpu():
    _radius_cluster(3, lambda r: OracleShard(16), "cpu")


def test_shard_owner_split_is_balanced():
    w, ops = make_tick(n_peers=2000, n_msgs=20000)
    be = OracleShard(16)
    own = be.shard_ops(w.ops, 8)
    c = np.bincount(own, minlength=8)
    assert c.min() > 0.8 * len(own) / 8


# ---------------------------------------------------------------------------------------------
# GPU: real kernels, G shards as threads on cuda:0
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 2, 3, 5])
def test_cube_sharded_tick_gpu_threads(G):
    from worldql_server_amd.router import Router
    from worldql_server_amd.sharded import DeviceShard

    def make(rank):
        return DeviceShard(Router(16, 0), torch.cuda.Stream(device=0))

    _thread_cluster(G, make, "cuda:0")


@pytest.mark.gpu
def test_shard_kernels_match_restatement_gpu():
    from worldql_server_amd.router import Router
    from worldql_server_amd.sharded import DeviceShard
    w, ops = make_tick(n_peers=1000, n_msgs=50_000)
    r = Router(16, 0)
    be = DeviceShard(r, torch.cuda.Stream(device=0))
    fake = OracleShard(16)
    for G in (1, 2, 7, 8, 64):
        assert np.array_equal(r.shard_ops(ops, G), fake.shard_ops(ops, G))
        args = [torch.from_numpy(np.ascontiguousarray(a)) for a in (w.pos, w.world, w.sender, w.repl)]
        with torch.cuda.stream(be.stream):
            recs, counts = be.shard(args[0].cuda(), None, *[a.cuda() for a in args[1:]], G)
            be.stream.synchronize()
        want_recs, want_counts = fake.shard(args[0], None, *args[1:], G)
        assert np.array_equal(counts.cpu().numpy(), want_counts.numpy())
        assert np.array_equal(recs.cpu().numpy(), want_recs.numpy())  # stable grouping, bit-exact


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 2, 3])
def test_radius_sharded_tick_gpu_threads(G):
    from worldql_server_amd.router import Router
    from worldql_server_amd.sharded import DeviceShard

    def make(rank):
        return DeviceShard(Router(16, 0), torch.cuda.Stream(device=0))

    _radius_cluster(G, make, "cuda:0")
