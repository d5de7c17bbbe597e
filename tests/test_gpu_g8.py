"""Every multi-GPU form at the node's real shard count, G = 8, against the oracle
holding the WHOLE table (area_map.rs:52-60: whatever the split, each message's recipients are the one
table's). The box has one GPU, so the eight shards / devices are eight handles on cuda:0 — the same
kernels, exchanges and budgets as on an 8-GPU node, without the link time.

  hub slot tick      C3-shaped (scaled to 1M messages, hotspot skew), an exact first tick, a churn
                     batch, a budgeted second tick; every shard's slice checked by wqo_route_check
  hub radius tick    C5-shaped (1M moving entities, r = 16): the owners return rows and pools, every
                     ingesting shard filters by radius; two ticks with the move's churn between them
  hub irregular      keys without a packed form (two slots on the wire), by position and by raw key
  hub owner slots    the owner form (pairs left on the owners) on the C3-shaped tick, mapped back to
                     every source's messages
  multi handle       wq_router_create_multi_mode with 8 devices, both layouts, the slice form
                     (wq_route_tick_slices_device) on the C3-shaped tick
"""
import threading

import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi

pytestmark = pytest.mark.gpu

G = 8


def _slice(M, rank):
    return rank * M // G, (rank + 1) * M // G


def _run_shards(body, timeout=600):
    errors = []

    def wrap(rank):
        try:
            body(rank)
        except Exception as e:  # noqa: BLE001
            errors.append((rank, e))

    th = [threading.Thread(target=wrap, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not any(t.is_alive() for t in th), "a shard did not finish"
    assert not errors, errors


def _tick(r, pos, world, sender, repl, dev, keys=None, cap_per_msg=64):
    """One sharded tick of host arrays on shard r: (rc, offsets, peers), copied out after a
    WQ_E_CAPACITY."""
    import torch
    M = len(world)
    kt = None if keys is None else torch.from_numpy(np.ascontiguousarray(keys)).to(dev)
    p = torch.from_numpy(np.ascontiguousarray(pos)).to(dev)
    wo = torch.from_numpy(np.ascontiguousarray(world).view(np.int32)).to(dev)
    se = torch.from_numpy(np.ascontiguousarray(sender).view(np.int32)).to(dev)
    rp = torch.from_numpy(np.ascontiguousarray(repl)).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = cap_per_msg * M + 64
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    rc, P = r.sharded_route_device(None if kt is not None else p.data_ptr(), wo.data_ptr(), se.data_ptr(),
                                   rp.data_ptr(), M, offs.data_ptr(), peers.data_ptr(), None, cap,
                                   keys_ptr=None if kt is None else kt.data_ptr())
    if rc == abi.WQ_E_CAPACITY:
        peers = torch.empty(P, dtype=torch.int32, device=dev)
        r.sharded_copy_out(offs.data_ptr(), peers.data_ptr(), None, P)
    torch.cuda.synchronize(dev)
    return rc, offs.cpu().numpy().view(np.uint32), peers.cpu().numpy().view(np.uint32)[:P]


def _c3_churn(w, seed=41):
    """An unsubscribe of ~2% of the build's subscriptions and a few disconnects."""
    rng = np.random.default_rng(seed)
    un = w.ops[rng.choice(len(w.ops), len(w.ops) // 50, replace=False)].copy()
    un["kind"] = abi.OP_UNSUBSCRIBE
    rm = abi.ops_array(np.full(64, abi.WORLD_INVALID, np.uint32), rng.choice(w.n_peers, 64, replace=False),
                       np.full(64, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((64, 3)))
    return abi.concat_ops([un, rm])


def test_hub_g8_c3_slot_tick_route_check():
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Hub, Router
    w = synth_ext.config_c3(scale=0.1)
    churn = _c3_churn(w)
    M = len(w.world)
    assert M >= 1_000_000
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.set_fanout_hint(40.0)
        lo, hi = _slice(M, rank)
        args = (w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], dev)
        r.sharded_apply_ops(w.ops)
        first = _tick(r, *args)
        r.sharded_apply_ops(churn)
        second = _tick(r, *args)
        results[rank] = (first, second, r.shard_tick_stats(), r.stats()["n_entries"])

    _run_shards(body)
    for r in routers:
        r.close()
    hub.close()
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    checks = [[], []]
    for rank in range(G):
        lo, hi = _slice(M, rank)
        first = results[rank][0]
        checks[0].append(o.route_check(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], first[1],
                                       first[2]))
    o.apply_ops(churn)
    P = 0
    for rank in range(G):
        lo, hi = _slice(M, rank)
        second = results[rank][1]
        checks[1].append(o.route_check(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], second[1],
                                       second[2]))
        P += len(second[2])
        assert results[rank][2] == (1, 1), results[rank][2]  # an exact first tick, a budgeted second
    for k in range(2):
        assert all(bad == 0 for bad, _ in checks[k]), (k, checks[k])
    assert sum(res[3] for res in results) == o.counts()[0]  # the eight shards partition the table
    assert P > 2e7


def _owner_slot_view(r, pos, world, sender, repl, dev):
    """One wq_sharded_route_owner_slots tick of host arrays on shard r, its view copied to the host."""
    import ctypes

    import torch
    t = [torch.from_numpy(np.ascontiguousarray(x)).to(dev)
         for x in (pos, world.view(np.int32), sender.view(np.int32), repl)]
    torch.cuda.synchronize(dev)
    v = r.sharded_route_owner_slots(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), len(world))
    R, P, S = int(v.n_slots), int(v.n_pairs), int(v.send_seg[G])
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    offs, peers, perm = np.empty(R + 1, np.uint32), np.empty(max(P, 1), np.uint32), np.empty(max(S, 1), np.uint32)
    assert hip.hipMemcpy(offs.ctypes.data, v.offsets, (R + 1) * 4, 2) == 0
    if P:
        assert hip.hipMemcpy(peers.ctypes.data, v.peers, P * 4, 2) == 0
    if S:
        assert hip.hipMemcpy(perm.ctypes.data, v.send_perm, S * 4, 2) == 0
    return dict(offs=offs, peers=peers[:P], perm=perm[:S], seg=np.array(v.seg[:G + 1], np.int64),
                send_seg=np.array(v.send_seg[:G + 1], np.int64))


def _owner_views_to_csr(views, n_msgs):
    """The owners' CSRs over their received slots -> each source's CSR in message order (numpy)."""
    out = []
    for s in range(G):
        msg, cnt, start, owner = [], [], [], []
        for o in range(G):
            v = views[o]
            k0, k1 = v["seg"][s], v["seg"][s + 1]
            sb = views[s]["send_seg"][o]
            m = views[s]["perm"][sb:sb + (k1 - k0)].astype(np.int64)
            keep = m != 0xFFFFFFFF
            slots = np.arange(k0, k1)[keep]
            msg.append(m[keep])
            cnt.append((v["offs"][slots + 1] - v["offs"][slots]).astype(np.int64))
            start.append(v["offs"][slots].astype(np.int64))
            owner.append(np.full(int(keep.sum()), o))
        msg, cnt, start, owner = (np.concatenate(x) for x in (msg, cnt, start, owner))
        assert len(msg) == n_msgs[s] and len(np.unique(msg)) == n_msgs[s]  # every message once
        order = np.argsort(msg, kind="stable")
        cnt, start, owner = cnt[order], start[order], owner[order]
        offs = np.zeros(n_msgs[s] + 1, np.int64)
        offs[1:] = np.cumsum(cnt)
        peers = np.empty(int(offs[-1]), np.uint32)
        for o in range(G):  # each owner's rows, gathered in one vectorised copy
            sel = owner == o
            c, st, dst = cnt[sel], start[sel], offs[:-1][sel]
            if not c.sum():
                continue
            within = np.arange(int(c.sum())) - np.repeat(np.cumsum(c) - c, c)
            peers[np.repeat(dst, c) + within] = views[o]["peers"][np.repeat(st, c) + within]
        out.append((offs.astype(np.uint32), peers))
    return out


def test_hub_g8_c3_owner_slots_route_check():
    """The owner form on slots (wq_sharded_route_owner_slots) at G = 8 on the C3-shaped tick: an exact
    tick, a churn batch, a budgeted tick; the owners' CSRs mapped back to each source's messages
    through the sources' slot -> message maps, every slice checked by wqo_route_check."""
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Hub, Router
    w = synth_ext.config_c3(scale=0.1)
    churn = _c3_churn(w)
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.set_fanout_hint(40.0)
        lo, hi = _slice(M, rank)
        args = (w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], dev)
        r.sharded_apply_ops(w.ops)
        first = _owner_slot_view(r, *args)
        r.sharded_apply_ops(churn)
        second = _owner_slot_view(r, *args)
        results[rank] = (first, second, r.shard_tick_stats())

    _run_shards(body)
    for r in routers:
        r.close()
    hub.close()
    n_msgs = [_slice(M, s)[1] - _slice(M, s)[0] for s in range(G)]
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    P = 0
    for k in range(2):
        if k == 1:
            o.apply_ops(churn)
        csr = _owner_views_to_csr([res[k] for res in results], n_msgs)
        for s in range(G):
            lo, hi = _slice(M, s)
            bad, first_bad = o.route_check(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], *csr[s])
            assert bad == 0, (k, s, bad, first_bad)
            P += len(csr[s][1]) if k == 1 else 0
    for res in results:
        assert res[2] == (1, 1), res[2]  # an exact first tick, a budgeted second
    assert P > 2e7


def test_hub_g8_radius_slot_tick_route_check():
    """C5 over 8 shards: 1M moving entities with r = 16, a tick, the move's churn + new positions,
    a second tick; the ingesting shards filter the owners' rows by radius."""
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Hub, Router
    c5 = synth_ext.config_c5(scale=1.0)
    init = c5.initial_ops()
    pos0 = c5.pos.copy()
    ops1 = c5.step()
    pos1 = c5.pos.copy()
    N = c5.n
    world = np.zeros(N, np.uint32)
    sender = np.arange(N, dtype=np.uint32)
    repl = (sender % 3).astype(np.uint8)  # mixed replication: Except / Include / Only self
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.set_radius(c5.radius)
        lo, hi = _slice(N, rank)
        r.sharded_apply_ops(init)
        r.set_peer_positions(pos0)
        first = _tick(r, pos0[lo:hi], world[lo:hi], sender[lo:hi], repl[lo:hi], dev, cap_per_msg=16)
        r.sharded_apply_ops(ops1)
        r.set_peer_positions(pos1)
        second = _tick(r, pos1[lo:hi], world[lo:hi], sender[lo:hi], repl[lo:hi], dev, cap_per_msg=16)
        results[rank] = (first, second)

    _run_shards(body)
    for r in routers:
        r.close()
    hub.close()
    o = orc.COracle(16)
    o.set_fast(True)  # checker mode: the same sets without remove_subscription's O(#cubes) scan
    o.apply_ops(init)
    bad = []
    for k, (pos, ops) in enumerate([(pos0, None), (pos1, ops1)]):
        if ops is not None:
            o.apply_ops(ops)
        P = 0
        for rank in range(G):
            lo, hi = _slice(N, rank)
            rc, offs, peers = results[rank][k]
            bad.append(o.route_check(pos[lo:hi], world[lo:hi], sender[lo:hi], repl[lo:hi], offs, peers,
                                     peer_pos=pos, radius=c5.radius))
            P += len(peers)
        assert P > 1e6
    assert all(b == 0 for b, _ in bad), bad


def test_hub_g8_irregular_keys():
    """Keys without a packed form (NaN-free huge / infinite coordinates, world ids >= 2^24 - 1, raw
    off-grid keys) across eight shards, by position and by raw key."""
    import torch
    from test_gpu_sharded_native import _irregular_workload
    from worldql_server_amd.router import Hub, Router
    w, keys, key_ops = _irregular_workload()
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        lo, hi = _slice(M, rank)
        r.sharded_apply_ops(w.ops)
        r.sharded_apply_ops(key_ops)
        args = (w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], dev)
        results[rank] = (_tick(r, w.pos[lo:hi], *args), _tick(r, w.pos[lo:hi], *args, keys=keys[lo:hi]))

    _run_shards(body)
    for r in routers:
        r.close()
    hub.close()
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    o.apply_ops(key_ops)
    total = 0
    for rank in range(G):
        lo, hi = _slice(M, rank)
        by_pos, by_key = results[rank]
        wo_, wp_, _ = o.route(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])
        assert (by_pos[1] == wo_).all() and (by_pos[2] == wp_).all(), rank
        wo_, wp_, _ = o.route(None, w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], keys=keys[lo:hi])
        assert (by_key[1] == wo_).all() and (by_key[2] == wp_).all(), rank
        total += len(by_key[2])
    assert total > 0


class _DevWords:
    """32-bit words at a device address, for torch.as_tensor (__cuda_array_interface__)."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i4", "data": (ptr, False), "version": 3}


def _view_arrays(v):
    import torch

    def get(ptr, cnt):
        if cnt == 0:
            return np.empty(0, np.uint32)
        return torch.as_tensor(_DevWords(ptr, cnt), device="cuda:0").cpu().numpy().view(np.uint32)
    return get(v.offsets, int(v.n_msgs) + 1), get(v.peers, int(v.n_pairs))


@pytest.mark.parametrize("mode", ["cube", "replicate"])
def test_multi_g8_slices_c3_route_check(mode):
    """One handle over eight devices (all cuda:0 here), the scaling form: each device routes its
    eighth of a C3-shaped tick (1M messages) and keeps its CSR; every slice against the oracle."""
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router
    w = synth_ext.config_c3(scale=0.1)
    churn = _c3_churn(w, seed=43)
    M = len(w.world)
    dev = torch.device("cuda:0")
    r = Router.multi(16, [0] * G, mode=mode)
    assert r.n_gpus() == G
    r.apply_ops(w.ops)
    r.apply_ops(churn)
    r.set_fanout_hint(40.0)
    sl = []
    for g in range(G):
        lo, hi = _slice(M, g)
        sl.append((lo, hi, (torch.from_numpy(np.ascontiguousarray(w.pos[lo:hi])).to(dev),
                            torch.from_numpy(np.ascontiguousarray(w.world[lo:hi]).view(np.int32)).to(dev),
                            torch.from_numpy(np.ascontiguousarray(w.sender[lo:hi]).view(np.int32)).to(dev),
                            torch.from_numpy(np.ascontiguousarray(w.repl[lo:hi])).to(dev))))
    torch.cuda.synchronize()
    got = None
    for _ in range(2):  # the second reuses the staging
        views = r.route_slices_device([(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), hi - lo)
                                       for lo, hi, t in sl])
        got = [_view_arrays(v) for v in views]
    assert r.route_health() == (0, 0)
    n_entries = r.stats()["n_entries"]
    r.close()
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    o.apply_ops(churn)
    assert n_entries == o.counts()[0]
    P = 0
    for (lo, hi, _), (offs, peers) in zip(sl, got):
        bad, first = o.route_check(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], offs, peers)
        assert bad == 0, f"slice [{lo}, {hi}): {bad} messages differ, first {first}"
        P += len(peers)
    assert P > 2e7
