"""Asynchronous sharded ticks back to back (wq_sharded_route_tick_async,
wq_sharded_route_owner_slots_async; csrc/wq_sharded.hip), G = 8 hub shards on cuda:0.

The reference owns the table in one task and handles every event in order (thread.rs:113-148): every
tick's result must arrive, in order, and be the one table's. The asynchronous forms end a tick without
a host read: its small vectors go to a pinned snapshot ring that later calls fold in (budgets from the
tick two calls back). Here 64+ ticks are enqueued back to back with no synchronisation between them, a
tick with twice the messages outgrows its budgets (error bit 64 on every shard), a 7-message tick
shrinks them, and every other tick is checked against the whole-table oracle: the slot form's CSR
per tick (each tick writes its own output buffers), the owner form's P per tick summed over the
owners and its last view mapped back to every source.

Local failures: a shard whose step fails on a budgeted asynchronous tick must queue its
snapshot like its peers, or the shards fold different ticks and size their next exchanges
differently (a hang over RCCL, 'sizes disagree' over the hub). Failures at step 1 and 3 on one shard,
then more asynchronous ticks, checked against the oracle.
"""
import threading

import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth

pytestmark = pytest.mark.gpu

N_TICKS = 72


def _workload(seed=41, n_peers=3000, n_msgs=24000):
    return synth.uniform_box(seed, n_peers, n_msgs, 96.0, neighbourhood=True, repl_mode="mixed", n_worlds=3)


def _slice(M, G, rank):
    return rank * M // G, (rank + 1) * M // G


def _run(G, body, timeout=300):
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
    assert not any(t.is_alive() for t in th), "a shard never finished (a lost asynchronous result?)"
    assert not errors, errors


# the tick schedule: message set per tick ("full" slice, "half", "dbl" = the slice twice, "tiny" = 7)
def _schedule():
    kinds = ["full"] * N_TICKS
    kinds[10] = kinds[11] = "half"
    kinds[40] = "dbl"          # outgrows its budgets: bit 64, not valid
    kinds[50] = "tiny"
    kinds[60] = "half"
    return kinds


def _arrays(w, lo, hi, kind):
    sl = [x[lo:hi] for x in (w.pos, w.world, w.sender, w.repl)]
    if kind == "half":
        sl = [x[:len(x) // 2] for x in sl]
    elif kind == "dbl":
        sl = [np.concatenate([x, x]) for x in sl]
    elif kind == "tiny":
        sl = [x[:7] for x in sl]
    return [np.ascontiguousarray(x) for x in sl]


def _oracle(w):
    o = orc.COracle(w.cube_size)
    o.apply_ops(w.ops)
    return o


def test_hub_g8_slot_ticks_back_to_back():
    """72 wq_sharded_route_tick_async calls per shard with no wait between them: every tick not
    flagged 64 is the oracle's CSR, the doubled tick is flagged on every shard, and flags only appear
    where a tick outgrew the one two calls back."""
    import torch
    from worldql_server_amd.router import Hub, Router
    G = 8
    w = _workload()
    M = len(w.world)
    dev = torch.device("cuda:0")
    kinds = _schedule()
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.sharded_apply_ops(w.ops)
        lo, hi = _slice(M, G, rank)
        ins = {}
        for k in set(kinds):
            a = _arrays(w, lo, hi, k)
            ins[k] = [torch.from_numpy(a[0]).to(dev), torch.from_numpy(a[1].view(np.int32)).to(dev),
                      torch.from_numpy(a[2].view(np.int32)).to(dev), torch.from_numpy(a[3]).to(dev)]
        outs = []
        for k in kinds:
            m = len(ins[k][1])
            cap = 64 * m + 64
            outs.append((torch.empty(m + 1, dtype=torch.int32, device=dev),
                         torch.empty(cap, dtype=torch.int32, device=dev),
                         torch.empty(cap, dtype=torch.int32, device=dev), cap))
        cnt = torch.full((N_TICKS * 24,), 0xEE, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        for t, k in enumerate(kinds):
            a = ins[k]
            o, p, q, cap = outs[t]
            r.sharded_route_async(a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr(), a[3].data_ptr(), len(a[1]),
                                  o.data_ptr(), p.data_ptr(), q.data_ptr(), cap, cnt.data_ptr() + 24 * t)
        torch.cuda.synchronize(dev)
        c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE).copy()
        host = [(o.cpu().numpy().view(np.uint32), p.cpu().numpy().view(np.uint32), q.cpu().numpy().view(np.uint32))
                for o, p, q, _ in outs]
        results[rank] = (c, host, r.shard_tick_stats(), r.route_health())

    _run(G, body)
    o = _oracle(w)
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        want = {k: o.route(*_arrays(w, lo, hi, k))[:2] for k in set(kinds)}
        c, host, stats, health = results[rank]
        sizes = [len(_arrays(w, lo, hi, k)[1]) for k in kinds]
        flagged = []
        for t, k in enumerate(kinds):
            err = int(c[t]["error"])
            if err & 64:
                flagged.append(t)
                # a budget can only be short when this tick outgrew the one two calls back
                assert t >= 2 and sizes[t] > sizes[t - 2], (rank, t, k, sizes[t - 2:t + 1])
                continue
            assert err == 0 and int(c[t]["overflow"]) == 0, (rank, t, k, c[t])
            offs, peers, msgs = host[t]
            w_offs, w_peers = want[k]
            P = int(c[t]["n_pairs"])
            assert P == len(w_peers), (rank, t, k, P, len(w_peers))
            assert (offs == w_offs).all(), (rank, t, k)
            assert (peers[:P] == w_peers).all(), (rank, t, k)
            assert (msgs[:P] == np.repeat(np.arange(len(w_offs) - 1, dtype=np.uint32), np.diff(w_offs))).all()
        assert 40 in flagged, (rank, flagged)
        assert len(flagged) <= 6, (rank, flagged)
        assert stats[1] >= N_TICKS - 10, stats        # nearly every tick ran on budgets
        assert health[0] & 64
    for r in routers:
        r.close()
    hub.close()


def test_hub_g8_owner_slot_ticks_back_to_back():
    """72 wq_sharded_route_owner_slots_async calls per shard with no wait between them: per tick the
    owners' P summed over the shards equals the oracle's pairs over every source's messages (ticks
    not flagged 64), and the last tick's views map back to every source's messages exactly."""
    import ctypes

    import torch
    from worldql_server_amd.router import Hub, Router
    G = 8
    w = _workload(seed=43)
    M = len(w.world)
    dev = torch.device("cuda:0")
    kinds = _schedule()
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    barrier = threading.Barrier(G)

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.sharded_apply_ops(w.ops)
        lo, hi = _slice(M, G, rank)
        ins = {}
        for k in set(kinds):
            a = _arrays(w, lo, hi, k)
            ins[k] = [torch.from_numpy(a[0]).to(dev), torch.from_numpy(a[1].view(np.int32)).to(dev),
                      torch.from_numpy(a[2].view(np.int32)).to(dev), torch.from_numpy(a[3]).to(dev)]
        cnt = torch.full((N_TICKS * 24,), 0xEE, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        sync_P = {}
        for t, k in enumerate(kinds):
            a = ins[k]
            v = r.sharded_route_owner_slots_async(a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr(),
                                                  a[3].data_ptr(), len(a[1]), cnt.data_ptr() + 24 * t)
            if int(v.n_pairs) != 2 ** 64 - 1:
                sync_P[t] = int(v.n_pairs)
        torch.cuda.synchronize(dev)
        R = int(v.n_slots)
        send_seg = list(v.send_seg[:G + 1])
        offs = np.empty(R + 1, np.uint32)
        perm = np.empty(max(send_seg[-1], 1), np.uint32)
        assert hip.hipMemcpy(offs.ctypes.data, v.offsets, (R + 1) * 4, 2) == 0
        P = int(offs[-1])
        peers = np.empty(max(P, 1), np.uint32)
        if P:
            assert hip.hipMemcpy(peers.ctypes.data, v.peers, P * 4, 2) == 0
        if send_seg[-1]:
            assert hip.hipMemcpy(perm.ctypes.data, v.send_perm, send_seg[-1] * 4, 2) == 0
        view = dict(offs=offs, peers=peers[:P], perm=perm[:send_seg[-1]], seg=list(v.seg[:G + 1]), send_seg=send_seg)
        c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE).copy()
        barrier.wait()
        results[rank] = (c, view, sync_P, r.shard_tick_stats())

    _run(G, body)
    o = _oracle(w)
    want = {k: [o.route(*_arrays(w, *_slice(M, G, s), k))[:2] for s in range(G)] for k in set(kinds)}
    for t, k in enumerate(kinds):
        flags = [int(results[g][0][t]["error"]) for g in range(G)]
        if any(f & 64 for f in flags):
            assert all(f & 64 for f in flags), (t, flags)     # every shard hears of a short budget
            continue
        assert flags == [0] * G, (t, k, flags)
        assert all(int(results[g][0][t]["overflow"]) == 0 for g in range(G)), t
        got = sum(int(results[g][0][t]["n_pairs"]) for g in range(G))
        assert got == sum(len(want[k][s][1]) for s in range(G)), (t, k)
    assert all(int(results[g][0][40]["error"]) & 64 for g in range(G))
    # the last tick's views: every source's messages routed once, with the oracle's recipients
    views = [res[1] for res in results]
    got = {}
    for ow, v in enumerate(views):
        for s in range(G):
            base = views[s]["send_seg"][ow]
            for j in range(v["seg"][s + 1] - v["seg"][s]):
                i = v["seg"][s] + j
                m = int(views[s]["perm"][base + j])
                if m == 0xFFFFFFFF:
                    assert v["offs"][i + 1] == v["offs"][i]
                    continue
                got[(s, m)] = v["peers"][v["offs"][i]:v["offs"][i + 1]]
    last = kinds[-1]
    for s in range(G):
        w_offs, w_peers = want[last][s]
        for m in range(len(w_offs) - 1):
            assert (got.pop((s, m)) == w_peers[w_offs[m]:w_offs[m + 1]]).all(), (s, m)
    assert not got
    for g in range(G):
        assert results[g][3][1] >= N_TICKS - 10, results[g][3]
    for r in routers:
        r.close()
    hub.close()


@pytest.mark.parametrize("form", ["slots", "owner_slots"])
def test_hub_async_ticks_with_local_failures(form):
    """Asynchronous budgeted ticks with a failure injected on shard 1 at step 1, later at step 3:
    the failing shard returns WQ_E_INVALID and its peers go on (bit 32 where the status reaches them);
    the following asynchronous ticks of every shard are exact (no exchange-size disagreement, no hang)."""
    import torch
    from worldql_server_amd.router import Hub, Router, WQError
    G = 3
    w = _workload(seed=47, n_msgs=9000)
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G
    plan = ["ok"] * 4 + ["f1"] + ["ok"] * 4 + ["f3"] + ["ok"] * 4

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.sharded_apply_ops(w.ops)
        lo, hi = _slice(M, G, rank)
        a = _arrays(w, lo, hi, "full")
        t_in = [torch.from_numpy(a[0]).to(dev), torch.from_numpy(a[1].view(np.int32)).to(dev),
                torch.from_numpy(a[2].view(np.int32)).to(dev), torch.from_numpy(a[3]).to(dev)]
        m = len(a[1])
        cap = 64 * m + 64
        outs = [(torch.empty(m + 1, dtype=torch.int32, device=dev), torch.empty(cap, dtype=torch.int32, device=dev),
                 torch.empty(cap, dtype=torch.int32, device=dev)) for _ in plan]
        cnt = torch.full((len(plan) * 24,), 0xEE, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        codes, owner_P = [], []
        for t, step in enumerate(plan):
            if rank == 1 and step != "ok":
                r.inject_shard_failure(int(step[1]))
            try:
                if form == "slots":
                    o, p, q = outs[t]
                    r.sharded_route_async(t_in[0].data_ptr(), t_in[1].data_ptr(), t_in[2].data_ptr(),
                                          t_in[3].data_ptr(), m, o.data_ptr(), p.data_ptr(), q.data_ptr(), cap,
                                          cnt.data_ptr() + 24 * t)
                else:
                    v = r.sharded_route_owner_slots_async(t_in[0].data_ptr(), t_in[1].data_ptr(), t_in[2].data_ptr(),
                                                          t_in[3].data_ptr(), m, cnt.data_ptr() + 24 * t)
                codes.append(None)
            except WQError as e:
                codes.append(e.code)
        torch.cuda.synchronize(dev)
        c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE).copy()
        host = [tuple(x.cpu().numpy().view(np.uint32) for x in oo) for oo in outs]
        results[rank] = (codes, c, host, r.route_health())

    _run(G, body)
    o = _oracle(w)
    want = [o.route(*_arrays(w, *_slice(M, G, s), "full"))[:2] for s in range(G)]
    total = sum(len(x[1]) for x in want)
    for t, step in enumerate(plan):
        codes = [results[g][0][t] for g in range(G)]
        if step == "ok":
            assert codes == [None] * G, (t, codes)
        else:
            assert codes[1] == abi.WQ_E_INVALID and codes[0] is None and codes[2] is None, (t, step, codes)
            if step == "f1" or form == "slots":  # the failing shard's status reached every peer
                for g in (0, 2):
                    assert int(results[g][1][t]["error"]) & 32, (t, g, results[g][1][t])
            continue
        errs = [int(results[g][1][t]["error"]) for g in range(G)]
        assert errs == [0] * G, (t, errs)
        if form == "slots":
            for g in range(G):
                offs, peers, msgs = results[g][2][t]
                P = int(results[g][1][t]["n_pairs"])
                assert P == len(want[g][1]) and (offs == want[g][0]).all() and (peers[:P] == want[g][1]).all(), (t, g)
        else:
            assert sum(int(results[g][1][t]["n_pairs"]) for g in range(G)) == total, t
    for r in routers:
        r.close()
    hub.close()
