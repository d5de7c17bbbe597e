"""The multi-GPU tick behind the C ABI (wq_sharded_route_tick_device, csrc/wq_sharded.hip) against
the oracle holding the WHOLE table (sharding must not change any result).

Both return forms: "slots" (default — 20-byte slots out, row references plus one pool of cube lists
per destination back) and "expanded" (40-byte records out, expanded pairs back; the radius
filter's form, forced here with wq_debug_set_shard_form).

Exchanges exercised:
  hub       G in {1, 2, 3, 5} router handles as threads of this process, all on cuda:0;
  callback  2 processes on cuda:0 whose exchange is a gloo all-to-all (the C path with the
            caller's own transport);
  RCCL      1 rank (the self segment), and 2 processes on one GPU where RCCL allows it.
Every shard is given the same op stream (churn and REMOVE_PEER included) and its own slice of the
messages; each slice's recipients must equal the oracle's, per message, in message order.
"""
import ctypes
import os
import socket
import threading

import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth

pytestmark = pytest.mark.gpu


def _workload(seed=11, n_peers=3000, n_msgs=20000):
    w = synth.uniform_box(9, n_peers, n_msgs, 96.0, neighbourhood=True, repl_mode="mixed", n_worlds=3)
    rng = np.random.default_rng(seed)
    # churn on top: unsubscribe some of the build's ops, then disconnect a few peers
    un = w.ops[rng.choice(len(w.ops), 2000, replace=False)].copy()
    un["kind"] = abi.OP_UNSUBSCRIBE
    rm = abi.ops_array(np.full(40, abi.WORLD_INVALID, np.uint32), rng.choice(n_peers, 40, replace=False),
                       np.full(40, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((40, 3)))
    return w, abi.concat_ops([un, rm])


def _expected(ops_list, w, lo, hi):
    o = orc.COracle(w.cube_size)
    for ops in ops_list:
        o.apply_ops(ops)
    offs, peers, _ = o.route(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])
    return offs, peers


def _slice(M, G, rank):
    return rank * M // G, (rank + 1) * M // G


def _tick(r, w, lo, hi, dev, cap=None, keys=None):
    """One sharded tick of messages [lo, hi) on router r; returns (rc, offsets, peers, msgs).
    keys (M x 3 int64, optional): raw CubeArea keys instead of the positions."""
    import torch
    M = hi - lo
    pos = torch.from_numpy(np.ascontiguousarray(w.pos[lo:hi])).to(dev)
    kt = None if keys is None else torch.from_numpy(np.ascontiguousarray(keys[lo:hi])).to(dev)
    wo = torch.from_numpy(np.ascontiguousarray(w.world[lo:hi]).view(np.int32)).to(dev)
    se = torch.from_numpy(np.ascontiguousarray(w.sender[lo:hi]).view(np.int32)).to(dev)
    rp = torch.from_numpy(np.ascontiguousarray(w.repl[lo:hi])).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 64 * M + 64 if cap is None else cap
    peers = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    msgs = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    rc, P = r.sharded_route_device(None if kt is not None else pos.data_ptr(), wo.data_ptr(), se.data_ptr(),
                                   rp.data_ptr(), M, offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap,
                                   keys_ptr=None if kt is None else kt.data_ptr())
    if rc == abi.WQ_E_CAPACITY:
        peers = torch.empty(P, dtype=torch.int32, device=dev)
        msgs = torch.empty(P, dtype=torch.int32, device=dev)
        r.sharded_copy_out(offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), P)
    torch.cuda.synchronize(dev)
    o = offs.cpu().numpy().view(np.uint32)
    return rc, o, peers.cpu().numpy().view(np.uint32)[:P], msgs.cpu().numpy().view(np.uint32)[:P]


def _check(got, want, M):
    rc, offs, peers, msgs = got
    w_offs, w_peers = want
    assert (offs == w_offs).all()
    assert (peers == w_peers).all()  # ascending per message on both sides
    assert (msgs == np.repeat(np.arange(M, dtype=np.uint32), np.diff(offs.astype(np.int64)))).all()


@pytest.mark.parametrize("G,form", [(1, "slots"), (2, "slots"), (3, "slots"), (5, "slots"), (2, "expanded"),
                                    (3, "expanded")])
def test_hub_sharded_ticks_vs_whole_table_oracle(G, form):
    import torch
    from worldql_server_amd.router import Hub, Router
    w, churn = _workload()
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            r.set_shard_form(form == "expanded")
            assert r.shard_info() == (G, rank)
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            first = _tick(r, w, lo, hi, dev, cap=7)  # too small: WQ_E_CAPACITY, then copy_out
            r.sharded_apply_ops(churn)
            second = _tick(r, w, lo, hi, dev)
            empty = _tick(r, w, lo, lo, dev)  # a shard with no messages still takes part
            results[rank] = (first, second, empty, r.stats()["n_entries"])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    assert sum(res[3] for res in results) > 0
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        first, second, empty, _ = results[rank]
        assert first[0] == (abi.WQ_E_CAPACITY if len(first[2]) > 7 else 0)
        _check(first, _expected([w.ops], w, lo, hi), hi - lo)
        _check(second, _expected([w.ops, churn], w, lo, hi), hi - lo)
        assert empty[1].tolist() == [0] and len(empty[2]) == 0
    o.apply_ops(churn)
    assert sum(res[3] for res in results) == o.counts()[0]  # the shards partition the table
    for r in routers:
        r.close()
    hub.close()


@pytest.mark.parametrize("n_peers", [40, 600])
def test_hub_hot_cubes_vs_whole_table_oracle(n_peers):
    """Every message in a few dozen (world, cube) buckets: a block of the owner's received slots holds
    the same (source, cube) pair many times over, so the per-block LDS claim table (k_ref_claim)
    deduplicates nearly every slot before the global claims. 40 peers: the rows are inline records;
    600: long lists."""
    import torch
    from worldql_server_amd.router import Hub, Router
    G = 3
    w = synth.uniform_box(13, n_peers, 30000, 20.0, neighbourhood=True, repl_mode="mixed", n_worlds=3)
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            cap = 256 * (hi - lo) + 64  # above the 161 recipients of the busiest message
            results[rank] = (_tick(r, w, lo, hi, dev, cap=cap), _tick(r, w, lo, hi, dev, cap=cap))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        want = _expected([w.ops], w, lo, hi)
        for got in results[rank]:  # the exact first tick, then a budgeted one
            _check(got, want, hi - lo)
    for r in routers:
        r.close()
    hub.close()


@pytest.mark.parametrize("G", [1, 2, 3])
def test_hub_owner_form_vs_whole_table_oracle(G):
    """wq_sharded_route_owner_device: the pairs stay on their owner; across the shards every message of
    every ingesting slice appears exactly once, with the oracle's recipients."""
    import torch
    from worldql_server_amd.router import Hub, Router
    w, churn = _workload(seed=13)
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            r.sharded_apply_ops(churn)
            n = hi - lo
            pos = torch.from_numpy(np.ascontiguousarray(w.pos[lo:hi])).to(dev)
            wo = torch.from_numpy(np.ascontiguousarray(w.world[lo:hi]).view(np.int32)).to(dev)
            se = torch.from_numpy(np.ascontiguousarray(w.sender[lo:hi]).view(np.int32)).to(dev)
            rp = torch.from_numpy(np.ascontiguousarray(w.repl[lo:hi])).to(dev)
            torch.cuda.synchronize(dev)
            v = r.sharded_route_owner_device(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), n)
            R, P = int(v.n_recs), int(v.n_pairs)
            hip = ctypes.CDLL("libamdhip64.so.7")
            hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            recs = np.empty(max(R, 1), abi.MSG_REC_DTYPE)
            offs = np.empty(R + 1, np.uint32)
            peers = np.empty(max(P, 1), np.uint32)
            torch.cuda.synchronize(dev)
            if R:
                assert hip.hipMemcpy(recs.ctypes.data, v.recs, R * 40, 2) == 0
                assert hip.hipMemcpy(peers.ctypes.data, v.peers, P * 4, 2) == 0 or P == 0
            assert hip.hipMemcpy(offs.ctypes.data, v.offsets, (R + 1) * 4, 2) == 0
            results[rank] = (recs[:R], offs, peers[:P], list(v.seg[:G + 1]))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    got = {}
    for rank in range(G):
        recs, offs, peers, seg = results[rank]
        assert offs[0] == 0 and offs[-1] == len(peers) and seg[-1] == len(recs)
        for src in range(G):
            for i in range(seg[src], seg[src + 1]):
                key = (src, int(recs[i]["msg"]))
                assert key not in got  # each message is routed by exactly one owner
                got[key] = peers[offs[i]:offs[i + 1]]
    for src in range(G):
        lo, hi = _slice(M, G, src)
        w_offs, w_peers = _expected([w.ops, churn], w, lo, hi)
        for m in range(hi - lo):
            want = w_peers[w_offs[m]:w_offs[m + 1]]
            assert (got.pop((src, m)) == want).all(), (src, m)
    assert not got
    for r in routers:
        r.close()
    hub.close()


def _owner_slot_tick(r, pos, world, sender, repl, dev, keys=None):
    """One wq_sharded_route_owner_slots tick of the given host arrays; the view copied to the host."""
    import torch
    t = [torch.from_numpy(np.ascontiguousarray(x)).to(dev)
         for x in (pos, world.view(np.int32), sender.view(np.int32), repl)]
    kt = None if keys is None else torch.from_numpy(np.ascontiguousarray(keys)).to(dev)
    torch.cuda.synchronize(dev)
    v = r.sharded_route_owner_slots(None if kt is not None else t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
                                    t[3].data_ptr(), len(world), keys_ptr=None if kt is None else kt.data_ptr())
    R, P = int(v.n_slots), int(v.n_pairs)
    G = r.shard_info()[0]
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    send_seg = list(v.send_seg[:G + 1])
    offs = np.empty(R + 1, np.uint32)
    peers = np.empty(max(P, 1), np.uint32)
    perm = np.empty(max(send_seg[-1], 1), np.uint32)
    torch.cuda.synchronize(dev)
    assert hip.hipMemcpy(offs.ctypes.data, v.offsets, (R + 1) * 4, 2) == 0
    if P:
        assert hip.hipMemcpy(peers.ctypes.data, v.peers, P * 4, 2) == 0
    if send_seg[-1]:
        assert hip.hipMemcpy(perm.ctypes.data, v.send_perm, send_seg[-1] * 4, 2) == 0
    return dict(offs=offs, peers=peers[:P], perm=perm[:send_seg[-1]], seg=list(v.seg[:G + 1]),
                send_seg=send_seg)


def _check_owner_slots(views, want):
    """views[o]: owner o's tick; want[s]: (offsets, peers) the whole-table oracle gives for source
    s's messages. Every message of every source must be routed by exactly one owner, with the
    oracle's recipients; padding and second slots route to nobody."""
    G = len(views)
    got = {}
    for o, v in enumerate(views):
        offs, peers = v["offs"], v["peers"]
        assert offs[0] == 0 and offs[-1] == len(peers) and v["seg"][-1] == len(offs) - 1
        assert (np.diff(offs.astype(np.int64)) >= 0).all()
        for s in range(G):
            base = views[s]["send_seg"][o]
            assert v["seg"][s + 1] - v["seg"][s] == views[s]["send_seg"][o + 1] - base  # the budgets agree
            for k in range(v["seg"][s + 1] - v["seg"][s]):
                i = v["seg"][s] + k
                m = int(views[s]["perm"][base + k])
                if m == 0xFFFFFFFF:
                    assert offs[i + 1] == offs[i], (o, s, k)
                    continue
                assert (s, m) not in got
                got[(s, m)] = peers[offs[i]:offs[i + 1]]
    for s in range(G):
        w_offs, w_peers = want[s]
        for m in range(len(w_offs) - 1):
            assert (got.pop((s, m)) == w_peers[w_offs[m]:w_offs[m + 1]]).all(), (s, m)
    assert not got


@pytest.mark.parametrize("G", [1, 2, 3, 8])
def test_hub_owner_slots_vs_whole_table_oracle(G):
    """wq_sharded_route_owner_slots, the owner form on budgeted slots: an exact first tick, a budgeted
    one after churn, one with four times the messages (budgets short: every shard redoes it
    exactly), a budgeted one again, a slot tick in between (its budgets leave out the self segment,
    so the next owner tick runs exact) — every message routed once, against the whole-table oracle."""
    import torch
    from worldql_server_amd.router import Hub, Router
    w, churn = _workload(seed=17)
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []
    barrier = threading.Barrier(G)

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            lo, hi = _slice(M, G, rank)
            sl = (w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])
            dbl = tuple(np.concatenate([x] * 4) for x in sl)
            r.sharded_apply_ops(w.ops)
            t1 = _owner_slot_tick(r, *sl, dev)
            r.sharded_apply_ops(churn)
            t2 = _owner_slot_tick(r, *sl, dev)
            st2 = r.shard_tick_stats()
            t3 = _owner_slot_tick(r, *dbl, dev)
            st3 = r.shard_tick_stats()
            t4 = _owner_slot_tick(r, *sl, dev)
            slot = _tick(r, w, lo, hi, dev)
            t5 = _owner_slot_tick(r, *sl, dev)
            st5 = r.shard_tick_stats()
            barrier.wait()
            results[rank] = (t1, t2, t3, t4, slot, t5, st2, st3, st5)
        except Exception as e:  # noqa: BLE001
            errors.append(e)
            barrier.abort()

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    want1 = [_expected([w.ops], w, *_slice(M, G, s)) for s in range(G)]
    want2 = [_expected([w.ops, churn], w, *_slice(M, G, s)) for s in range(G)]
    want_dbl = []
    for s in range(G):
        lo, hi = _slice(M, G, s)
        o = orc.COracle(w.cube_size)
        o.apply_ops(w.ops)
        o.apply_ops(churn)
        dbl = [np.concatenate([x[lo:hi]] * 4) for x in (w.pos, w.world, w.sender, w.repl)]
        want_dbl.append(o.route(*dbl)[:2])
    _check_owner_slots([res[0] for res in results], want1)
    for k, want in ((1, want2), (2, want_dbl), (3, want2), (5, want2)):
        _check_owner_slots([res[k] for res in results], want)
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        _check(results[rank][4], want2[rank], hi - lo)
        st2, st3, st5 = results[rank][6:]
        if G > 1:
            assert st2[1] >= 1            # the second owner tick ran on budgets
            assert st3[0] == st2[0] + 1   # four times the messages: short budgets, redone exactly
        assert st5[0] > st3[0]            # after the slot tick: exact again
    for r in routers:
        r.close()
    hub.close()


def _view_to_host(r, v, G):
    """An owner-slot view (its tick finished) copied to the host, as _owner_slot_tick returns it."""
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
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
    return dict(offs=offs, peers=peers[:P], perm=perm[:send_seg[-1]], seg=list(v.seg[:G + 1]), send_seg=send_seg)


@pytest.mark.parametrize("G", [1, 2, 3])
def test_hub_owner_slots_async_vs_whole_table_oracle(G):
    """wq_sharded_route_owner_slots_async: the first call runs exact (synchronously, n_pairs filled),
    the next ones return at once with P in the caller's counters; the last tick's view against the
    whole-table oracle; four times the messages on budgets: error bit 64 on every shard (outputs not
    valid); a synchronous call after it folds that tick in, redoes itself exactly and is right."""
    import torch
    from worldql_server_amd.router import Hub, Router
    w, churn = _workload(seed=23)
    M = len(w.world)
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []
    counters_dtype = abi.COUNTERS_DTYPE

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            r.sharded_apply_ops(churn)
            arr = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
                   (w.pos[lo:hi], w.world[lo:hi].view(np.int32), w.sender[lo:hi].view(np.int32), w.repl[lo:hi])]
            quad = [torch.cat([x] * 4) for x in arr]
            cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)

            def tick(a):
                return r.sharded_route_owner_slots_async(a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr(),
                                                         a[3].data_ptr(), len(a[1]), cnt.data_ptr())
            first = tick(arr)
            n_first = int(first.n_pairs)
            for _ in range(3):
                v = tick(arr)
            torch.cuda.synchronize(dev)
            c_last = cnt.cpu().numpy().view(counters_dtype)[0].copy()
            view_last = _view_to_host(r, v, G)
            r.route_health()  # clear
            vq = tick(quad)   # budgets short everywhere
            torch.cuda.synchronize(dev)
            c_quad = cnt.cpu().numpy().view(counters_dtype)[0].copy()
            sync_quad = int(vq.n_pairs) != 2 ** 64 - 1
            health = r.route_health()
            # synchronous: folds the flagged tick in and redoes itself exactly
            after = r.sharded_route_owner_slots(quad[0].data_ptr(), quad[1].data_ptr(), quad[2].data_ptr(),
                                                quad[3].data_ptr(), len(quad[1]))
            torch.cuda.synchronize(dev)
            results[rank] = (n_first, c_last, view_last, c_quad, sync_quad, health, int(after.n_pairs),
                             _view_to_host(r, after, G), r.shard_tick_stats())
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    want = [_expected([w.ops, churn], w, *_slice(M, G, s)) for s in range(G)]
    _check_owner_slots([res[2] for res in results], want)
    want_quad = []
    for s in range(G):
        lo, hi = _slice(M, G, s)
        o = orc.COracle(w.cube_size)
        o.apply_ops(w.ops)
        o.apply_ops(churn)
        want_quad.append(o.route(*[np.concatenate([x[lo:hi]] * 4) for x in (w.pos, w.world, w.sender, w.repl)])[:2])
    _check_owner_slots([res[7] for res in results], want_quad)
    for rank in range(G):
        n_first, c_last, view_last, c_quad, sync_quad, health, n_after, _, stats = results[rank]
        assert n_first != 2 ** 64 - 1                      # the first tick ran exact
        assert c_last["error"] == 0 and c_last["overflow"] == 0
        assert int(c_last["n_pairs"]) == int(view_last["offs"][-1])
        assert not sync_quad and (int(c_quad["error"]) & 64)  # the short budgets, seen on every shard
        assert health[0] & 64
        assert n_after == int(results[rank][7]["offs"][-1])
        assert stats[1] >= 3                               # asynchronous ticks ran on budgets
    for r in routers:
        r.close()
    hub.close()


def test_hub_owner_slots_irregular_keys_and_failure():
    """Keys without a packed form (two slots: the second routes to nobody) by position and by raw
    key, then local failures on one shard: before the exchange (step 1) every shard returns the
    error, since it travels in the A vectors; after it (step 3: the owner's own routing) only that
    shard does, the others' pairs are complete. The tick after each is right."""
    import torch
    from worldql_server_amd.router import Hub, Router, WQError
    w, keys, key_ops = _irregular_workload()
    M, G = len(w.world), 3
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            lo, hi = _slice(M, G, rank)
            sl = (w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])
            r.sharded_apply_ops(w.ops)
            r.sharded_apply_ops(key_ops)
            by_pos = _owner_slot_tick(r, *sl, dev)
            by_key = _owner_slot_tick(r, *sl, dev, keys=keys[lo:hi])
            codes, after = [], []
            for step in (1, 3):
                if rank == 1:
                    r.inject_shard_failure(step)
                try:
                    _owner_slot_tick(r, *sl, dev)
                    codes.append(None)
                except WQError as e:
                    codes.append(e.code)
                after.append(_owner_slot_tick(r, *sl, dev))
            results[rank] = (by_pos, by_key, codes, after)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    o.apply_ops(key_ops)
    want_pos, want_key = [], []
    for s in range(G):
        lo, hi = _slice(M, G, s)
        want_pos.append(o.route(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])[:2])
        want_key.append(o.route(None, w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], keys=keys[lo:hi])[:2])
    _check_owner_slots([res[0] for res in results], want_pos)
    _check_owner_slots([res[1] for res in results], want_key)
    assert [res[2][0] for res in results] == [abi.WQ_E_INVALID] * G
    assert [res[2][1] for res in results] == [None, abi.WQ_E_INVALID, None]
    for k in range(2):
        _check_owner_slots([res[3][k] for res in results], want_pos)
    for r in routers:
        r.close()
    hub.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_exchange(dist):
    """The caller's all-to-all for wq_shard_attach_exchange: device -> host, gloo, host -> device."""
    hip = ctypes.CDLL("libamdhip64.so.7")  # the HIP runtime PyTorch already loaded
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    import torch

    def fn(send, sb, recv, rb, stream):
        assert hip.hipStreamSynchronize(stream or None) == 0
        src = np.empty(max(sum(sb), 1), np.uint8)
        if sum(sb):
            assert hip.hipMemcpy(src.ctypes.data, send, sum(sb), 4) == 0
        dst = torch.empty(sum(rb), dtype=torch.uint8)
        dist.all_to_all_single(dst, torch.from_numpy(src[:sum(sb)]), list(rb), list(sb))
        if sum(rb):
            assert hip.hipMemcpy(recv, dst.numpy().ctypes.data, sum(rb), 4) == 0
    return fn


def _proc(rank, G, port, mode, out):
    import torch
    import torch.distributed as dist
    from worldql_server_amd.router import Router, WQError, rccl_unique_id
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    try:
        w, churn = _workload(seed=5)
        M = len(w.world)
        dev = torch.device("cuda:0")
        r = Router(16, 0)
        if mode == "callback":
            r.attach_exchange(G, rank, _gloo_exchange(dist))
        else:
            uid = [rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            try:
                r.attach_rccl(G, rank, uid[0])
            except WQError as e:
                out[rank] = ("rccl-attach", str(e))
                return
        lo, hi = _slice(M, G, rank)
        r.sharded_apply_ops(w.ops)
        r.sharded_apply_ops(churn)
        rc, offs, peers, msgs = _tick(r, w, lo, hi, dev)
        want = _expected([w.ops, churn], w, lo, hi)
        ok = bool((offs == want[0]).all() and (peers == want[1]).all())
        if mode == "callback":  # the owner form too (its self segment goes through the callback)
            sl = (w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])
            _owner_slot_tick(r, *sl, dev)       # exact
            v = _owner_slot_tick(r, *sl, dev)   # on budgets
            views = [None] * G
            dist.all_gather_object(views, v)
            if rank == 0:
                _check_owner_slots(views, [_expected([w.ops, churn], w, *_slice(M, G, q)) for q in range(G)])
        out[rank] = ("ok" if ok else "mismatch", int(len(peers)))
        r.close()
    except Exception as e:  # noqa: BLE001
        out[rank] = ("error", repr(e))
    finally:
        dist.destroy_process_group()


def _run_procs(G, mode):
    import torch.multiprocessing as mp
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_proc, args=(G, port, mode, out), nprocs=G, join=True)
    return dict(out)


@pytest.mark.parametrize("G", [2, 3])
def test_callback_exchange_gloo_processes(G):
    """The native slot tick, then the owner-slot tick, across G processes (one per shard, all on
    cuda:0) whose exchange is the caller's own gloo all-to-all (wq_shard_attach_exchange) — the
    multi-process form of the product path, as one process per GPU runs it."""
    res = _run_procs(G, "callback")
    assert [res[k][0] for k in range(G)] == ["ok"] * G, res
    assert sum(res[k][1] for k in range(G)) > 0


def test_rccl_exchange_one_rank():
    import torch
    from worldql_server_amd.router import Router, rccl_unique_id
    w, churn = _workload(seed=3)
    M = len(w.world)
    r = Router(16, 0)
    r.attach_rccl(1, 0, rccl_unique_id())
    r.sharded_apply_ops(w.ops)
    r.sharded_apply_ops(churn)
    dev = torch.device("cuda:0")
    want = _expected([w.ops, churn], w, 0, M)
    _check(_tick(r, w, 0, M, dev), want, M)
    # the owner form over RCCL: its self segment written in place (no self copy), exact then budgeted
    sl = (w.pos, w.world, w.sender, w.repl)
    for _ in range(2):
        _check_owner_slots([_owner_slot_tick(r, *sl, dev)], [want])
    r.detach_shard()
    r.close()


@pytest.mark.skipif(os.environ.get("WQ_TEST_RCCL_MULTI") != "1",
                    reason="two RCCL ranks on ONE GPU: run on request (WQ_TEST_RCCL_MULTI=1) under an outer timeout; on the "
                           "MI355X pool RCCL refuses it (ncclCommInitRank: invalid usage, "
                           "profiles/r03_rccl_two_ranks_one_gpu.log), so multi-rank RCCL needs a multi-GPU node")
def test_rccl_exchange_two_processes_one_gpu():
    res = _run_procs(2, "rccl")
    if any(v[0] == "rccl-attach" for v in res.values()):
        pytest.skip(f"RCCL refuses two ranks on one GPU here: {res}")
    assert [res[k][0] for k in range(2)] == ["ok", "ok"], res


def _irregular_workload():
    """Regular traffic plus messages and subscriptions whose cubes have no packed key (the two-slot
    form on the wire): coordinates beyond +-2^23 cubes, +-inf, a world id >= 2^24 - 1, and raw
    off-grid CubeArea keys. Returns (workload, keys[M x 3] for the same messages, the key ops)."""
    base = synth.uniform_box(21, 1500, 6000, 64.0, neighbourhood=True, repl_mode="mixed", n_worlds=2)
    rng = np.random.default_rng(21)
    n = 240
    huge = rng.uniform(-48, 48, (n, 3)) + np.array([3e12, -5e11, 1e10])
    inf = np.tile(np.array([[np.inf, 1.0, -np.inf]]), (n, 1))
    normal = rng.uniform(-48, 48, (n, 3))
    wide_world = 0xFFFFFFF0
    sub_peers = rng.integers(0, 1500, 3 * n).astype(np.uint32)
    ops = abi.concat_ops([
        base.ops,
        abi.ops_array(np.zeros(n, np.uint32), sub_peers[:n], np.zeros(n, np.uint8), pos=huge),
        abi.ops_array(np.ones(n, np.uint32), sub_peers[n:2 * n], np.zeros(n, np.uint8), pos=inf),
        abi.ops_array(np.full(n, wide_world, np.uint32), sub_peers[2 * n:], np.zeros(n, np.uint8), pos=normal),
    ])
    m_pos = np.concatenate([base.pos, huge[rng.permutation(n)], inf, normal[rng.permutation(n)]])
    m_world = np.concatenate([base.world, np.zeros(n, np.uint32), np.ones(n, np.uint32),
                              np.full(n, wide_world, np.uint32)])
    M = len(m_world)
    perm = rng.permutation(M)  # irregular messages spread over every slot group
    w = synth.Workload("irregular", 16, ops, np.ascontiguousarray(m_pos[perm]), m_world[perm],
                       rng.integers(0, 1500, M).astype(np.uint32), rng.integers(0, 4, M).astype(np.uint8), 1500)
    keys = orc.quantize_np(w.pos, 16).reshape(-1, 3)
    # off-grid raw keys (unreachable from any Vector3): subscribed by key, routed by key
    off = rng.integers(-5, 5, (n, 3)).astype(np.int64) * 16 + 3
    key_ops = abi.ops_array(np.zeros(n, np.uint32), rng.integers(0, 1500, n), np.zeros(n, np.uint8), key=off)
    keys[:n] = off
    return w, keys, key_ops


@pytest.mark.parametrize("form", ["slots", "expanded"])
def test_hub_irregular_keys_vs_whole_table_oracle(form):
    """Keys without a packed form travel as two slots (head + tail); positions and raw keys both."""
    import torch
    from worldql_server_amd.router import Hub, Router
    w, keys, key_ops = _irregular_workload()
    M = len(w.world)
    G = 3
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            r.set_shard_form(form == "expanded")
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            r.sharded_apply_ops(key_ops)
            results[rank] = (_tick(r, w, lo, hi, dev), _tick(r, w, lo, hi, dev, keys=keys))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    o.apply_ops(key_ops)
    total = 0
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        by_pos, by_key = results[rank]
        _check(by_pos, o.route(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])[:2], hi - lo)
        want = o.route(None, w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], keys=keys[lo:hi])[:2]
        _check(by_key, want, hi - lo)
        total += len(by_key[2])
    assert total > 0
    for r in routers:
        r.close()
    hub.close()


@pytest.mark.parametrize("form,step", [("slots", 1), ("slots", 3), ("expanded", 1), ("expanded", 3)])
def test_hub_local_failure_keeps_the_collective(form, step):
    """A shard whose local step fails (test hook) still completes every exchange of the tick: both
    shards return an error instead of one of them waiting on the other, the hub stays usable, and
    the next tick is exact again (no early return between exchanges)."""
    import time

    import torch
    from worldql_server_amd.router import Hub, Router, WQError
    w, churn = _workload(seed=17)
    M = len(w.world)
    G = 2
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            r.set_shard_form(form == "expanded")
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            if rank == 1:
                r.inject_shard_failure(step)
            t0 = time.perf_counter()
            try:
                _tick(r, w, lo, hi, dev)
                first = None
            except WQError as e:
                first = e.code
            dt = time.perf_counter() - t0
            results[rank] = (first, dt, _tick(r, w, lo, hi, dev))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        first, dt, second = results[rank]
        assert first == abi.WQ_E_INVALID, (rank, first)  # every shard of the tick reports it
        assert dt < 60.0                                 # ... without waiting out the hub's timeout
        _check(second, _expected([w.ops], w, lo, hi), hi - lo)
    for r in routers:
        r.close()
    hub.close()


def test_hub_full_c3_two_shards_route_check():
    """The north_star configuration through the sharded tick: full C3 (1M peers x 27 cubes, 10M
    hotspot messages, P = 4.17e8) as 2 shards of one process on cuda:0, each ingesting half of the
    messages; every message's recipients checked against the whole-table oracle (wqo_route_check),
    and the slot form's traffic between the shards measured (wq_shard_last_bytes)."""
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Hub, Router
    w = synth_ext.config_c3()
    M = len(w.world)
    G = 2
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            r.set_fanout_hint(40.0)
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            got = _tick(r, w, lo, hi, dev, cap=48 * (hi - lo))
            results[rank] = (got[0], got[1], got[2], r.shard_last_bytes())
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not errors, errors
    for r in routers:
        r.close()
    hub.close()
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    P = 0
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        rc, offs, peers, (sent, recvd) = results[rank]
        assert rc == 0 and int(offs[-1]) == len(peers)
        bad, first = o.route_check(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], offs, peers)
        assert bad == 0, f"shard {rank}: {bad} messages differ, first {first}"
        P += len(peers)
        # what crossed: far less than the expanded pairs a remote owner would otherwise return
        assert 0 < sent < 4 * len(peers), (sent, len(peers))
    assert P > 4e8


def _run_shards(G, body, timeout=300):
    errors = []

    def wrap(rank):
        try:
            body(rank)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=wrap, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not errors, errors


def test_hub_budgeted_ticks_grow_and_redo():
    """The slot tick's exchanges are sized by budgets from the previous tick (no read-back before
    them): the first tick runs exact, the next on budgets; a tick with twice the messages outgrows
    them, every shard learns it from the exchanged status words and all redo that tick exactly; the
    results are the whole-table oracle's every time."""
    import torch
    from worldql_server_amd.router import Hub, Router
    w, _ = _workload(seed=23)
    M = len(w.world)
    G = 3
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.sharded_apply_ops(w.ops)
        lo, hi = _slice(M, G, rank)
        half = lo + (hi - lo) // 2
        got = [_tick(r, w, lo, half, dev), _tick(r, w, lo, half, dev), _tick(r, w, lo, hi, dev),
               _tick(r, w, lo, hi, dev), _tick(r, w, lo, lo + 7, dev)]
        results[rank] = (got, r.shard_tick_stats())

    _run_shards(G, body)
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        half = lo + (hi - lo) // 2
        got, (exact, budgeted) = results[rank]
        for g, (a, b) in zip(got, [(lo, half), (lo, half), (lo, hi), (lo, hi), (lo, lo + 7)]):
            _check(g, _expected([w.ops], w, a, b), b - a)
        # tick 1 exact; 2 budgeted; 3 budgeted, outgrown, redone exact; 4 and 5 budgeted
        assert (exact, budgeted) == (2, 4), (exact, budgeted)
    for r in routers:
        r.close()
    hub.close()


def test_hub_segment_exactly_at_its_budget():
    """a (source, owner) segment whose slot count equals its budget exactly — every
    slot fit — must keep its last slot (slot_pad_kernel pads from the count, not from budget - 1).
    Shard 0 ingests messages that shard 1 owns: 512 on the first (exact: budget = whole blocks of the
    count = 512) tick, then 1,024 = slot_budget(512) on a budgeted tick; each checked per message."""
    import torch
    from worldql_server_amd.router import Hub, Router
    G = 2
    rng = np.random.default_rng(47)
    n_peers = 400
    centre = rng.uniform(-40.0, 40.0, (n_peers, 3))
    nb = np.array([[dx, dy, dz] for dx in (-1, 0, 1) for dy in (-1, 0, 1) for dz in (-1, 0, 1)], np.float64)
    sub = (centre[:, None, :] + 16.0 * nb[None]).reshape(-1, 3)
    ops = abi.ops_array(np.zeros(len(sub), np.uint32), np.repeat(np.arange(n_peers, dtype=np.uint32), 27),
                        np.zeros(len(sub), np.uint8), pos=sub)
    cand = rng.uniform(-56.0, 56.0, (20000, 3))
    probe = Router(16, 0)
    owner = probe.shard_ops(abi.ops_array(np.zeros(len(cand), np.uint32), np.zeros(len(cand), np.uint32),
                                          np.zeros(len(cand), np.uint8), pos=cand), G)
    probe.close()
    remote = cand[owner == 1]
    local = cand[owner == 0]
    assert len(remote) >= 1536 + 300 and len(local) >= 100

    def msgs(pos):
        n = len(pos)
        return type("W", (), {"pos": np.ascontiguousarray(pos), "world": np.zeros(n, np.uint32),
                              "sender": rng.integers(0, n_peers, n).astype(np.uint32),
                              "repl": rng.integers(0, 3, n).astype(np.uint8), "cube_size": 16})
    # shard 0: 512 remote (+ own) then 1,024 remote (+ own); shard 1: its own slices
    t0 = [msgs(np.concatenate([remote[:512], local[:100]])), msgs(np.concatenate([local[100:150], remote[512:1536]]))]
    t1 = [msgs(remote[1536:1736]), msgs(remote[1736:1836])]
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.sharded_apply_ops(ops)
        ticks = t0 if rank == 0 else t1
        got = [_tick(r, w, 0, len(w.world), dev) for w in ticks]
        results[rank] = (got, r.shard_tick_stats())

    _run_shards(G, body)
    for rank in range(G):
        got, stats = results[rank]
        # the first tick exact, the second on budgets (a pool that outgrew its budget would redo it
        # exactly, with the slot segment again exactly full)
        assert stats[1] == 1 and stats[0] >= 1, stats
        for g, w in zip(got, t0 if rank == 0 else t1):
            M = len(w.world)
            want = _expected([ops], w, 0, M)
            assert np.diff(want[0].astype(np.int64)).astype(bool).mean() > 0.5  # most messages have recipients
            _check(g, want, M)
    for r in routers:
        r.close()
    hub.close()


def test_copy_out_after_a_table_change_is_refused():
    """a slot tick's own-cube rows point into the table, so wq_sharded_copy_out after any
    change of the table (here an op batch) must refuse instead of mixing old counts with new lists."""
    import torch
    from worldql_server_amd.router import Hub, Router, WQError
    w, churn = _workload(seed=29)
    M = len(w.world)
    G = 2
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    codes = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.sharded_apply_ops(w.ops)
        lo, hi = _slice(M, G, rank)
        n = hi - lo
        pos = torch.from_numpy(np.ascontiguousarray(w.pos[lo:hi])).to(dev)
        wo = torch.from_numpy(np.ascontiguousarray(w.world[lo:hi]).view(np.int32)).to(dev)
        se = torch.from_numpy(np.ascontiguousarray(w.sender[lo:hi]).view(np.int32)).to(dev)
        rp = torch.from_numpy(np.ascontiguousarray(w.repl[lo:hi])).to(dev)
        offs = torch.empty(n + 1, dtype=torch.int32, device=dev)
        small = torch.empty(8, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        rc, P = r.sharded_route_device(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), n,
                                       offs.data_ptr(), small.data_ptr(), None, 8)
        assert rc == abi.WQ_E_CAPACITY and P > 8
        r.sharded_apply_ops(churn)
        big = torch.empty(P, dtype=torch.int32, device=dev)
        try:
            r.sharded_copy_out(offs.data_ptr(), big.data_ptr(), None, P)
            codes[rank] = 0
        except WQError as e:
            codes[rank] = e.code

    _run_shards(G, body)
    assert codes == [abi.WQ_E_INVALID] * G
    for r in routers:
        r.close()
    hub.close()


def _radius_workload(seed=21):
    """Peers around their subscription centres (positions jittered off them), most in a sparse box
    (cube lists of a few peers: rows short enough for a survivor mask) plus a dense cluster (lists
    longer than a record's 24 inline peers: rows re-filtered from the pool), mixed replication."""
    rng = np.random.default_rng(seed)
    sparse = rng.uniform(-200.0, 200.0, (2500, 3))
    dense = rng.normal(0.0, 10.0, (500, 3))
    centre = np.concatenate([sparse, dense])
    n = len(centre)
    nb = np.array([[dx, dy, dz] for dx in (-1, 0, 1) for dy in (-1, 0, 1) for dz in (-1, 0, 1)], np.float64)
    sub = (centre[:, None, :] + 16.0 * nb[None]).reshape(-1, 3)
    ops = abi.ops_array(np.zeros(len(sub), np.uint32), np.repeat(np.arange(n, dtype=np.uint32), 27),
                        np.zeros(len(sub), np.uint8), pos=sub)
    peer_pos = centre + rng.uniform(-6.0, 6.0, centre.shape)
    M = 12000
    src = rng.integers(0, n, M)
    mpos = centre[src] + rng.uniform(-12.0, 12.0, (M, 3))
    sender = rng.integers(0, n, M).astype(np.uint32)
    sender[: M // 3] = src[: M // 3]  # a third sent by a peer subscribed where it speaks
    repl = rng.integers(0, 4, M).astype(np.uint8)  # 3: an unknown code (ExceptSelf)
    un = ops[rng.choice(len(ops), 3000, replace=False)].copy()
    un["kind"] = abi.OP_UNSUBSCRIBE
    return ops, un, peer_pos, mpos, np.zeros(M, np.uint32), sender, repl


@pytest.mark.parametrize("G,form", [(1, "slots"), (2, "slots"), (3, "slots"), (2, "expanded")])
def test_hub_radius_ticks_vs_whole_table_oracle(G, form):
    """The radius filter through the sharded tick (C5 over G GPUs): the slot form filters the pool
    rows on the ingesting GPU (short rows as survivor masks, long ones re-filtered by the emit) and
    its own cubes with count_radius_kernel; both forms against the whole-table oracle, per message."""
    import torch
    from worldql_server_amd.router import Hub, Router
    ops, churn, peer_pos, mpos, world, sender, repl = _radius_workload()
    radius = 14.0
    M = len(world)
    w = type("W", (), {"pos": mpos, "world": world, "sender": sender, "repl": repl, "cube_size": 16})
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            r.set_shard_form(form == "expanded")
            r.set_peer_positions(peer_pos)
            r.set_radius(radius)
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(ops)
            first = _tick(r, w, lo, hi, dev, cap=5)  # too small: WQ_E_CAPACITY, then copy_out
            r.sharded_apply_ops(churn)
            second = _tick(r, w, lo, hi, dev)
            results[rank] = (first, second)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    o = orc.COracle(16)
    o.apply_ops(ops)
    want1 = o.route_radius(mpos, world, sender, repl, peer_pos, radius)[:2]
    o.apply_ops(churn)
    want2 = o.route_radius(mpos, world, sender, repl, peer_pos, radius)[:2]
    lens = np.diff(want1[0].astype(np.int64))
    assert lens.max() > 24 and (lens[lens > 0] <= 24).mean() > 0.3  # both row kinds occur
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        for got, (wo_, wp_) in zip(results[rank], (want1, want2)):
            want = (wo_[lo:hi + 1] - wo_[lo], wp_[wo_[lo]:wo_[hi]])
            _check(got, want, hi - lo)
    for r in routers:
        r.close()
    hub.close()


@pytest.mark.parametrize("form", ["slots", "expanded"])
def test_hub_radius_irregular_keys_vs_whole_table_oracle(form):
    """The radius filter on keys without a packed form (two slots on the wire, slot-table cubes on the
    owner: coordinates beyond +-2^23 cubes, +-inf, a world id >= 2^24 - 1) — and the collective
    error when a shard gives raw keys instead of the positions the filter needs."""
    import torch
    from worldql_server_amd.router import Hub, Router, WQError
    w, keys, key_ops = _irregular_workload()
    M, G, radius = len(w.world), 3, 20.0
    peer_pos = np.random.default_rng(5).uniform(-48.0, 48.0, (1500, 3))
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results, errors = [None] * G, []

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            r.set_shard_form(form == "expanded")
            r.set_peer_positions(peer_pos)
            r.set_radius(radius)
            lo, hi = _slice(M, G, rank)
            r.sharded_apply_ops(w.ops)
            by_pos = _tick(r, w, lo, hi, dev)
            try:  # raw keys, no positions: every shard's tick fails, after the collective
                rc_key = _tick(r, w, lo, hi, dev, keys=keys)[0]
            except WQError as e:
                rc_key = e.code
            results[rank] = (by_pos, rc_key)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    wo_, wp_ = o.route_radius(w.pos, w.world, w.sender, w.repl, peer_pos, radius)[:2]
    total = 0
    for rank in range(G):
        lo, hi = _slice(M, G, rank)
        by_pos, rc_key = results[rank]
        _check(by_pos, (wo_[lo:hi + 1] - wo_[lo], wp_[wo_[lo]:wo_[hi]]), hi - lo)
        total += len(by_pos[2])
        assert rc_key == abi.WQ_E_INVALID
    assert total > 0
    for r in routers:
        r.close()
    hub.close()


def _tick_async(r, w, lo, hi, dev, cap=None):
    """wq_sharded_route_tick_async on messages [lo, hi): (counters, offsets, peers, msgs) once the
    stream is done (the call itself does not wait)."""
    import torch
    M = hi - lo
    pos = torch.from_numpy(np.ascontiguousarray(w.pos[lo:hi])).to(dev)
    wo = torch.from_numpy(np.ascontiguousarray(w.world[lo:hi]).view(np.int32)).to(dev)
    se = torch.from_numpy(np.ascontiguousarray(w.sender[lo:hi]).view(np.int32)).to(dev)
    rp = torch.from_numpy(np.ascontiguousarray(w.repl[lo:hi])).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 64 * M + 64 if cap is None else cap
    peers = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    msgs = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    cnt = torch.full((24,), 0xEE, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    r.sharded_route_async(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), M, offs.data_ptr(),
                          peers.data_ptr(), msgs.data_ptr(), cap, cnt.data_ptr())
    torch.cuda.synchronize(dev)  # the handle's stream is done when the device is
    c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]
    P = int(c["n_pairs"])
    return c, offs.cpu().numpy().view(np.uint32), peers.cpu().numpy().view(np.uint32)[:P], \
        msgs.cpu().numpy().view(np.uint32)[:P]


def test_hub_async_ticks_vs_whole_table_oracle():
    """wq_sharded_route_tick_async (no end-of-tick read; budgets from the tick two calls back): exact
    and budgeted ticks give the oracle's CSR with P in the device counters; a tick that outgrows its
    budgets reports bit 64 on every shard (outputs not valid) and later ticks recover — through an
    asynchronous tick on budgets folded in from before it, and through a synchronous tick that redoes
    itself exactly."""
    import torch
    from worldql_server_amd.router import Hub, Router
    w, _ = _workload(seed=31)
    M = len(w.world)
    G = 3
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    results = [None] * G

    def body(rank):
        r = routers[rank]
        r.attach_hub(hub, rank)
        r.sharded_apply_ops(w.ops)
        lo, hi = _slice(M, G, rank)
        half = lo + (hi - lo) // 2
        got = [("a", lo, half, _tick_async(r, w, lo, half, dev)),
               ("a", lo, half, _tick_async(r, w, lo, half, dev)),
               ("a", lo, hi, _tick_async(r, w, lo, hi, dev)),     # twice the messages: over budget
               ("a", lo, half, _tick_async(r, w, lo, half, dev))]
        h1 = r.route_health()
        got.append(("s", lo, hi, _tick(r, w, lo, hi, dev)))      # synchronous: redone exactly
        got.append(("a", lo, lo + 7, _tick_async(r, w, lo, lo + 7, dev)))
        got.append(("a", lo, hi, _tick_async(r, w, lo, hi, dev)))
        results[rank] = (got, h1, r.route_health(), r.shard_tick_stats())

    _run_shards(G, body)
    for rank in range(G):
        got, h1, h2, stats = results[rank]
        for k, (kind, a, b, g) in enumerate(got):
            want = _expected([w.ops], w, a, b)
            if kind == "s":
                _check(g, want, b - a)
                continue
            c, offs, peers, msgs = g
            if k == 2:  # outgrew its budgets: flagged, not valid
                assert int(c["error"]) & 64, (rank, c)
                continue
            assert int(c["error"]) == 0 and int(c["overflow"]) == 0, (rank, k, c)
            assert int(c["n_pairs"]) == len(want[1])
            _check((0, offs, peers, msgs), want, b - a)
        assert h1[0] & 64 and not (h2[0] & 64), (h1, h2)
    for r in routers:
        r.close()
    hub.close()
