"""One handle over G GPUs (wq_router_create_multi_mode, csrc/wq_multi.hip) against the oracle: the
reference keeps ONE WorldMap in one task (worldql_server/src/processing/thread.rs:119), and the
multi handle must answer every call with that one table's result, in both layouts (cube-hash shards,
and replicas of the whole table). G in {1, 2, 3}, all on cuda:0 here (the box has one GPU; devices
may repeat)."""
import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth

pytestmark = pytest.mark.gpu


def _workload():
    w = synth.uniform_box(31, 2500, 12000, 80.0, neighbourhood=True, repl_mode="mixed", n_worlds=3)
    rng = np.random.default_rng(31)
    un = w.ops[rng.choice(len(w.ops), 3000, replace=False)].copy()
    un["kind"] = abi.OP_UNSUBSCRIBE
    rm = abi.ops_array(np.full(30, abi.WORLD_INVALID, np.uint32), rng.choice(2500, 30, replace=False),
                       np.full(30, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((30, 3)))
    return w, abi.concat_ops([un, rm])


MODES = ["cube", "replicate"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("G", [1, 2, 3])
def test_multi_handle_is_one_table(G, mode):
    import torch
    from worldql_server_amd.router import Router
    w, churn = _workload()
    M = len(w.world)
    r = Router.multi(16, [0] * G, mode=mode)
    assert r.n_gpus() == G and r.multi_mode() == {"cube": abi.MULTI_CUBE_HASH, "replicate": abi.MULTI_REPLICATE}[mode]
    o = orc.COracle(16)
    r.apply_ops(w.ops)
    o.apply_ops(w.ops)
    r.apply_ops(churn)
    o.apply_ops(churn)
    r.remove_peers(np.array([3, 4, 5], np.uint32))
    o.apply_ops(abi.ops_array(np.full(3, abi.WORLD_INVALID, np.uint32), np.array([3, 4, 5]),
                              np.full(3, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((3, 3))))

    # the hot path, host arrays (twice: the second reuses the shards' staging)
    want_offs, want_peers, _ = o.route(w.pos, w.world, w.sender, w.repl)
    for _ in range(2):
        offs, peers, msgs = r.route(w.pos, w.world, w.sender, w.repl, with_msgs=True)
        assert (offs == want_offs).all() and (peers == want_peers).all()
        assert (msgs == np.repeat(np.arange(M, dtype=np.uint32), np.diff(want_offs.astype(np.int64)))).all()
    # a capacity too small: WQ_E_CAPACITY with the size, then the retry inside route()
    offs, peers, _ = r.route(w.pos, w.world, w.sender, w.repl, capacity=None)
    assert (peers == want_peers).all()

    # device pointers on devices[0]
    dev = torch.device("cuda:0")
    pos = torch.from_numpy(w.pos).to(dev)
    wo = torch.from_numpy(w.world.view(np.int32)).to(dev)
    se = torch.from_numpy(w.sender.view(np.int32)).to(dev)
    rp = torch.from_numpy(w.repl).to(dev)
    d_off = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = len(want_peers) + 100
    d_peers = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    r.route_device(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), M, d_off.data_ptr(), d_peers.data_ptr(),
                   None, cap, cnt.data_ptr())
    torch.cuda.synchronize()
    c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]
    assert int(c["n_pairs"]) == len(want_peers) and c["overflow"] == 0 and c["error"] == 0
    assert (d_off.cpu().numpy().view(np.uint32) == want_offs).all()
    assert (d_peers[:len(want_peers)].cpu().numpy().view(np.uint32) == want_peers).all()

    # queries (area_map.rs:33-67)
    idx = np.arange(0, len(w.ops), 37)
    ops = w.ops[idx]
    got = r.is_subscribed(ops["world"], ops["peer"], False, ops["pos"])
    want = np.array([o.is_subscribed(int(x["world"]), int(x["peer"]), False, x["pos"]) for x in ops])
    assert (got == want).all() and want.any() and not want.all()
    peers_q = np.arange(0, 2500, 7, dtype=np.uint32)
    for world in range(3):
        got = r.is_subscribed_any(np.full(len(peers_q), world, np.uint32), peers_q)
        want = np.array([o.is_subscribed_any(world, int(p)) for p in peers_q])
        assert (got == want).all()
        assert (r.world_peers(world) == o.world_peers(world)).all()
    st = r.stats()
    e, cubes = o.counts()
    assert st["n_entries"] == e and st["n_cubes"] == cubes
    assert st["n_any"] == sum(len(o.world_peers(x)) for x in range(3))

    # GlobalMessage to a world (global_message.rs:36-84) on the merged any-keys
    gw = np.array([0, 1, 2, 7, 1], np.uint32)
    gs = np.array([10, 11, 12, 13, 6], np.uint32)
    gr = np.array([0, 1, 2, 0, 2], np.uint8)
    g_offs, g_peers, _ = r.route_global(gw, gs, gr)
    wo_, wp_ = o.route_global(gw, gs, gr)
    assert (g_offs == wo_).all() and (g_peers == wp_).all()

    # after more ops the merged any-keys follow
    more = abi.ops_array(np.zeros(5, np.uint32), np.arange(5000, 5005), np.zeros(5, np.uint8),
                         pos=np.ones((5, 3)) * 7.0)
    r.apply_ops(more)
    o.apply_ops(more)
    assert (r.world_peers(0) == o.world_peers(0)).all()
    assert r.route_health()[0] == 0  # no error bits (overflow holds route()'s capacity retries)
    r.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("G", [2, 3])
def test_multi_handle_radius_filter(G, mode):
    """C5's exact radius filter through the multi handle: positions and radius go to every shard."""
    from worldql_server_amd.router import Router
    w = synth.uniform_box(33, 3000, 9000, 64.0, neighbourhood=True, repl_mode="mixed")
    rng = np.random.default_rng(33)
    peer_pos = rng.uniform(-64, 64, (3000, 3))
    r = Router.multi(16, [0] * G, mode=mode)
    r.apply_ops(w.ops)
    r.set_peer_positions(peer_pos)
    r.set_radius(14.0)
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    offs, peers, _ = r.route(w.pos, w.world, w.sender, w.repl)
    wo_, wp_ = o.route_radius(w.pos, w.world, w.sender, w.repl, peer_pos, 14.0)[:2]
    assert (offs == wo_).all() and (peers == wp_).all() and len(peers) > 0
    r.close()


def _dev_slices(w, G, dev):
    """G contiguous slices of the tick's messages as device tensors (one per device of the handle)."""
    import torch
    M = len(w.world)
    out = []
    for g in range(G):
        lo, hi = M * g // G, M * (g + 1) // G
        t = (torch.from_numpy(np.ascontiguousarray(w.pos[lo:hi])).to(dev),
             torch.from_numpy(np.ascontiguousarray(w.world[lo:hi]).view(np.int32)).to(dev),
             torch.from_numpy(np.ascontiguousarray(w.sender[lo:hi]).view(np.int32)).to(dev),
             torch.from_numpy(np.ascontiguousarray(w.repl[lo:hi])).to(dev))
        out.append((lo, hi, t))
    torch.cuda.synchronize()
    return out


class _DevWords:
    """32-bit words at a device address, for torch.as_tensor (__cuda_array_interface__)."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i4", "data": (ptr, False), "version": 3}


def _view_arrays(v):
    """A slice view's CSR (device pointers into the handle's workspace) copied to the host."""
    import torch
    n, P = int(v.n_msgs), int(v.n_pairs)

    def get(ptr, cnt):
        if cnt == 0:
            return np.empty(0, np.uint32)
        return torch.as_tensor(_DevWords(ptr, cnt), device="cuda:0").cpu().numpy().view(np.uint32)
    return get(v.offsets, n + 1), get(v.peers, P), (get(v.msgs, P) if v.msgs else None)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("G", [1, 2, 3])
def test_multi_slices_stay_on_their_devices(G, mode):
    """wq_route_tick_slices_device: every device routes its own ingested slice and keeps its CSR
    (the scaling form: no pair crosses to devices[0]); each view equals the oracle's CSR of that
    slice, twice (the second reuses the staging)."""
    import torch
    from worldql_server_amd.router import Router
    w, churn = _workload()
    r = Router.multi(16, [0] * G, mode=mode)
    o = orc.COracle(16)
    for ops in (w.ops, churn):
        r.apply_ops(ops)
        o.apply_ops(ops)
    dev = torch.device("cuda:0")
    sl = _dev_slices(w, G, dev)
    for _ in range(2):
        views = r.route_slices_device([(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), hi - lo)
                                       for lo, hi, t in sl], with_msgs=True)
        for (lo, hi, _), v in zip(sl, views):
            want_offs, want_peers, _ = o.route(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])
            offs, peers, msgs = _view_arrays(v)
            assert v.device == 0 and v.n_msgs == hi - lo
            assert (offs == want_offs).all() and (peers == want_peers).all()
            assert (msgs == np.repeat(np.arange(hi - lo, dtype=np.uint32), np.diff(want_offs.astype(np.int64)))).all()
    assert r.route_health() == (0, 0)
    r.close()


@pytest.mark.parametrize("mode", MODES)
def test_multi_slice_views_survive_other_calls(mode):
    """the views of wq_route_tick_slices_device live in a staging of their own, so every
    other call on the handle — a full route, the read-only queries (area_map.rs:33-67), stats, a
    GlobalMessage, even an op batch — leaves them intact until the next slices call."""
    import torch
    from worldql_server_amd.router import Router
    w, churn = _workload()
    G = 3
    r = Router.multi(16, [0] * G, mode=mode)
    o = orc.COracle(16)
    r.apply_ops(w.ops)
    o.apply_ops(w.ops)
    sl = _dev_slices(w, G, torch.device("cuda:0"))
    views = r.route_slices_device([(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), hi - lo)
                                   for lo, hi, t in sl], with_msgs=True)
    want = [o.route(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi])[:2] for lo, hi, _ in sl]
    # everything else the handle offers, in between
    r.route(w.pos[::-1].copy(), w.world[::-1].copy(), w.sender[::-1].copy(), w.repl[::-1].copy(), with_msgs=True)
    ops = w.ops[::41]
    r.is_subscribed(ops["world"], ops["peer"], False, ops["pos"])
    r.is_subscribed_any(np.zeros(50, np.uint32), np.arange(50, dtype=np.uint32))
    r.world_peers(1)
    r.stats()
    r.route_global(np.array([0, 1], np.uint32), np.array([1, 2], np.uint32), np.array([0, 0], np.uint8))
    r.apply_ops(churn)
    torch.cuda.synchronize()
    for (lo, hi, _), v, (w_offs, w_peers) in zip(sl, views, want):
        offs, peers, msgs = _view_arrays(v)
        assert (offs == w_offs).all() and (peers == w_peers).all()
        assert (msgs == np.repeat(np.arange(hi - lo, dtype=np.uint32), np.diff(w_offs.astype(np.int64)))).all()
    r.close()


@pytest.mark.parametrize("mode", MODES)
def test_multi_device_batches_back_to_back(mode):
    """device batches issued back to back, each larger than the last (the handle's
    staging grows while the sub-handles may still copy the previous batch out of it), each caller
    buffer rewritten on the handle's stream right after its call; the table must end as the oracle's."""
    import torch
    from worldql_server_amd.router import Router
    w, churn = _workload()
    G = 3
    r = Router.multi(16, [0] * G, mode=mode)
    stream = torch.cuda.Stream()
    r.set_stream(stream.cuda_stream)
    o = orc.COracle(16)
    r.apply_ops(w.ops)
    o.apply_ops(w.ops)
    sub_unsub = churn[churn["kind"] != abi.OP_REMOVE_PEER]
    rng = np.random.default_rng(7)
    more = w.ops[rng.choice(len(w.ops), 6000, replace=False)].copy()
    more["kind"] = abi.OP_UNSUBSCRIBE
    more["kind"][::2] = abi.OP_SUBSCRIBE
    more["peer"] = rng.integers(0, 2500, len(more))
    allops = abi.concat_ops([sub_unsub, more])
    bounds = [0, 100, 400, 1200, 3000, len(allops)]
    dev = torch.device("cuda:0")
    with torch.cuda.stream(stream):
        for a, b in zip(bounds[:-1], bounds[1:]):
            part = np.ascontiguousarray(allops[a:b])
            d = torch.from_numpy(part.view(np.uint8).copy()).to(dev, non_blocking=False)
            stream.synchronize()
            r.apply_ops_device(d.data_ptr(), len(part))
            d.fill_(0xAB)  # the caller reuses its buffer as soon as its stream has passed the call
            o.apply_ops(part)
    stream.synchronize()
    want_offs, want_peers, _ = o.route(w.pos, w.world, w.sender, w.repl)
    offs, peers, _ = r.route(w.pos, w.world, w.sender, w.repl)
    assert (offs == want_offs).all() and (peers == want_peers).all()
    assert r.route_health() == (0, 0)
    assert r.stats()["n_entries"] == o.counts()[0]
    r.close()


@pytest.mark.parametrize("mode", MODES)
def test_multi_device_batches(mode):
    """wq_apply_ops_device on a multi handle keeps the single-GPU contract: a valid batch
    is applied (cube hash: partitioned by owner on devices[0]; replicate: on every replica,
    asynchronously), a batch holding an invalid op is not applied at all, the call returns WQ_OK and
    wq_route_health reports error bit 16."""
    import torch
    from worldql_server_amd.router import Router
    w, churn = _workload()
    G = 3
    r = Router.multi(16, [0] * G, mode=mode)
    o = orc.COracle(16)
    r.apply_ops(w.ops)
    o.apply_ops(w.ops)
    sub_unsub = churn[churn["kind"] != abi.OP_REMOVE_PEER]
    dev = torch.device("cuda:0")
    d_ops = torch.from_numpy(np.ascontiguousarray(sub_unsub).view(np.uint8).copy()).to(dev)
    torch.cuda.synchronize()
    r.apply_ops_device(d_ops.data_ptr(), len(sub_unsub))
    o.apply_ops(sub_unsub)
    want_offs, want_peers, _ = o.route(w.pos, w.world, w.sender, w.repl)
    offs, peers, _ = r.route(w.pos, w.world, w.sender, w.repl)
    assert (offs == want_offs).all() and (peers == want_peers).all()
    assert r.route_health() == (0, 0)
    bad = np.ascontiguousarray(w.ops[:50]).copy()
    bad["kind"] = abi.OP_UNSUBSCRIBE
    bad["kind"][17] = abi.OP_REMOVE_PEER
    d_bad = torch.from_numpy(bad.view(np.uint8).copy()).to(dev)
    torch.cuda.synchronize()
    r.apply_ops_device(d_bad.data_ptr(), len(bad))  # returns WQ_OK: the rejection is in the health bits
    offs, peers, _ = r.route(w.pos, w.world, w.sender, w.repl)
    assert (offs == want_offs).all() and (peers == want_peers).all()  # nothing of it applied
    err, _ = r.route_health()
    assert err & 16, err
    r.close()


@pytest.mark.parametrize("mode", MODES)
def test_multi_health_counts_only_the_callers_capacity(mode):
    """the multi handle's internal staging starts at 16 pairs per message and grows; that
    must not show as an overflow in wq_route_health when the caller's own capacity was enough —
    while a caller capacity that is too small must."""
    import torch
    from worldql_server_amd.router import Router
    w = synth.uniform_box(37, 400, 3000, 24.0, neighbourhood=True, repl_mode="mixed")  # ~100 per message
    G = 2
    r = Router.multi(16, [0] * G, mode=mode)
    o = orc.COracle(16)
    r.apply_ops(w.ops)
    o.apply_ops(w.ops)
    want_offs, want_peers, _ = o.route(w.pos, w.world, w.sender, w.repl)
    assert len(want_peers) > 20 * len(w.world)
    offs, peers, _ = r.route(w.pos, w.world, w.sender, w.repl, capacity=len(want_peers) + 10)
    assert (peers == want_peers).all()
    assert r.route_health() == (0, 0)
    from worldql_server_amd.router import WQError
    with pytest.raises(WQError):
        r.route(w.pos, w.world, w.sender, w.repl, capacity=len(want_peers) // 2)
    assert r.route_health()[1] == 1
    r.close()


def test_multi_global_route_keeps_shard_errors():
    """wq_route_health on a multi handle ORs its own words into the shards' bits (a route
    on the handle's own any-keys must not overwrite a shard's error)."""
    import torch
    from worldql_server_amd.router import Router
    w, _ = _workload()
    r = Router.multi(16, [0] * 2, mode="cube")
    r.apply_ops(w.ops)
    r.route_global(np.array([0, 1], np.uint32), np.array([1, 2], np.uint32), np.array([0, 0], np.uint8))
    dev = torch.device("cuda:0")
    bad = np.ascontiguousarray(w.ops[:8]).copy()
    bad["world"][3] = abi.WORLD_INVALID
    d_bad = torch.from_numpy(bad.view(np.uint8).copy()).to(dev)
    torch.cuda.synchronize()
    r.apply_ops_device(d_bad.data_ptr(), len(bad))
    r.route_global(np.array([0], np.uint32), np.array([1], np.uint32), np.array([0], np.uint8))
    err, _ = r.route_health()
    assert err & 16, err
    r.close()


@pytest.mark.parametrize("mode", MODES)
def test_multi_slices_full_c3_two_devices(mode):
    """The north_star configuration through the scaling form of the multi handle: full C3 (1M peers x
    27 cubes, 10M hotspot messages) on a G = 2 handle (both on cuda:0 here), each device routing its
    5M messages; every message's recipients checked against the whole-table oracle."""
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router
    w = synth_ext.config_c3()
    G = 2
    r = Router.multi(16, [0] * G, mode=mode)
    r.apply_ops(w.ops)
    r.set_fanout_hint(40.0)
    sl = _dev_slices(w, G, torch.device("cuda:0"))
    views = r.route_slices_device([(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), hi - lo)
                                   for lo, hi, t in sl])
    got = [(_view_arrays(v)[:2]) for v in views]  # copied out before the handle's next call
    r.close()
    del sl
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    P = 0
    for (lo, hi), (offs, peers) in zip([(w_lo, w_hi) for w_lo, w_hi, _ in _dev_slices_bounds(len(w.world), G)],
                                       got):
        bad, first = o.route_check(w.pos[lo:hi], w.world[lo:hi], w.sender[lo:hi], w.repl[lo:hi], offs, peers)
        assert bad == 0, f"slice [{lo}, {hi}): {bad} messages differ, first {first}"
        P += len(peers)
    assert P > 4e8


def _dev_slices_bounds(M, G):
    return [(M * g // G, M * (g + 1) // G, None) for g in range(G)]
