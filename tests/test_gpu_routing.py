"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bar: bit-exact. Cube keys are compared as integers; recipient sets are compared per message as
sorted peer lists (the reference's AHashSet order is random per process).
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from worldql_server_amd.router import load_library
    return load_library()


def mk_router(cube_size=16, hash_bits=64):
    from worldql_server_amd.router import Router
    return Router(cube_size, 0, hash_bits=hash_bits)


# ---- kernel (1) -------------------------------------------------------------------------

def test_quantize_reference_kats(lib, kats):
    from worldql_server_amd.router import quantize
    for c, s, e in kats["coord_clamp"]:
        assert int(quantize(np.array([c]), s)[0]) == e
    for p, s, e in kats["from_vector3"]:
        assert quantize(np.array(p), s).tolist() == e


def test_quantize_edge_vectors(lib, golden_dir):
    from worldql_server_amd.router import quantize
    with open(os.path.join(golden_dir, "quantize_edges.json")) as f:
        vecs = json.load(f)["vectors"]
    x = np.array([float(v[0]) for v in vecs])
    s = np.array([v[1] for v in vecs])
    want = np.array([v[2] for v in vecs], dtype=np.int64)
    for size in np.unique(s):
        m = s == size
        got = quantize(x[m], int(size))
        assert (got == want[m]).all(), (size, x[m][got != want[m]])


def test_quantize_random_bit_patterns(lib, golden_dir):
    from worldql_server_amd.router import quantize
    z = np.load(os.path.join(golden_dir, "quantize_random.npz"))
    for key in z.files:
        if key.startswith("x_"):
            assert (quantize(z[key], int(key[2:])) == z["k_" + key[2:]]).all(), key
    rng = synth.SplitMix64(4242)
    x = rng.next_u64(2_000_000).view(np.float64)
    k = (rng.next_u64(500_000) >> np.uint64(11)).astype(np.float64)
    for s in (1, 7, 16, 65535):
        mult = k * s
        xs = np.concatenate([x, mult, -mult, np.nextafter(mult, np.inf), np.nextafter(-mult, -np.inf)])
        assert (quantize(xs, s) == orc.c_coord_clamp(xs, s)).all(), s


# ---- reference unit tests through the WorldMap / AreaMap façade on the GPU ----------------

@pytest.mark.parametrize("name", ["area_subscriptions", "world_subscriptions"])
def test_area_map_kats_gpu(kats, name):
    from tests.test_oracle import run_membership_sequence
    from worldql_server_amd.subscriptions import CubeArea, Vector3, WorldMap
    seq = kats[name]
    wm = WorldMap(seq["cube_size"])
    am = wm.get_mut("world")
    cube = lambda raw, k: CubeArea(*map(int, k)) if raw else Vector3(*map(float, k))  # noqa: E731
    run_membership_sequence(
        seq,
        add=lambda u, raw, k: am.add_subscription(u, cube(raw, k)),
        remove=lambda u, raw, k: am.remove_subscription(u, cube(raw, k)),
        remove_peer=lambda u: am.remove_peer(u),
        is_sub=lambda u, raw, k: am.is_peer_subscribed(u, cube(raw, k)),
        is_any=lambda u: am.is_peer_subscribed_any(u),
    )


def test_add_remove_return_values_gpu():
    """area_map.rs:69-119: add -> newly added; remove -> was present; absent cube -> false."""
    from worldql_server_amd.subscriptions import CubeArea, Vector3, WorldMap
    wm = WorldMap(16)
    am = wm.get_mut("world")
    assert am.add_subscription("u", Vector3(6.3, 1.0, 10.5)) is True
    assert am.add_subscription("u", CubeArea(16, 16, 16)) is False
    assert am.remove_subscription("u", CubeArea(0, 0, 0)) is False
    assert am.remove_subscription("u", CubeArea(16, 16, 16)) is True
    assert am.remove_subscription("u", CubeArea(16, 16, 16)) is False
    assert wm.get("other") is None
    assert sorted(wm.get_mut("w2").get_subscribed_any_peers()) == []
    am.add_subscription("v", CubeArea(16, 16, 16))
    assert list(am.get_subscribed_peers(Vector3(1.0, 1.0, 1.0))) == ["v"]
    assert wm.remove_peer("v") is True and wm.remove_peer("v") is False


# ---- routing parity ---------------------------------------------------------------------

def _compare(r, o, pos, world, sender, repl, keys=None):
    offs, peers, msgs = r.route(pos, world, sender, repl, keys=keys, with_msgs=True)
    o_offs, o_peers, _ = o.route(pos, world, sender, repl, keys=keys)
    assert (offs == o_offs).all()
    assert (peers == o_peers).all()  # GPU order is ascending per message; oracle sorted per message
    M = len(world)
    assert (msgs == np.repeat(np.arange(M, dtype=np.uint32), np.diff(offs.astype(np.int64)))).all()
    return len(peers)


def test_routing_golden_fixtures(golden_dir):
    z = np.load(os.path.join(golden_dir, "routing_cases.npz"))
    for c in range(int(z["n_cases"][0])):
        p = f"c{c}_"
        r = mk_router(int(z[p + "cube_size"][0]))
        r.apply_ops(z[p + "ops"].view(abi.OP_DTYPE))
        offs, peers, _ = r.route(z[p + "pos"], z[p + "world"], z[p + "sender"], z[p + "repl"])
        assert (offs == z[p + "offsets"]).all(), c
        assert (peers == z[p + "peers"]).all(), c


@pytest.mark.parametrize("hash_bits", [64, 6, 1])
def test_routing_vs_oracle_c1(hash_bits):
    """C1 (the reference's CPU config) with all replication modes; hash_bits < 64 forces bucket
    collisions so the exact build path and long probe walks are exercised."""
    w = synth.config_c1(repl_mode="mixed")
    r = mk_router(16, hash_bits)
    r.apply_ops(w.ops)
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    assert r.stats()["n_entries"] == o.counts()[0]
    assert r.stats()["n_cubes"] == o.counts()[1]
    if hash_bits < 64:
        assert r.stats()["hash_fallbacks"] >= 1
    P = _compare(r, o, w.pos, w.world, w.sender, w.repl)
    assert P > 0


def test_routing_vs_oracle_c2_scaled():
    w = synth.config_c2(repl_mode="mixed", scale=0.02)
    r = mk_router(16)
    r.apply_ops(w.ops)
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    _compare(r, o, w.pos, w.world, w.sender, w.repl)


def test_churn_sequences_vs_oracle():
    """Subscribe / unsubscribe / remove_peer batches applied incrementally (last op wins)."""
    rng = synth.SplitMix64(777)
    r = mk_router(10)
    o = orc.COracle(10)
    n_peers, n_worlds = 300, 4
    for tick in range(6):
        n = 3000
        kind = (rng.next_u64(n) % np.uint64(10)).astype(np.int64)
        kinds = np.where(kind < 6, abi.OP_SUBSCRIBE, np.where(kind < 9, abi.OP_UNSUBSCRIBE, abi.OP_REMOVE_PEER))
        world = rng.below(n_worlds, n)
        world = np.where((kinds == abi.OP_REMOVE_PEER) & (rng.below(2, n) == 0), abi.WORLD_INVALID, world)
        peer = rng.below(n_peers, n)
        pos = np.floor(rng.uniform(-60, 60, 3 * n).reshape(n, 3) / 5.0) * 5.0  # many repeats + multiples
        ops = abi.ops_array(world, peer, kinds, pos=pos)
        r.apply_ops(ops)
        o.apply_ops(ops)
        assert r.stats()["n_entries"] == o.counts()[0]
        M = 4000
        mpos = rng.uniform(-70, 70, 3 * M).reshape(M, 3)
        mw = rng.below(n_worlds + 1, M)
        ms = rng.below(n_peers, M)
        mr = rng.below(3, M).astype(np.uint8)
        _compare(r, o, mpos, mw, ms, mr)
        for wid in range(n_worlds):
            assert (r.world_peers(wid) == o.world_peers(wid)).all()
        q_w, q_p = rng.below(n_worlds + 1, 500), rng.below(n_peers, 500)
        assert (r.is_subscribed_any(q_w, q_p) == [o.is_subscribed_any(int(a), int(b)) for a, b in zip(q_w, q_p)]).all()


def test_raw_keys_and_off_grid():
    r = mk_router(16)
    o = orc.COracle(16)
    keys = np.array([[0, 0, 0], [16, 16, 16], [1, 2, 3], [-9223372036854775808, 5, 9223372036854775807]])
    ops = abi.ops_array(np.zeros(4, np.uint32), np.arange(4), np.zeros(4, np.uint8), key=keys)
    r.apply_ops(ops)
    o.apply_ops(ops)
    mk = np.concatenate([keys, [[0, 0, 1]]])
    M = len(mk)
    _compare(r, o, None, np.zeros(M, np.uint32), np.full(M, 99, np.uint32), np.ones(M, np.uint8), keys=mk)


def test_edge_positions_route():
    """NaN / inf / denormal / 2^63 positions land in the same buckets as in the reference."""
    r = mk_router(16)
    o = orc.COracle(16)
    vals = np.array([0.0, -0.0, 5e-324, -5e-324, np.nan, np.inf, -np.inf, 1e300, -1e300, 2.0**63, 16.0, -16.0])
    g = np.stack(np.meshgrid(vals, vals[:4], vals[4:8], indexing="ij"), -1).reshape(-1, 3)
    n = len(g)
    ops = abi.ops_array(np.zeros(n, np.uint32), np.arange(n) % 7, np.zeros(n, np.uint8), pos=g)
    r.apply_ops(ops)
    o.apply_ops(ops)
    _compare(r, o, g, np.zeros(n, np.uint32), np.arange(n, dtype=np.uint32) % 9, (np.arange(n) % 3).astype(np.uint8))


def test_empty_inputs():
    r = mk_router(16)
    offs, peers, _ = r.route(np.zeros((0, 3)), np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
    assert offs.tolist() == [0] and len(peers) == 0
    offs, peers, _ = r.route(np.zeros((5, 3)), np.zeros(5, np.uint32), np.zeros(5, np.uint32), np.zeros(5, np.uint8))
    assert offs.tolist() == [0] * 6
    r.apply_ops(np.zeros(0, abi.OP_DTYPE))
    r.remove_peers([1, 2, 3])
    assert r.stats()["n_entries"] == 0


def test_hot_cube_skew_and_ragged_tiles():
    """One cube with thousands of subscribers plus light cubes; M not a multiple of the tile."""
    r = mk_router(16)
    o = orc.COracle(16)
    n_hot = 5000
    ops = [abi.ops_array(np.zeros(n_hot, np.uint32), np.arange(n_hot), np.zeros(n_hot, np.uint8),
                         pos=np.full((n_hot, 3), 1.0))]
    rng = synth.SplitMix64(5)
    ops.append(abi.ops_array(np.zeros(2000, np.uint32), rng.below(9000, 2000), np.zeros(2000, np.uint8),
                             pos=rng.uniform(-200, 200, 6000).reshape(2000, 3)))
    ops = abi.concat_ops(ops)
    r.apply_ops(ops)
    o.apply_ops(ops)
    M = 3 * 1024 + 77
    pos = rng.uniform(-200, 200, 3 * M).reshape(M, 3)
    pos[::5] = 3.0  # every fifth message hits the hot cube
    P = _compare(r, o, pos, np.zeros(M, np.uint32), rng.below(n_hot, M), rng.below(3, M).astype(np.uint8))
    assert P > 300 * n_hot  # ~660 hot messages, 2/3 of them not OnlySelf


@pytest.mark.parametrize("per_cube", [23, 24, 25, 60])
def test_inline_boundary_and_stage_overflow(per_cube):
    """Cubes around the inline record boundary (kInline = 24 peers: 23/24/25) and far past it (60),
    every message landing in them, under every route kernel configuration."""
    r = mk_router(16)
    o = orc.COracle(16)
    n_cubes = 40
    cx = np.repeat(np.arange(n_cubes) * 16.0 + 8.0, per_cube)
    peer = np.arange(n_cubes * per_cube, dtype=np.uint32)
    pos = np.stack([cx, np.full_like(cx, 8.0), np.full_like(cx, -8.0)], 1)
    ops = abi.ops_array(np.zeros(len(cx), np.uint32), peer, np.zeros(len(cx), np.uint8), pos=pos)
    r.apply_ops(ops)
    o.apply_ops(ops)
    rng = synth.SplitMix64(per_cube)
    M = 5000
    mpos = np.stack([rng.below(n_cubes, M) * 16.0 + rng.uniform(0.5, 15.5, M), rng.uniform(0.5, 15.5, M),
                     -rng.uniform(0.5, 15.5, M)], 1)
    for cfg in range(r.route_config_count()):
        r.set_route_config(cfg)
        _compare(r, o, mpos, np.zeros(M, np.uint32), rng.below(n_cubes * per_cube, M),
                 rng.below(3, M).astype(np.uint8))


def test_capacity_overflow_reports_required_size():
    from worldql_server_amd.router import WQError
    r = mk_router(16)
    ops = abi.ops_array(np.zeros(100, np.uint32), np.arange(100), np.zeros(100, np.uint8), pos=np.ones((100, 3)))
    r.apply_ops(ops)
    with pytest.raises(WQError) as e:
        r.route(np.ones((10, 3)), np.zeros(10, np.uint32), np.full(10, 500, np.uint32), np.zeros(10, np.uint8),
                capacity=50)
    assert e.value.code == abi.WQ_E_CAPACITY
    offs, peers, _ = r.route(np.ones((10, 3)), np.zeros(10, np.uint32), np.full(10, 500, np.uint32),
                             np.zeros(10, np.uint8))
    assert len(peers) == 1000


def test_device_api_counters_and_stream():
    import torch
    from worldql_server_amd.router import Router
    w = synth.config_c2(scale=0.01)
    r = Router(16, 0)
    r.apply_ops(w.ops)
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev)
    r.set_stream(stream.cuda_stream)
    M = len(w.world)
    pos = torch.from_numpy(w.pos).to(dev)
    world = torch.from_numpy(w.world.view(np.int32)).to(dev)
    sender = torch.from_numpy(w.sender.view(np.int32)).to(dev)
    repl = torch.from_numpy(w.repl).to(dev)
    cap = 40 * M
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    r.route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
                   peers.data_ptr(), msgs.data_ptr(), cap, cnt.data_ptr())
    torch.cuda.synchronize()
    c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    o_offs, o_peers, F = o.route(w.pos, w.world, w.sender, w.repl)
    assert int(c["n_pairs"]) == len(o_peers) and int(c["n_candidates"]) == F
    assert c["overflow"] == 0 and c["error"] == 0
    assert (offs.cpu().numpy().view(np.uint32) == o_offs).all()
    assert (peers[: len(o_peers)].cpu().numpy().view(np.uint32) == o_peers).all()
    r.set_stream(None)


def test_full_c2_size_properties():
    """BASELINE config C2 at full size: size-independent properties, then the whole tick exact
    against the oracle (wqo_route_check: every message's recipients, no host sort)."""
    w = synth.config_c2()
    r = mk_router(16)
    r.apply_ops(w.ops)
    st = r.stats()
    assert st["n_entries"] == len(w.ops)  # positions are distinct: every subscription is live
    offs, peers, msgs = r.route(w.pos, w.world, w.sender, w.repl, with_msgs=True)
    d = np.diff(offs.astype(np.int64))
    assert (d >= 0).all() and offs[-1] == len(peers)
    # ascending (hence duplicate-free) peers inside every message, never the sender (ExceptSelf)
    same = msgs[1:] == msgs[:-1]
    assert (peers[1:][same] > peers[:-1][same]).all()
    assert not (peers == w.sender[msgs]).any()
    # exact on the whole tick against the oracle
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    bad, first = o.route_check(w.pos, w.world, w.sender, w.repl, offs, peers)
    assert bad == 0, f"{bad} messages differ, first {first}"
    assert 0.8e7 < len(peers) < 1.3e7  # P ≈ 1.0e7


def test_many_blocks_changing_tick_sizes():
    """Ticks of many 256-message blocks whose sizes grow, shrink and cross look-back windows (64
    blocks), alternating the single-launch tick (config 0: tagged granules, no clearing between
    calls) with the three-launch and spill shapes (1, 7) that share the counter ring."""
    w = synth.config_c2(repl_mode="mixed", scale=0.2)
    r = mk_router(16)
    o = orc.COracle(16)
    r.apply_ops(w.ops)
    o.apply_ops(w.ops)
    window = 64 * 256
    sizes = [3 * window + 17, 5 * 256, 7 * window + 1, 100, 2 * window, 2 * window, 12 * window - 3]
    cfgs = [0, 0, 1, 0, 7, 0, 0]
    for M, cfg in zip(sizes, cfgs):
        assert M <= len(w.world)
        r.set_route_config(cfg)
        _compare(r, o, w.pos[:M], w.world[:M], w.sender[:M], w.repl[:M])
    r.set_route_config(0)


def test_fanout_hint_selects_identical_shape():
    """wq_set_fanout_hint >= WQ_HEAVY_FANOUT (count / scan / emit with direct heavy emit) gives
    the same CSR as the single launch, on heavy fan-out (60 peers per cube) and on C2-like input."""
    r = mk_router(16)
    o = orc.COracle(16)
    n_cubes, per_cube = 40, 60
    cx = np.repeat(np.arange(n_cubes) * 16.0 + 8.0, per_cube)
    pos = np.stack([cx, np.full_like(cx, 8.0), np.full_like(cx, -8.0)], 1)
    ops = abi.ops_array(np.zeros(len(cx), np.uint32), np.arange(len(cx), dtype=np.uint32),
                        np.zeros(len(cx), np.uint8), pos=pos)
    r.apply_ops(ops)
    o.apply_ops(ops)
    rng = synth.SplitMix64(77)
    M = 20000
    mpos = np.stack([rng.below(n_cubes, M) * 16.0 + rng.uniform(0.5, 15.5, M), rng.uniform(0.5, 15.5, M),
                     -rng.uniform(0.5, 15.5, M)], 1)
    args = (mpos, np.zeros(M, np.uint32), rng.below(n_cubes * per_cube, M), rng.below(3, M).astype(np.uint8))
    for hint in (0.0, 60.0, float("nan"), 16.0):
        r.set_fanout_hint(hint)
        _compare(r, o, *args)


def test_auto_fanout_shape_from_host_ticks():
    """Without a hint, each host-array tick picks the next tick's shape from its own P / M (here
    ~60 pairs per message: the second tick runs count / scan / emit); results stay identical."""
    r = mk_router(16)
    o = orc.COracle(16)
    n_cubes, per_cube = 30, 60
    cx = np.repeat(np.arange(n_cubes) * 16.0 + 8.0, per_cube)
    pos = np.stack([cx, np.full_like(cx, 8.0), np.full_like(cx, 8.0)], 1)
    ops = abi.ops_array(np.zeros(len(cx), np.uint32), np.arange(len(cx), dtype=np.uint32),
                        np.zeros(len(cx), np.uint8), pos=pos)
    r.apply_ops(ops)
    o.apply_ops(ops)
    rng = synth.SplitMix64(91)
    assert r.route_shape() == (False, True)  # a fresh handle: single launch, automatic
    for M in (9000, 9000, 300):
        mpos = np.stack([rng.below(n_cubes, M) * 16.0 + rng.uniform(0.5, 15.5, M), rng.uniform(0.5, 15.5, M),
                         rng.uniform(0.5, 15.5, M)], 1)
        _compare(r, o, mpos, np.zeros(M, np.uint32), rng.below(n_cubes * per_cube, M),
                 rng.below(3, M).astype(np.uint8))
        assert r.route_shape() == (True, True)  # ~40 pairs per message: count / scan / emit next
    # a one-message query (AreaMap::get_subscribed_peers) must not pick the shape of real ticks
    r.route(np.array([[8.0, 8.0, 8.0]]), np.zeros(1, np.uint32), np.zeros(1, np.uint32),
            np.ones(1, np.uint8))
    assert r.route_shape() == (True, True)
    r.route(np.full((400, 3), -5000.0), np.zeros(400, np.uint32), np.zeros(400, np.uint32),
            np.zeros(400, np.uint8))  # an empty tick of >= one block: back to the single launch
    assert r.route_shape() == (False, True)
    r.set_fanout_hint(100.0)
    assert r.route_shape() == (True, False)
    r.route(np.full((400, 3), -5000.0), np.zeros(400, np.uint32), np.zeros(400, np.uint32),
            np.zeros(400, np.uint8))
    assert r.route_shape() == (True, False)  # the caller's hint holds
    r.set_fanout_hint(-1.0)
    assert r.route_shape()[1] is True  # a negative hint hands the choice back


@pytest.mark.parametrize("chunks", [2, 3, 7])
def test_pipelined_heavy_tick_is_identical(chunks):
    """wq_debug_set_route_chunks: the heavy tick in pipelined chunks (counts on a side stream, each
    chunk's scan carrying {P, F} into the next, its emit writing msgs from the chunk's first message)
    gives the oracle's CSR and msgs, and the same counters as one chunk — host arrays, device arrays,
    a capacity too small, and a tick too short to chunk."""
    import torch
    from worldql_server_amd import synth_ext
    w = synth_ext.config_c3(scale=0.02)  # 200k hotspot messages, 782 count tiles
    M = len(w.world)
    repl = synth.stream(3, 99).below(3, M).astype(np.uint8)
    r = mk_router(16)
    r.apply_ops(w.ops)
    r.set_fanout_hint(40.0)
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    r.set_route_chunks(chunks)
    P = _compare(r, o, w.pos, w.world, w.sender, repl)
    _compare(r, o, w.pos[:300], w.world[:300], w.sender[:300], repl[:300])  # 2 tiles: one chunk
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (w.pos, w.world.view(np.int32),
                                                                      w.sender.view(np.int32), repl)]
    got = {}
    for c in (1, chunks):
        r.set_route_chunks(c)
        for cap in (P + 64, P // 3):
            offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
            peers = torch.full((P + 64,), -1, dtype=torch.int32, device=dev)
            msgs = torch.full((P + 64,), -1, dtype=torch.int32, device=dev)
            cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            r.route_device(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), M, offs.data_ptr(),
                           peers.data_ptr(), msgs.data_ptr(), cap, cnt.data_ptr())
            torch.cuda.synchronize()
            k = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]
            got[(c, cap)] = (offs.cpu().numpy(), peers.cpu().numpy(), msgs.cpu().numpy(), int(k["n_pairs"]),
                             int(k["n_candidates"]), int(k["overflow"]), int(k["error"]))
        r.route_health()
    for cap in (P + 64, P // 3):
        a, b = got[(1, cap)], got[(chunks, cap)]
        assert a[3:] == b[3:] and a[3] == P, (a[3:], b[3:])
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all() and (a[2] == b[2]).all()
    assert got[(1, P // 3)][5] == 1  # the short capacity is reported, the kept prefix identical


@pytest.mark.parametrize("n_tiles", [2047, 2048, 4096, 4097, 8192 + 17])
def test_multi_block_tile_scan_boundaries(n_tiles):
    """Round 6: the count / scan / emit shape scans its per-256-message tile totals with the one-launch
    multi-block scan from 2,048 tiles on (4,096 tiles per block, 16 per thread): tile counts at and
    across its thresholds, its block boundary and its 16-tile vector tail, on C2-shaped input with
    mixed replication — the oracle's CSR and msgs, and P / F in the device counters."""
    w = synth.config_c2(repl_mode="mixed", scale=2.2)
    M = n_tiles * 256 - 37
    assert M <= len(w.world)
    r = mk_router(16)
    r.apply_ops(w.ops)
    o = orc.COracle(16)
    o.apply_ops(w.ops)
    r.set_route_config(10)  # count / tile_scan / emit
    _compare(r, o, w.pos[:M], w.world[:M], w.sender[:M], w.repl[:M])
    r.set_route_config(0)


@pytest.mark.parametrize("hash_bits", [64, 6, 1])
def test_compact_headers_heavy_shape_vs_oracle(hash_bits):
    """Round 6: the count pass probes the compact header table (load <= 1/2, its own probe runs, the
    record slot carried in the header). Heavy-fan-out messages through count / scan / emit: scaled C3
    hotspots, or (6 / 1 hash bits: every cube in one probe run of both tables) 40 cubes of 60 peers;
    then a churn batch (the headers go stale and the count probes the records) — against the oracle."""
    from worldql_server_amd import synth_ext
    if hash_bits == 64:
        w = synth_ext.config_c3(scale=0.01)
        ops, args = w.ops, (w.pos, w.world, w.sender, w.repl)
    else:
        n_cubes, per_cube = 40, 60
        cx = np.repeat(np.arange(n_cubes) * 16.0 + 8.0, per_cube)
        pos = np.stack([cx, np.full_like(cx, 8.0), np.full_like(cx, -8.0)], 1)
        ops = abi.ops_array(np.zeros(len(cx), np.uint32), np.arange(len(cx), dtype=np.uint32),
                            np.zeros(len(cx), np.uint8), pos=pos)
        rng = synth.SplitMix64(79)
        M = 20000
        mpos = np.stack([rng.below(n_cubes + 3, M) * 16.0 + rng.uniform(0.5, 15.5, M), rng.uniform(0.5, 15.5, M),
                         -rng.uniform(0.5, 15.5, M)], 1)
        args = (mpos, np.zeros(M, np.uint32), rng.below(n_cubes * per_cube, M), rng.below(3, M).astype(np.uint8))
    r = mk_router(16, hash_bits=hash_bits)
    r.apply_ops(ops)
    r.set_fanout_hint(40.0)
    o = orc.COracle(16)
    o.apply_ops(ops)
    _compare(r, o, *args)
    un = ops[::7].copy()
    un["kind"] = abi.OP_UNSUBSCRIBE
    r.apply_ops(un)
    o.apply_ops(un)
    _compare(r, o, *args)


def test_profile_phases_and_sclk_probe():
    """wq_profile_read_phases splits each three-launch tick into count / tile scan / emit (their sum is
    the bracketed launch time, within event granularity); wq_probe_sclk reports a plausible clock."""
    w = synth.config_c2(scale=0.3)
    r = mk_router(16)
    r.apply_ops(w.ops)
    r.set_route_config(10)
    r.route(w.pos, w.world, w.sender, w.repl)
    r.profile_enable(True)
    for _ in range(3):
        r.route(w.pos, w.world, w.sender, w.repl)
    ms, n, ph, nph = r.profile_read_phases()
    r.profile_enable(False)
    assert n == 3 and nph == 3
    assert all(x > 0 for x in ph)
    assert abs(sum(ph) - ms) <= 0.05 * ms + 0.02
    r.set_route_config(0)
    r.profile_enable(True)
    r.route(w.pos, w.world, w.sender, w.repl)  # single launch: not phased
    ms, n, ph, nph = r.profile_read_phases()
    r.profile_enable(False)
    assert n == 1 and nph == 0 and ph == [0.0, 0.0, 0.0]
    mhz = r.probe_sclk()
    assert 300.0 < mhz < 4000.0, mhz
