"""CPU: the restatements (oracle/) against the reference's own unit-test vectors.

The reference cannot be built here (Rust, no toolchain: SURVEY.md §8(c)), so these KATs —
transcribed from worldql_server/src/subscriptions/cube_area.rs:102-175,
worldql_server/src/utils/round.rs:28-76 and worldql_server/src/subscriptions/area_map.rs:154-254 —
are what pins the oracle.
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi


def test_coord_clamp_kats(kats):
    for c, s, e in kats["coord_clamp"]:
        assert int(orc.coord_clamp_np(c, s)) == e
        assert int(orc.c_coord_clamp(np.array([c]), s)[0]) == e


def test_from_vector3_kats(kats):
    for p, s, e in kats["from_vector3"]:
        assert orc.quantize_np(p, s).tolist() == e
        assert orc.c_coord_clamp(np.array(p), s).tolist() == e


def test_round_by_multiple_kats(kats):
    lib = orc.load_c_oracle()
    for n, m, e in kats["round_by_multiple"]:
        assert float(orc.round_by_multiple_np(n, m)) == e
        assert lib.wqo_round_by_multiple(n, m) == e


def _key(d):
    return (True, np.array(d["raw"], np.int64)) if "raw" in d else (False, np.array(d["pos"], np.float64))


def run_membership_sequence(seq, add, remove, remove_peer, is_sub, is_any):
    for step in seq["steps"]:
        op = step["op"]
        if op is not None:
            kind, peer, key = op
            if kind == "add":
                add(peer, *_key(key))
            elif kind == "remove":
                remove(peer, *_key(key))
            else:
                remove_peer(peer)
        for peer, key, want in step.get("expect", []):
            assert is_sub(peer, *_key(key)) == want, (step, peer, key)
        for peer, want in step.get("expect_any", []):
            assert is_any(peer) == want, (step, peer)


@pytest.mark.parametrize("name", ["area_subscriptions", "world_subscriptions"])
def test_area_map_kats_on_c_oracle(kats, name):
    seq = kats[name]
    o = orc.COracle(seq["cube_size"])
    ids = {}
    pid = lambda u: ids.setdefault(u, len(ids))  # noqa: E731
    run_membership_sequence(
        seq,
        add=lambda u, raw, k: o.add_subscription(0, pid(u), raw, k),
        remove=lambda u, raw, k: o.remove_subscription(0, pid(u), raw, k),
        remove_peer=lambda u: o.apply_ops(np.array([abi.make_op(0, pid(u), abi.OP_REMOVE_PEER)], abi.OP_DTYPE)),
        is_sub=lambda u, raw, k: o.is_subscribed(0, pid(u), raw, k),
        is_any=lambda u: o.is_subscribed_any(0, pid(u)),
    )


def test_edge_vectors_both_restatements(golden_dir):
    with open(os.path.join(golden_dir, "quantize_edges.json")) as f:
        vecs = json.load(f)["vectors"]
    x = np.array([float(v[0]) for v in vecs])
    s = np.array([v[1] for v in vecs])
    want = np.array([v[2] for v in vecs], dtype=np.int64)
    for size in np.unique(s):
        m = s == size
        assert (orc.coord_clamp_np(x[m], int(size)) == want[m]).all()
        assert (orc.c_coord_clamp(x[m], int(size)) == want[m]).all()


def test_appendix_a3_table(golden_dir):
    """SURVEY.md Appendix A.3 rows (derived from the code reading of cube_area.rs:23-44)."""
    rows = [(0.0, 16, 16), (-0.0, 16, 16), (5e-324, 16, 16), (-5e-324, 16, 0), (math.nan, 16, 16),
            (math.inf, 16, -9223372036854775793), (math.inf, 10, -9223372036854775799),
            (-math.inf, 16, -9223372036854775807), (1e300, 16, 2**63 - 1), (-1e300, 16, -2**63),
            (2.0**63, 10, -9223372036854775799), (-(2.0**63), 10, -9223372036854775807),
            (16.000000000000004, 16, 32), (-16.000000000000004, 16, -32), (15.999999999999998, 10, 20)]
    for c, s, e in rows:
        assert int(orc.coord_clamp_np(c, s)) == e, (c, s)
        assert int(orc.c_coord_clamp(np.array([c]), s)[0]) == e, (c, s)


def test_random_vectors_fixture_matches_c(golden_dir):
    z = np.load(os.path.join(golden_dir, "quantize_random.npz"))
    for key in z.files:
        if key.startswith("x_"):
            s = int(key[2:])
            assert (orc.c_coord_clamp(z[key], s) == z["k_" + key[2:]]).all()


def test_random_bit_patterns_numpy_vs_c():
    from worldql_server_amd.synth import SplitMix64
    rng = SplitMix64(12345)
    x = rng.next_u64(200_000).view(np.float64)
    for s in (1, 3, 7, 16, 255, 65535):
        assert (orc.coord_clamp_np(x, s) == orc.c_coord_clamp(x, s)).all()


def test_routing_fixture_reproducible(golden_dir):
    """The committed routing fixtures are re-derivable from the C restatement."""
    z = np.load(os.path.join(golden_dir, "routing_cases.npz"))
    for c in range(int(z["n_cases"][0])):
        p = f"c{c}_"
        o = orc.COracle(int(z[p + "cube_size"][0]))
        o.apply_ops(z[p + "ops"].view(abi.OP_DTYPE))
        offs, peers, F = o.route(z[p + "pos"], z[p + "world"], z[p + "sender"], z[p + "repl"])
        assert (offs == z[p + "offsets"]).all() and (peers == z[p + "peers"]).all()
        assert F == int(z[p + "F"][0])


def test_oracle_replication_semantics():
    """local_message.rs:60-86 on a hand-made cube: ExceptSelf, IncludingSelf, OnlySelf, unknown."""
    o = orc.COracle(16)
    for p in (3, 5, 9):
        o.add_subscription(0, p, True, np.array([16, 16, 16]))
    pos = np.full((6, 3), 1.0)
    world = np.zeros(6, np.uint32)
    sender = np.array([5, 5, 5, 7, 7, 5], np.uint32)
    repl = np.array([0, 1, 2, 0, 2, 200], np.uint8)
    offs, peers, F = o.route(pos, world, sender, repl)
    segs = [peers[offs[i]:offs[i + 1]].tolist() for i in range(6)]
    assert segs == [[3, 9], [3, 5, 9], [5], [3, 5, 9], [], [3, 9]]
    assert F == 18


def test_oracle_global_message_semantics():
    """global_message.rs:36-84 on hand-made worlds: the recipients are the world's subscribed-any
    peers (area_map.rs:65-67) under the replication filter; an absent world yields nothing."""
    o = orc.COracle(16)
    for w, p, k in [(1, 3, 16), (1, 5, 32), (1, 5, 48), (1, 9, -16), (2, 5, 16), (2, 4, 16)]:
        o.add_subscription(w, p, True, np.array([k, 16, 16]))
    world = np.array([1, 1, 1, 1, 1, 2, 7, 2, 2], np.uint32)
    sender = np.array([5, 5, 5, 7, 7, 5, 5, 3, 3], np.uint32)
    repl = np.array([0, 1, 2, 0, 2, 0, 1, 2, 200], np.uint8)
    offs, peers = o.route_global(world, sender, repl)
    segs = [peers[offs[i]:offs[i + 1]].tolist() for i in range(len(world))]
    assert segs == [[3, 9], [3, 5, 9], [5], [3, 5, 9], [], [4], [], [], [4, 5]]


def test_oracle_global_matches_world_peers():
    """route_global against the subscribed-any sets on a random table (python restatement)."""
    rng = np.random.default_rng(7)
    o = orc.COracle(16)
    n = 3000
    ops = abi.ops_array(rng.integers(0, 6, n).astype(np.uint32), rng.integers(0, 400, n).astype(np.uint32),
                        np.where(rng.random(n) < 0.8, abi.OP_SUBSCRIBE, abi.OP_UNSUBSCRIBE).astype(np.uint8),
                        pos=rng.uniform(-64, 64, (n, 3)))
    o.apply_ops(ops)
    M = 500
    world = rng.integers(0, 8, M).astype(np.uint32)
    sender = rng.integers(0, 420, M).astype(np.uint32)
    repl = rng.integers(0, 4, M).astype(np.uint8)
    offs, peers = o.route_global(world, sender, repl)
    wp = {w: o.world_peers(w).tolist() for w in range(8)}
    for i in range(M):
        s, r = int(sender[i]), int(repl[i])
        all_ = wp[int(world[i])]
        want = [q for q in all_ if q == s] if r == 2 else (all_ if r == 1 else [q for q in all_ if q != s])
        assert peers[offs[i]:offs[i + 1]].tolist() == want


def test_server_faithful_route_is_route_intersect_connected():
    """cpu_server_faithful_1t (wqo_route_faithful, peer_map.rs:151-163): per message, the
    recipients of wqo_route that are connected, in PeerMap order."""
    import ctypes
    from oracle import oracle as orc
    from worldql_server_amd import synth
    w = synth.config_c1(repl_mode="mixed")
    o = orc.COracle(w.cube_size)
    o.apply_ops(w.ops)
    offs, peers, _ = o.route(w.pos, w.world, w.sender, w.repl)
    vp = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    f = o.lib.wqo_route_faithful
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_size_t]
    M = len(w.world)
    rng = np.random.default_rng(5)
    for connected in (np.arange(w.n_peers, dtype=np.uint32)[::-1].copy(),
                      rng.permutation(w.n_peers)[: w.n_peers // 3].astype(np.uint32)):
        fo = np.empty(M + 1, np.uint32)
        fp = np.empty(64 * M + 64, np.uint32)
        args = [vp(np.ascontiguousarray(x)) for x in (w.pos, w.world, w.sender, w.repl)]
        P = f(o.h, *args, M, vp(connected), len(connected), vp(fo), vp(fp), len(fp))
        cs = set(connected.tolist())
        rank = {p: i for i, p in enumerate(connected.tolist())}
        for m in range(M):
            want = sorted((p for p in peers[offs[m]:offs[m + 1]].tolist() if p in cs), key=rank.get)
            assert fp[fo[m]:fo[m + 1]].tolist() == want, m
        assert fo[M] == P
    o.close()


def test_fast_mode_matches_faithful_scan():
    """wqo_set_fast (the checker mode of the full-size churn tests) answers remove_subscription's
    O(#cubes) scan (area_map.rs:113-116) from per-peer cube counts: identical sets on a churn-heavy
    op stream with duplicate / absent unsubscribes and REMOVE_PEER, world by world."""
    from worldql_server_amd import abi
    rng = np.random.default_rng(3)
    n = 20000
    kinds = rng.choice(3, n, p=[0.5, 0.45, 0.05]).astype(np.uint8)
    world = rng.integers(0, 3, n).astype(np.uint32)
    peer = rng.integers(0, 50, n).astype(np.uint32)
    world[kinds == abi.OP_REMOVE_PEER] = np.where(rng.random(int((kinds == 2).sum())) < 0.5, 0xFFFFFFFF, 1)
    pos = rng.uniform(-40, 40, (n, 3))
    ops = abi.ops_array(world, peer, kinds, pos=pos)
    a, b = orc.COracle(16), orc.COracle(16)
    b.set_fast(True)
    for lo in range(0, n, 1000):
        a.apply_ops(ops[lo:lo + 1000])
        b.apply_ops(ops[lo:lo + 1000])
        assert a.counts() == b.counts()
        for w in range(3):
            assert (a.world_peers(w) == b.world_peers(w)).all()
            for p in range(0, 50, 7):
                assert a.is_subscribed_any(w, p) == b.is_subscribed_any(w, p)
    with pytest.raises(ValueError):
        b.set_fast(False)  # only on an empty map
