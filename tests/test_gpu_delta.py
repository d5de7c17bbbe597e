"""GPU parity for incremental table updates (wq_delta.hip, SURVEY.md §8(d) C4 churn): small op
batches against a built table are applied in place; every tick is compared with the C
restatement (oracle/) — routing CSR, membership queries, any-sets and counts — and the tests
check that the incremental path (not the rebuild) is the one that ran."""
import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth, synth_ext

pytestmark = pytest.mark.gpu


def mk_router(cube_size=16, hash_bits=64):
    from worldql_server_amd.router import Router
    return Router(cube_size, 0, hash_bits=hash_bits)


def _check(r, o, pos, world, sender, repl):
    got = r.route(pos, world, sender, repl)
    want = o.route(pos, world, sender, repl)
    assert (got[0] == want[0]).all()
    assert (got[1] == want[1]).all()
    st = r.stats()
    e, c = o.counts()
    assert st["n_entries"] == e and st["n_cubes"] == c
    return len(got[1])


def _random_ops(rng, n, worlds, peers, half, sub_frac):
    return abi.ops_array(rng.integers(0, worlds, n).astype(np.uint32), rng.integers(0, peers, n).astype(np.uint32),
                         np.where(rng.random(n) < sub_frac, abi.OP_SUBSCRIBE, abi.OP_UNSUBSCRIBE).astype(np.uint8),
                         pos=rng.uniform(-half, half, (n, 3)))


@pytest.mark.parametrize("hash_bits,f", [(64, 1.0), (6, 0.05)])
def test_delta_random_churn_vs_oracle(hash_bits, f):
    """Random sub / unsub batches (duplicates, unsubs of absent triples, new and emptied cubes,
    lists that outgrow their capacity) — incremental every tick. hash_bits 6 puts every record
    on one probe sequence (f scales the sizes down for it)."""
    rng = np.random.default_rng(5 + hash_bits)
    r, o = mk_router(hash_bits=hash_bits), orc.COracle(16)
    half = 160.0 * f ** (1 / 3)
    base = _random_ops(rng, int(60000 * f), 3, 4000, half, 1.0)
    r.apply_ops(base)
    o.apply_ops(base)
    M = 4000
    for tick in range(8):
        # concentrated batches: a few hot cubes gain many peers (relocation), others churn
        ops = _random_ops(rng, int(4000 * f), 3, 4500, half, 0.55)
        nh = int(600 * f) if tick % 2 else 0  # odd ticks: one new hot cube (a lane merges 600 ops)
        hot = abi.ops_array(np.zeros(nh, np.uint32), rng.integers(0, 4500, nh).astype(np.uint32),
                            np.zeros(nh, np.uint8), pos=np.tile([[8.0 + 16 * tick, 8.0, 8.0]], (nh, 1)))
        if tick % 2 == 0 and tick:  # even ticks: churn on the previous tick's hot cube (wave path)
            nw = int(300 * f)
            warm = abi.ops_array(np.zeros(nw, np.uint32), rng.integers(0, 4500, nw).astype(np.uint32),
                                 rng.integers(0, 2, nw).astype(np.uint8),
                                 pos=np.tile([[8.0 + 16 * (tick - 1), 8.0, 8.0]], (nw, 1)))
            hot = abi.concat_ops([hot, warm])
        # re-issue some ops of this batch in reverse kind: last op wins per triple
        nf = int(500 * f)
        flip = ops[:nf].copy()
        flip["kind"] = 1 - flip["kind"]
        batch = abi.concat_ops([ops, hot, flip, ops[nf // 2:nf]])
        r.apply_ops(batch)
        o.apply_ops(batch)
        pos = rng.uniform(-half - 10, half + 10, (M, 3))
        pos[:200] = [8.0 + 16 * tick, 8.0, 8.0]
        world = rng.integers(0, 4, M).astype(np.uint32)
        sender = rng.integers(0, 4500, M).astype(np.uint32)
        repl = rng.integers(0, 3, M).astype(np.uint8)
        assert _check(r, o, pos, world, sender, repl) > 0
    inc, fb, wave = r.update_counts(lanes=True)
    assert inc == 8 and fb == 0 and (wave >= 3 or f < 1)  # ticks touching an old hot cube: its list > kLaneList
    # membership and any-sets after churn (regenerated from the records)
    for w in range(4):
        assert (r.world_peers(w) == o.world_peers(w)).all()
    q = 3000
    qw = rng.integers(0, 3, q).astype(np.uint32)
    qp = rng.integers(0, 4500, q).astype(np.uint32)
    qpos = rng.uniform(-half, half, (q, 3))
    got = r.is_subscribed(qw, qp, False, qpos)
    want = np.array([o.is_subscribed(int(a), int(b), False, c) for a, b, c in zip(qw, qp, qpos)])
    assert (got == want).all()
    got = r.is_subscribed_any(qw, qp)
    want = np.array([o.is_subscribed_any(int(a), int(b)) for a, b in zip(qw, qp)])
    assert (got == want).all()


def test_delta_empty_and_revive_cubes():
    """Cubes emptied by a batch keep a count-0 record; later batches revive them in place."""
    r, o = mk_router(), orc.COracle(16)
    peers = np.arange(4000, dtype=np.uint32)
    cells = (peers % 200).astype(np.float64) * 16.0 + 8.0
    pos = np.stack([cells, np.full(4000, 8.0), np.full(4000, 8.0)], 1)
    base = abi.ops_array(np.zeros(4000, np.uint32), peers, np.zeros(4000, np.uint8), pos=pos)
    r.apply_ops(base)
    o.apply_ops(base)
    mpos = np.stack([np.arange(200) * 16.0 + 8.0, np.full(200, 8.0), np.full(200, 8.0)], 1)
    zeros = np.zeros(200, np.uint32)
    sel = np.isin(peers % 200, np.arange(0, 200, 2))[:800]  # empty the even cells among peers < 800
    for kind in (abi.OP_UNSUBSCRIBE, abi.OP_SUBSCRIBE):
        b = abi.ops_array(np.zeros(800, np.uint32), peers[:800], np.full(800, kind, np.uint8), pos=pos[:800])
        r.apply_ops(b)
        o.apply_ops(b)
        _check(r, o, mpos, zeros, np.arange(200, dtype=np.uint32), np.ones(200, np.uint8))
    assert sel.any()
    assert r.update_counts() == (2, 0)


def test_delta_row_and_wave_path_edges():
    """Cubes built at sizes around the bucket apply's limits (24 inline peers, 64-cube / 1,024-word
    rounds, lists past kLaneList for the wave path) get batches that grow them past 24, shrink them
    below 24, empty them, keep an inline cube inline under many ops, and put many ops on one cube;
    every tick is checked against the oracle and must stay incremental."""
    rng = np.random.default_rng(77)
    r, o = mk_router(), orc.COracle(16)
    sizes = [0, 1, 10, 20, 23, 24, 25, 30, 40, 50, 60, 63, 64, 65, 100, 300]
    cells = np.array([[16.0 * i + 8.0, 8.0, 8.0] for i in range(len(sizes))])
    w, p, ps = [], [], []
    for i, n in enumerate(sizes):
        pe = rng.choice(5000, n, replace=False).astype(np.uint32)
        p.append(pe)
        ps.append(np.tile(cells[i], (n, 1)))
    allp = np.concatenate(p)
    base = abi.ops_array(np.zeros(len(allp), np.uint32), allp, np.zeros(len(allp), np.uint8),
                         pos=np.concatenate(ps))
    r.apply_ops(base)
    o.apply_ops(base)
    # a filler table so a later batch stays incremental (a batch must be <= 1/4 of the table)
    fill = _random_ops(rng, 60000, 2, 6000, 400.0, 1.0)
    fill["world"] += 1
    r.apply_ops(fill)
    o.apply_ops(fill)
    mpos = np.repeat(cells, 4, 0)
    M = len(mpos)
    for tick in range(6):
        parts = []
        for i, n in enumerate(sizes):
            k = [0, 3, 12, 40, 41, 1, 4, 80, 24, 14, 4, 1, 0, 2, 30, 10][i] + tick
            kinds = rng.integers(0, 2, k).astype(np.uint8)
            if tick == 2 and i in (3, 7):   # empty two cubes completely
                cur = o.route(cells[i:i + 1], np.zeros(1, np.uint32), np.zeros(1, np.uint32),
                              np.ones(1, np.uint8))[1]
                pe = cur.astype(np.uint32)
                kinds = np.ones(len(pe), np.uint8)
            else:
                pe = np.concatenate([rng.choice(p[i], min(len(p[i]), k // 2)) if len(p[i]) else
                                     np.zeros(0, np.uint32),
                                     rng.integers(5000, 5200, k - min(len(p[i]), k // 2))]).astype(np.uint32)
                rng.shuffle(pe)
            parts.append(abi.ops_array(np.zeros(len(pe), np.uint32), pe, kinds[:len(pe)],
                                       pos=np.tile(cells[i], (len(pe), 1))))
        batch = abi.concat_ops(parts)
        r.apply_ops(batch)
        o.apply_ops(batch)
        _check(r, o, mpos, np.zeros(M, np.uint32), rng.integers(0, 5200, M).astype(np.uint32),
               np.tile(np.array([0, 1, 2, 1], np.uint8), M // 4))
    assert r.update_counts()[1] == 0


def test_delta_fallbacks_and_remove_peer():
    """An irregular key in a small batch takes the rebuild; REMOVE_PEER after incremental
    batches works from the regenerated state."""
    rng = np.random.default_rng(9)
    r, o = mk_router(), orc.COracle(16)
    base = _random_ops(rng, 40000, 2, 3000, 128.0, 1.0)
    r.apply_ops(base)
    o.apply_ops(base)
    M = 3000
    args = lambda: (rng.uniform(-130, 130, (M, 3)), rng.integers(0, 2, M).astype(np.uint32),
                    rng.integers(0, 3000, M).astype(np.uint32), rng.integers(0, 3, M).astype(np.uint8))
    b = _random_ops(rng, 2000, 2, 3000, 128.0, 0.5)
    r.apply_ops(b)
    o.apply_ops(b)
    _check(r, o, *args())
    assert r.update_counts() == (1, 0)
    # a raw off-grid key (not a multiple of the cube size) has no packed key: full rebuild
    raw = abi.ops_array(np.zeros(3, np.uint32), np.array([1, 2, 3], np.uint32), np.zeros(3, np.uint8),
                        key=np.array([[1, 2, 3], [16, 16, 17], [0, 0, 0]]))
    b = abi.concat_ops([_random_ops(rng, 500, 2, 3000, 128.0, 0.5), raw])
    r.apply_ops(b)
    o.apply_ops(b)
    _check(r, o, *args())
    assert r.update_counts() == (1, 1)
    # incremental again (the table now also holds full-key slot cubes), then REMOVE_PEER
    b = _random_ops(rng, 1500, 2, 3000, 128.0, 0.5)
    r.apply_ops(b)
    o.apply_ops(b)
    _check(r, o, *args())
    assert r.update_counts() == (2, 1)
    rm = abi.ops_array(np.full(40, abi.WORLD_INVALID, np.uint32), np.arange(0, 400, 10, dtype=np.uint32),
                       np.full(40, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((40, 3)))
    r.apply_ops(rm)
    o.apply_ops(rm)
    _check(r, o, *args())
    assert r.is_subscribed(np.zeros(1, np.uint32), np.array([1], np.uint32), True, np.array([[1, 2, 3]]))[0] == \
        o.is_subscribed(0, 1, True, np.array([1, 2, 3]))


def test_delta_list_space_exhaustion_rebuilds():
    """Repeated growth of the same cubes relocates their lists until `list` runs out of room; the
    batch that would overflow takes the rebuild, which compacts, and results stay exact."""
    rng = np.random.default_rng(13)
    r, o = mk_router(), orc.COracle(16)
    base = _random_ops(rng, 30000, 1, 30000, 64.0, 1.0)
    r.apply_ops(base)
    o.apply_ops(base)
    M = 2000
    nxt = 30000
    for tick in range(40):
        n = 1500
        peers = np.arange(nxt, nxt + n, dtype=np.uint32)
        nxt += n
        b = abi.ops_array(np.zeros(n, np.uint32), peers, np.zeros(n, np.uint8),
                          pos=np.tile([[8.0, 8.0, 8.0], [24.0, 8.0, 8.0], [40.0, 8.0, 8.0]], (n // 3, 1)))
        r.apply_ops(b)
        o.apply_ops(b)
        if tick % 8 == 7:
            pos = rng.uniform(-64, 64, (M, 3))
            pos[:30] = [8.0, 8.0, 8.0]
            _check(r, o, pos, np.zeros(M, np.uint32), rng.integers(0, nxt, M).astype(np.uint32),
                   rng.integers(0, 3, M).astype(np.uint8))
    inc, fb = r.update_counts()
    assert inc > 20 and fb >= 1


def test_c4_scaled_churn_is_incremental():
    c4 = synth_ext.config_c4(scale=0.02, worlds=range(0, 64, 8))
    r, o = mk_router(), orc.COracle(16)
    ops = c4.initial_ops()
    r.apply_ops(ops)
    o.apply_ops(ops)
    for _ in range(5):
        ops, pos, w, s, rp = c4.step()
        r.apply_ops(ops)
        o.apply_ops(ops)
        rp = synth.stream(4, 3).below(3, len(w)).astype(np.uint8)
        assert _check(r, o, pos, w, s, rp) > 0
    assert r.update_counts() == (5, 0)  # C4 churn: incremental throughout
    for wid in (0, 8, 56):
        assert (r.world_peers(wid) == o.world_peers(wid)).all()


@pytest.mark.parametrize("hash_bits", [64, 6])
def test_remove_peers_in_place_vs_oracle(hash_bits):
    """WorldMap::remove_peer / AreaMap::remove_peer batches applied in place on every list
    (every-world and one-world removals, long lists, full-key slot cubes), interleaved with
    incremental churn; the table then keeps routing and answering queries exactly."""
    rng = np.random.default_rng(21 + hash_bits)
    f = 1.0 if hash_bits == 64 else 0.05
    r, o = mk_router(hash_bits=hash_bits), orc.COracle(16)
    half = 96.0 * f ** (1 / 3)
    n_peers = 3000
    base = _random_ops(rng, int(40000 * f), 3, n_peers, half, 1.0)
    hot = abi.ops_array(np.zeros(400, np.uint32), np.arange(400, dtype=np.uint32), np.zeros(400, np.uint8),
                        pos=np.tile([[8.0, 8.0, 8.0]], (400, 1)))  # a 400-peer list
    raw = abi.ops_array(np.ones(60, np.uint32), rng.integers(0, n_peers, 60).astype(np.uint32),
                        np.zeros(60, np.uint8), key=rng.integers(-4, 4, (60, 3)) * 3)  # off-grid: slot table
    ops = abi.concat_ops([base, hot, raw])
    r.apply_ops(ops)
    o.apply_ops(ops)
    M = 3000

    def check():
        pos = rng.uniform(-half - 8, half + 8, (M, 3))
        pos[:100] = [8.0, 8.0, 8.0]
        world = rng.integers(0, 3, M).astype(np.uint32)
        sender = rng.integers(0, n_peers, M).astype(np.uint32)
        repl = rng.integers(0, 3, M).astype(np.uint8)
        _check(r, o, pos, world, sender, repl)
        keys = rng.integers(-4, 4, (200, 3)) * 3
        kw = np.ones(200, np.uint32)
        kp = rng.integers(0, n_peers, 200).astype(np.uint32)
        got = r.is_subscribed(kw, kp, True, keys)
        assert (got == np.array([o.is_subscribed(1, int(p), True, k) for p, k in zip(kp, keys)])).all()
        for w in range(3):
            assert (r.world_peers(w) == o.world_peers(w)).all()

    for t in range(3):
        gone = rng.choice(n_peers, 150, replace=False).astype(np.uint32)
        r.remove_peers(gone)          # every world
        o.apply_ops(abi.ops_array(np.full(150, abi.WORLD_INVALID, np.uint32), gone,
                                  np.full(150, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((150, 3))))
        one = abi.ops_array(np.full(80, t % 3, np.uint32), rng.choice(n_peers, 80, replace=False).astype(np.uint32),
                            np.full(80, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((80, 3)))  # one world
        churn = _random_ops(rng, int(2000 * f), 3, n_peers, half, 0.6)
        b = abi.concat_ops([one, churn])
        r.apply_ops(b)
        o.apply_ops(b)
        check()
    inc, fb = r.update_counts()
    assert inc == 3 and fb == 0  # the churn after each removal stays incremental


def test_device_batch_without_packed_key_is_reapplied():
    """wq_apply_ops_device returns without waiting for the GPU. A batch with an op that has no
    packed key (an off-grid raw key) cannot be applied by the incremental kernels: a tick issued
    right after it is either exact (the handle already folded the batch in) or flagged with error
    bit 8; the next call re-applies the batch through the rebuild, and from then on every tick is
    exact again."""
    import torch
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(31)
    r, o = mk_router(), orc.COracle(16)
    r.set_stream(torch.cuda.current_stream().cuda_stream)
    base = _random_ops(rng, 40000, 2, 3000, 128.0, 1.0)
    r.apply_ops(base)
    o.apply_ops(base)
    raw = abi.ops_array(np.zeros(2, np.uint32), np.array([5, 6], np.uint32), np.zeros(2, np.uint8),
                        key=np.array([[16, 16, 17], [3, 0, 0]]))
    b = abi.concat_ops([_random_ops(rng, 1500, 2, 3000, 128.0, 0.5), raw])
    d_ops = torch.from_numpy(np.ascontiguousarray(b).view(np.uint8).copy()).to(dev)
    r.apply_ops_device(d_ops.data_ptr(), len(b))
    o.apply_ops(b)
    M = 3000
    pos = rng.uniform(-130, 130, (M, 3))
    world = rng.integers(0, 2, M).astype(np.uint32)
    sender = rng.integers(0, 3000, M).astype(np.uint32)
    repl = rng.integers(0, 3, M).astype(np.uint8)
    t_pos = torch.from_numpy(pos).to(dev)
    t_w = torch.from_numpy(world.view(np.int32)).to(dev)
    t_s = torch.from_numpy(sender.view(np.int32)).to(dev)
    t_r = torch.from_numpy(repl).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 64 * M
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    r.route_device(t_pos.data_ptr(), t_w.data_ptr(), t_s.data_ptr(), t_r.data_ptr(), M, offs.data_ptr(),
                   peers.data_ptr(), None, cap, cnt.data_ptr())
    torch.cuda.synchronize(dev)
    err = int(cnt.cpu().numpy()[20:24].view(np.uint32)[0])
    want = o.route(pos, world, sender, repl)
    if err == 0:  # the batch had been folded in (re-applied) before the tick
        got_offs = offs.cpu().numpy().view(np.uint32)
        assert (got_offs == want[0]).all()
        assert (peers.cpu().numpy().view(np.uint32)[: got_offs[-1]] == want[1]).all()
    else:
        assert err == 8
    inc, fb = r.update_counts()  # folds the batch in: re-applied through the rebuild
    assert fb == 1
    r.route_health()  # clear the sticky bits of the flagged tick, if any
    _check(r, o, pos, world, sender, repl)
    assert r.route_health() == (0, 0)
    del d_ops


def test_invalid_device_batch_does_not_drop_the_next_call():
    """A device batch holding an invalid op (REMOVE_PEER kind) is not applied; the next call on the
    handle — a valid host batch here — still does its own work, and the rejection shows as error
    bit 16 of wq_route_health."""
    import torch
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(37)
    r, o = mk_router(), orc.COracle(16)
    r.set_stream(torch.cuda.current_stream().cuda_stream)
    base = _random_ops(rng, 40000, 2, 3000, 128.0, 1.0)
    r.apply_ops(base)
    o.apply_ops(base)
    bad = abi.concat_ops([_random_ops(rng, 500, 2, 3000, 128.0, 1.0),
                          abi.ops_array(np.zeros(1, np.uint32), np.array([9], np.uint32),
                                        np.full(1, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((1, 3)))])
    d_ops = torch.from_numpy(np.ascontiguousarray(bad).view(np.uint8).copy()).to(dev)
    r.apply_ops_device(d_ops.data_ptr(), len(bad))  # rejected on the device: nothing of it applies
    good = _random_ops(rng, 800, 2, 3000, 128.0, 1.0)
    r.apply_ops(good)  # folds the rejected batch in, then applies its own ops in full
    o.apply_ops(good)
    got = r.is_subscribed(good["world"], good["peer"], False, good["pos"])
    want = np.array([o.is_subscribed(int(x["world"]), int(x["peer"]), False, x["pos"]) for x in good])
    assert (got == want).all() and got.any()
    assert r.stats()["n_entries"] == o.counts()[0]
    e, _ = r.route_health()
    assert e & 16
    M = 2000
    pos = rng.uniform(-130, 130, (M, 3))
    world = rng.integers(0, 2, M).astype(np.uint32)
    sender = rng.integers(0, 3000, M).astype(np.uint32)
    repl = rng.integers(0, 3, M).astype(np.uint8)
    _check(r, o, pos, world, sender, repl)
    assert r.route_health() == (0, 0)
    del d_ops
