"""GPU parity for the configurations past C2: C3 hotspot skew, C4 world churn,
C5 exact radius filter — the HIP path through the C ABI against the C restatement (oracle/).

Bar: bit-exact per message (recipients compared as ascending peer lists). The radius predicate is
f64, left to right, no FMA on both sides; C5 is an extension the reference lacks (it stores no
peer positions), so its results are pinned to the restatement only.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth, synth_ext

pytestmark = pytest.mark.gpu


def mk_router(cube_size=16):
    from worldql_server_amd.router import Router
    return Router(cube_size, 0)


def _same(got, want):
    offs, peers = got[0], got[1]
    o_offs, o_peers = want[0], want[1]
    assert (offs == o_offs).all()
    assert (peers == o_peers).all()
    return len(peers)


# ---- C5: radius ------------------------------------------------------------------------------

def test_c5_radius_scaled_vs_oracle():
    c5 = synth_ext.config_c5(scale=0.004)
    ops = c5.initial_ops()
    r, o = mk_router(), orc.COracle(16)
    r.apply_ops(ops)
    o.apply_ops(ops)
    r.set_peer_positions(c5.pos)
    r.set_radius(c5.radius)
    for tick in range(3):
        pos, w, s, _ = c5.messages()
        rp = synth.stream(5, 50 + tick).below(3, len(w)).astype(np.uint8)
        P = _same(r.route(pos, w, s, rp), o.route_radius(pos, w, s, rp, c5.pos, c5.radius))
        assert P > 0
        ops = c5.step()
        r.apply_ops(ops)
        o.apply_ops(ops)
        r.set_peer_positions(c5.pos)
    # the filter off again: plain broadphase
    r.set_radius(0.0)
    pos, w, s, rp = c5.messages()
    _same(r.route(pos, w, s, rp), o.route(pos, w, s, rp))


def test_radius_unknown_replication_codes():
    """Every replication code, unknown ones included (replication.rs:34-43: ExceptSelf), through the
    radius filter's inline-mask and long-list paths. Codes >= 3 once lost their recipients in the
    inline path (a miscompiled switch in repl_keeps, route_emit.hpp)."""
    c5 = synth_ext.config_c5(scale=0.004)
    ops = c5.initial_ops()
    r, o = mk_router(), orc.COracle(16)
    r.apply_ops(ops)
    o.apply_ops(ops)
    # a dense cluster on top: lists longer than the 24 inline peers
    rng = np.random.default_rng(5)
    n0 = len(c5.pos)
    centre = rng.normal(0.0, 6.0, (200, 3))
    nb = np.array([[dx, dy, dz] for dx in (-1, 0, 1) for dy in (-1, 0, 1) for dz in (-1, 0, 1)], np.float64)
    sub = (centre[:, None, :] + 16.0 * nb[None]).reshape(-1, 3)
    extra = abi.ops_array(np.zeros(len(sub), np.uint32), np.repeat(np.arange(n0, n0 + 200, dtype=np.uint32), 27),
                          np.zeros(len(sub), np.uint8), pos=sub)
    r.apply_ops(extra)
    o.apply_ops(extra)
    pp = np.concatenate([c5.pos, centre + rng.uniform(-4.0, 4.0, centre.shape)])
    r.set_peer_positions(pp)
    r.set_radius(c5.radius)
    pos, w, s, _ = c5.messages()
    M = len(w)
    pos = np.concatenate([pos, centre[rng.integers(0, 200, 2000)] + rng.uniform(-8, 8, (2000, 3))])
    s = np.concatenate([s, rng.integers(0, n0 + 200, 2000).astype(np.uint32)])
    w = np.zeros(len(s), np.uint32)
    for codes in ((0, 1, 2, 3), (3, 4, 255)):
        rp = np.array(codes, np.uint8)[rng.integers(0, len(codes), len(s))]
        P = _same(r.route(pos, w, s, rp), o.route_radius(pos, w, s, rp, pp, c5.radius))
        assert P > 0
    assert M > 0


def test_radius_boundary_long_lists_and_missing_positions():
    r, o = mk_router(), orc.COracle(16)
    rng = synth.SplitMix64(99)
    # cube (16,16,16) holds 60 peers (a long list), cube (32,16,16) holds 10 (inline)
    n_long, n_short = 60, 10
    peer = np.arange(n_long + n_short, dtype=np.uint32)
    sub = np.concatenate([np.full((n_long, 3), 8.0), np.tile([[24.0, 8.0, 8.0]], (n_short, 1))])
    ops = abi.ops_array(np.zeros(len(peer), np.uint32), peer, np.zeros(len(peer), np.uint8), pos=sub)
    r.apply_ops(ops)
    o.apply_ops(ops)
    radius = 5.0
    # peer positions: some exactly at distance r from (8, 8, 8), some a hair beyond, one NaN;
    # peers 66..69 have no position at all (n_pos = 66)
    pp = rng.uniform(0.0, 16.0, 3 * 66).reshape(66, 3)
    pp[0] = [13.0, 8.0, 8.0]                       # d2 == r2 exactly: kept
    pp[1] = [np.nextafter(13.0, 20.0), 8.0, 8.0]   # just outside: dropped
    pp[2] = [8.0, 8.0, 8.0 - 5.0]                  # exact, other axis
    pp[3] = [np.nan, 8.0, 8.0]
    pp[60] = [27.0, 8.0, 8.0]                      # inline cube, d2 == r2 from (24, 8, 8)
    r.set_peer_positions(pp)
    r.set_radius(radius)
    M = 400
    mpos = np.where((np.arange(M) % 2 == 0)[:, None], [[8.0, 8.0, 8.0]], [[24.0, 8.0, 8.0]])
    mpos = mpos + np.where((np.arange(M) % 5 == 0)[:, None], rng.uniform(-3, 3, 3 * M).reshape(M, 3), 0.0)
    sender = rng.below(n_long + n_short, M)
    repl = rng.below(3, M).astype(np.uint8)
    got = r.route(mpos, np.zeros(M, np.uint32), sender, repl)
    want = o.route_radius(mpos, np.zeros(M, np.uint32), sender, repl, pp, radius)
    P = _same(got, want)
    assert P > 0
    # an IncludingSelf message exactly at (8, 8, 8): peers 0 and 2 sit exactly on the sphere
    m = next(i for i in range(M) if i % 2 == 0 and i % 5 and repl[i] == abi.REPL_INCLUDING_SELF)
    seg = got[1][got[0][m]:got[0][m + 1]]
    assert 0 in seg and 2 in seg and 1 not in seg and 3 not in seg


def test_radius_f32_first_test_edges():
    """within_radius decides from an f32 copy of the peer positions when the f64 result is certain
    and reads the f64 coordinates otherwise: peers on the sphere to a few ulps (the deferred case),
    coordinates where f32 has an ulp of 1 (1e7), beyond f32 (1e39 -> inf), subnormals, +-inf and NaN,
    a radius that is not representable, for a long list (60 peers) and an inline cube (20 peers)."""
    r, o = mk_router(), orc.COracle(16)
    rng = synth.SplitMix64(7)
    n_a, n_b = 60, 20
    centre_a, centre_b = np.array([8.1, 7.3, 9.7]), np.array([1e7 + 8.3, 8.2, -7.9])
    peer = np.arange(n_a + n_b, dtype=np.uint32)
    sub = np.concatenate([np.tile(centre_a, (n_a, 1)), np.tile(centre_b, (n_b, 1))])
    ops = abi.ops_array(np.zeros(len(peer), np.uint32), peer, np.zeros(len(peer), np.uint8), pos=sub)
    r.apply_ops(ops)
    o.apply_ops(ops)
    radius = 5.1
    u = rng.uniform(-1.0, 1.0, 3 * (n_a + n_b)).reshape(-1, 3)
    u /= np.linalg.norm(u, axis=1)[:, None]
    k = (np.arange(n_a + n_b) % 9 - 4).astype(np.float64)  # -4 .. 4 ulps around the sphere
    d = radius * (1.0 + k * 2.0 ** -52)
    pp = np.concatenate([centre_a + d[:n_a, None] * u[:n_a], centre_b + d[n_a:, None] * u[n_a:]])
    pp[50] = [1e39, 8.0, 8.0]        # beyond f32: inf in the copy
    pp[51] = [5e-310, 7.0, 9.0]      # subnormal in f64, 0 in f32
    pp[52] = [np.inf, 7.0, 9.0]
    pp[53] = [-np.inf, 7.0, 9.0]
    pp[54] = [np.nan, 7.0, 9.0]
    pp[55] = centre_a                # distance 0
    pp[56] = centre_a + [radius, 0.0, 0.0]
    r.set_peer_positions(pp)
    r.set_radius(radius)
    M = 300
    mpos = np.where((np.arange(M) % 2 == 0)[:, None], centre_a[None, :], centre_b[None, :])
    jit = np.where((np.arange(M) % 3 == 0)[:, None], rng.uniform(-1e-9, 1e-9, 3 * M).reshape(M, 3), 0.0)
    mpos = mpos + jit * np.abs(mpos)
    sender = rng.below(n_a + n_b, M)
    repl = rng.below(3, M).astype(np.uint8)
    got = r.route(mpos, np.zeros(M, np.uint32), sender, repl)
    want = o.route_radius(mpos, np.zeros(M, np.uint32), sender, repl, pp, radius)
    assert _same(got, want) > 0


def test_radius_needs_positions():
    from worldql_server_amd.router import WQError
    r = mk_router()
    r.apply_ops(abi.ops_array(np.zeros(1, np.uint32), [0], [0], pos=np.ones((1, 3))))
    r.set_peer_positions(np.ones((1, 3)))
    r.set_radius(4.0)
    with pytest.raises(WQError) as e:
        r.route(None, np.zeros(1, np.uint32), np.zeros(1, np.uint32), np.zeros(1, np.uint8),
                keys=np.array([[16, 16, 16]]))
    assert e.value.code == abi.WQ_E_INVALID


# ---- C3: hotspot skew ------------------------------------------------------------------------

def test_c3_hotspots_scaled_vs_oracle():
    """Heavy, skewed fan-out: most messages land in long lists (> kInline peers)."""
    w = synth_ext.config_c3(scale=0.003)
    r, o = mk_router(), orc.COracle(16)
    r.apply_ops(w.ops)
    o.apply_ops(w.ops)
    assert r.stats()["n_entries"] == o.counts()[0]
    repl = synth.stream(3, 9).below(3, len(w.world)).astype(np.uint8)
    got = r.route(w.pos, w.world, w.sender, repl)
    want = o.route(w.pos, w.world, w.sender, repl)
    P = _same(got, want)
    assert P > 10 * len(w.world)  # the hotspots make the mean fan-out large
    for cfg in range(r.route_config_count()):
        r.set_route_config(cfg)
        _same(r.route(w.pos, w.world, w.sender, repl), want)


# ---- C4: world churn -------------------------------------------------------------------------

def test_c4_churn_ticks_vs_oracle():
    c4 = synth_ext.config_c4(scale=0.01, worlds=range(0, 64, 4))
    r, o = mk_router(), orc.COracle(16)
    ops = c4.initial_ops()
    r.apply_ops(ops)
    o.apply_ops(ops)
    for tick in range(4):
        ops, pos, w, s, rp = c4.step()
        r.apply_ops(ops)
        o.apply_ops(ops)
        assert r.stats()["n_entries"] == o.counts()[0]
        P = _same(r.route(pos, w, s, rp), o.route(pos, w, s, rp))
        assert P > 0
    for wid in (0, 4, 60):
        assert (r.world_peers(wid) == o.world_peers(wid)).all()


def test_radius_position_code_edges():
    """The first radius test reads a 4-byte code per peer (x, y on 11 bits, z on 10, over the
    positions' bounding box) and decides only when the reference's f64 result is certain; the
    rest go to the f32 and f64 tests. Peers in a 64-unit box (steps of ~0.03 / 0.06) at distances
    straddling the code's uncertainty band and the exact sphere, on a long list and an inline cube,
    every replication mode; then the same peers in a 1e6-unit box (steps ~500: every code defers)."""
    rng = synth.SplitMix64(41)
    n_a, n_b = 70, 22
    centre_a, centre_b = np.array([3.3, -2.1, 5.7]), np.array([-20.5, 14.25, -9.0])
    peer = np.arange(n_a + n_b, dtype=np.uint32)
    sub = np.concatenate([np.tile(centre_a, (n_a, 1)), np.tile(centre_b, (n_b, 1))])
    ops = abi.ops_array(np.zeros(len(peer), np.uint32), peer, np.zeros(len(peer), np.uint8), pos=sub)
    radius = 5.0
    u = rng.uniform(-1.0, 1.0, 3 * (n_a + n_b)).reshape(-1, 3)
    u /= np.linalg.norm(u, axis=1)[:, None]
    d = radius + rng.uniform(-0.12, 0.12, n_a + n_b)   # across the code's band (~0.05 wide here)
    d[::7] = radius                                     # on the sphere (to rounding)
    pp = np.concatenate([centre_a + d[:n_a, None] * u[:n_a], centre_b + d[n_a:, None] * u[n_a:]])
    pp[3] = centre_a + [radius, 0.0, 0.0]               # d2 == r2 exactly
    pp[4] = centre_a + [0.0, 0.0, -radius]
    pp[5] = [np.nan, 1.0, 1.0]                          # no code: the f32 / f64 tests decide
    pp[6] = [32.0, 32.0, -32.0]                         # a box corner
    pp[7] = [-32.0, -32.0, 32.0]
    M = 400
    mpos = np.where((np.arange(M) % 2 == 0)[:, None], centre_a[None, :], centre_b[None, :])
    mpos = mpos + np.where((np.arange(M) % 3 == 0)[:, None], rng.uniform(-0.5, 0.5, 3 * M).reshape(M, 3), 0.0)
    sender = rng.below(n_a + n_b, M)
    repl = rng.below(3, M).astype(np.uint8)
    for scale in (1.0, 1e6):
        q = pp.copy()
        if scale != 1.0:
            q[8] = [scale, -scale, scale]  # a far peer widens the box: every code step ~500 units
        r, o = mk_router(), orc.COracle(16)
        r.apply_ops(ops)
        o.apply_ops(ops)
        r.set_peer_positions(q)
        r.set_radius(radius)
        got = r.route(mpos, np.zeros(M, np.uint32), sender, repl)
        want = o.route_radius(mpos, np.zeros(M, np.uint32), sender, repl, q, radius)
        assert _same(got, want) > 0
        r.close()
