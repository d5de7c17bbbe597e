"""CPU: host-side logic — world names, synthetic generator, the C ABI's exported symbols and
record layouts, the host instance of the quantiser, and tick batching (flush-on-reorder)."""
import ctypes
import glob
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth
from worldql_server_amd.world_names import SanitizeError, WorldIds, sanitize_world_name

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sanitize_kats(kats):
    """world_names.rs:127-171."""
    for raw, want in kats["sanitize_ok"]:
        assert sanitize_world_name(raw) == want
    for raw, kind in kats["sanitize_err"]:
        with pytest.raises(SanitizeError) as e:
            sanitize_world_name(raw)
        assert e.value.kind == kind


def test_world_ids_collapse_sanitized_names():
    ids = WorldIds()
    a = ids.intern(sanitize_world_name("a b"))
    b = ids.intern(sanitize_world_name("a_b"))
    assert a == b and len(ids) == 1


def test_splitmix64_known_values():
    # reference splitmix64 (seed 0): first outputs
    r = synth.SplitMix64(0)
    assert [int(v) for v in r.next_u64(3)] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]
    u = synth.SplitMix64(7).uniform(-1.0, 1.0, 1000)
    assert u.min() >= -1.0 and u.max() < 1.0


def test_config_shapes():
    w = synth.config_c1()
    assert len(w.ops) == 1000 and w.pos.shape == (10_000, 3)
    w2 = synth.config_c2(scale=0.01)
    assert len(w2.ops) == 27 * 1000 and w2.pos.shape == (10_000, 3)


def _header_functions():
    names = set()
    for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))):  # wq_router.h, wq_codec.h
        with open(h) as f:
            txt = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
        names |= set(re.findall(r"\b(wq_[a-z0-9_]+)\s*\(", txt))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    from worldql_server_amd.build import LIB
    if not os.path.exists(LIB):
        from worldql_server_amd.build import build
        build()
    lib = ctypes.CDLL(LIB)  # loading needs no GPU; nothing below computes
    names = _header_functions()
    assert "wq_route_tick_device" in names and "wq_decode_messages" in names and len(names) >= 19
    for n in names:
        assert hasattr(lib, n), n


def test_product_does_not_reference_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "worldql_server_amd")):
        for fn in files:
            if fn.endswith((".py", ".hip", ".hpp", ".h", ".cpp")):
                with open(os.path.join(dirpath, fn)) as f:
                    src = f.read()
                assert "oracle" not in src.replace("oracle/", "").lower() or fn == "__init__.py", fn


def test_op_record_layout_matches_header():
    assert abi.OP_DTYPE.itemsize == 40
    assert abi.OP_DTYPE.fields["pos"][1] == 16 and abi.OP_DTYPE.fields["key"][1] == 16
    assert abi.COUNTERS_DTYPE.itemsize == 24


@pytest.fixture(scope="module")
def host_shim(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("shim") / "libshim.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-ffp-contract=off",
                           "-fno-fast-math", "-fPIC", "-shared", "-o", out,
                           os.path.join(ROOT, "tests", "cpp", "quantize_host_shim.hip")])
    lib = ctypes.CDLL(out)
    lib.wq_test_coord_clamp_host.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint16, ctypes.c_void_p]
    lib.wq_test_cube_hash_host.restype = ctypes.c_uint64
    lib.wq_test_cube_hash_host.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
    lib.wq_test_shard_of_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                          ctypes.c_void_p]
    return lib


def _host_clamp(lib, x, s):
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty(x.shape, np.int64)
    lib.wq_test_coord_clamp_host(x.ctypes.data, x.size, s, out.ctypes.data)
    return out


def test_device_quantiser_host_instance_matches_oracle(host_shim, golden_dir, kats):
    """The kernel's divisibility rewrite (q == trunc(q) && fma(q, s, -a) == 0) == fmod(a, s) == 0."""
    for c, s, e in kats["coord_clamp"]:
        assert int(_host_clamp(host_shim, np.array([c]), s)[0]) == e
    z = np.load(os.path.join(golden_dir, "quantize_random.npz"))
    for key in z.files:
        if key.startswith("x_"):
            assert (_host_clamp(host_shim, z[key], int(key[2:])) == z["k_" + key[2:]]).all()
    rng = synth.SplitMix64(99)
    bits = rng.next_u64(300_000).view(np.float64)
    # exact multiples and near-multiples at every magnitude
    k = (rng.next_u64(100_000) >> np.uint64(11)).astype(np.float64)
    for s in (1, 3, 10, 16, 17, 100, 4097, 65535):
        mult = k * s * np.ldexp(1.0, (rng.next_u64(100_000) % np.uint64(40)).astype(np.int64) - 20)
        x = np.concatenate([bits, mult, np.nextafter(mult, np.inf), np.nextafter(mult, -np.inf), -mult])
        assert (_host_clamp(host_shim, x, s) == orc.c_coord_clamp(x, s)).all(), s


def test_cube_hash_host_instance_is_stable(host_shim):
    a = host_shim.wq_test_cube_hash_host(0, 16, 16, 16)
    b = host_shim.wq_test_cube_hash_host(1, 16, 16, 16)
    c = host_shim.wq_test_cube_hash_host(0, 16, 16, 32)
    assert len({a, b, c}) == 3


def test_shard_owner_host_instance_matches_oracle(host_shim):
    """shard_of (csrc/wq_device.hpp) == oracle.shard_of_np: where every bucket lives."""
    rng = synth.SplitMix64(7)
    n = 50_000
    w = (rng.next_u64(n) % np.uint64(70)).astype(np.uint32)
    k = rng.next_u64(3 * n).view(np.int64).copy()
    k[: 3 * n // 2] = (k[: 3 * n // 2] % 4096) * 16  # on-grid keys
    for G in (1, 2, 3, 8, 64):
        out = np.empty(n, np.uint32)
        host_shim.wq_test_shard_of_host(w.ctypes.data, k.ctypes.data, n, G, out.ctypes.data)
        ref = orc.shard_of_np(w, k[0::3], k[1::3], k[2::3], G)
        assert (out == ref).all(), G
        assert out.max() < G
        if G > 1:  # owners spread evenly
            assert np.bincount(out, minlength=G).min() > 0.8 * n / G


# ---- flush-on-reorder batching, with the C oracle standing in for the GPU table -------------

class OracleBackedRouter:
    """Test double with Router's interface, computing with the C restatement (CPU tests only)."""

    def __init__(self, cube_size):
        self.o = orc.COracle(cube_size)
        self.calls = []

    def apply_ops(self, ops):
        self.calls.append(("ops", len(ops)))
        self.o.apply_ops(ops)

    def route(self, pos, world, sender, repl, keys=None, with_msgs=False):
        self.calls.append(("route", len(world)))
        offs, peers, _ = self.o.route(pos, world, sender, repl, keys=keys)
        return offs, peers, None

    def route_global(self, world, sender, repl, with_msgs=False):
        self.calls.append(("global", len(world)))
        offs, peers = self.o.route_global(world, sender, repl)
        return offs, peers, None

    def is_subscribed(self, world, peer, raw, k):
        k = np.asarray(k).reshape(-1, 3)
        return np.array([self.o.is_subscribed(int(w), int(p), raw, kk) for w, p, kk in zip(world, peer, k)])

    def is_subscribed_any(self, world, peer):
        return np.array([self.o.is_subscribed_any(int(w), int(p)) for w, p in zip(world, peer)])

    def world_peers(self, world):
        return self.o.world_peers(world)


def test_tick_batching_preserves_sequential_order():
    from worldql_server_amd.processing import (AREA_SUBSCRIBE, AREA_UNSUBSCRIBE, DISCONNECT, LOCAL_MESSAGE,
                                               Message, SubscriptionProcessor)
    from worldql_server_amd.subscriptions import Vector3, WorldMap
    r = OracleBackedRouter(16)
    wm = WorldMap(16, router=r)
    proc = SubscriptionProcessor(wm)
    v = Vector3(1.0, 2.0, 3.0)
    ev = [
        Message(AREA_SUBSCRIBE, "a", "world", v),
        Message(AREA_SUBSCRIBE, "b", "world one", v),       # sanitized to world_one: another world
        Message(LOCAL_MESSAGE, "c", "world", v),            # -> [a]
        Message(AREA_SUBSCRIBE, "c", "world", v),
        Message(LOCAL_MESSAGE, "a", "world", v),            # ExceptSelf -> [c]
        Message(LOCAL_MESSAGE, "a", "world", v, abi.REPL_INCLUDING_SELF),  # -> [a, c]
        Message(AREA_UNSUBSCRIBE, "a", "world", v),
        Message(LOCAL_MESSAGE, "c", "world", v, abi.REPL_ONLY_SELF),       # -> [c]
        Message(LOCAL_MESSAGE, "c", "@global", v),          # dropped
        Message(LOCAL_MESSAGE, "c", "world", None),         # dropped (no position)
        Message(LOCAL_MESSAGE, "c", "0bad", v),             # dropped (InvalidStart)
        Message(LOCAL_MESSAGE, "c", "nowhere", v),          # no such world -> nothing broadcast
        Message(DISCONNECT, "c"),
        Message(LOCAL_MESSAGE, "b", "world", v, abi.REPL_INCLUDING_SELF),  # -> []
        Message(LOCAL_MESSAGE, "x", "world_one", v),        # -> [b]
    ]
    res = proc.process_tick(ev)
    assert res[2] == ["a"]
    assert res[4] == ["c"]
    assert sorted(res[5]) == ["a", "c"]
    assert res[7] == ["c"]
    assert res[8] is None and res[9] is None and res[10] is None
    assert res[11] is None
    assert res[13] == [] and res[14] == ["b"]
    kinds = [c[0] for c in r.calls]
    assert kinds == ["ops", "route", "ops", "route", "ops", "route", "ops", "route"]


def test_global_messages_and_peer_id_recycling():
    """GlobalMessage runs interleave with LocalMessages in one read run (thread.rs:134); a
    disconnected peer's id is recycled for the next new peer (peer_map.rs:121-141)."""
    from worldql_server_amd.processing import (AREA_SUBSCRIBE, DISCONNECT, GLOBAL_MESSAGE, LOCAL_MESSAGE, Message,
                                               PeerMapBroadcast, SubscriptionProcessor)
    from worldql_server_amd.subscriptions import Vector3, WorldMap
    r = OracleBackedRouter(16)
    wm = WorldMap(16, router=r)
    seen = []
    proc = SubscriptionProcessor(wm, broadcast=lambda ev, rec: seen.append((ev.sender_uuid, rec)))
    v, far = Vector3(1.0, 2.0, 3.0), Vector3(500.0, 2.0, 3.0)
    res = proc.process_tick([
        Message(AREA_SUBSCRIBE, "a", "world", v),
        Message(AREA_SUBSCRIBE, "b", "world", far),
        Message(GLOBAL_MESSAGE, "a", "world"),                          # -> [b]
        Message(LOCAL_MESSAGE, "b", "world", v),                        # -> [a]
        Message(GLOBAL_MESSAGE, "a", "world", None, abi.REPL_ONLY_SELF),  # -> [a]
        Message(GLOBAL_MESSAGE, "z", "@global", None, 7),               # PeerMap broadcast, ExceptSelf
        Message(GLOBAL_MESSAGE, "a", "nowhere"),                        # no such world: nothing
        Message(GLOBAL_MESSAGE, "a", "0bad"),                           # invalid name: dropped
        Message(DISCONNECT, "a"),
        Message(GLOBAL_MESSAGE, "b", "world", None, abi.REPL_INCLUDING_SELF),  # -> [b]
        Message(AREA_SUBSCRIBE, "c", "world", v),                        # takes a's recycled id
        Message(LOCAL_MESSAGE, "b", "world", v),                        # -> [c]
    ])
    assert res[2] == ["b"] and res[3] == ["a"] and res[4] == ["a"]
    assert res[5] == PeerMapBroadcast(abi.REPL_EXCEPT_SELF, "z")
    assert res[6] is None and res[7] is None
    assert res[9] == ["b"] and res[11] == ["c"]
    assert [s[0] for s in seen] == ["a", "b", "a", "z", "b", "b"]  # arrival order
    assert wm.peer_ids.high_water == 2 and len(wm.peer_ids) == 2
    kinds = [c[0] for c in r.calls]
    assert kinds == ["ops", "route", "global", "ops", "global", "ops", "route"]


def test_random_interleaving_vs_sequential_reference():
    """Flush-on-reorder over 2,000 random events (sub / unsub / disconnect / Local / Global, bad
    names, missing positions, unknown replication codes) in ticks of 1..97 events, against the
    reference loop applied one event at a time (tests/seq_reference.py). CPU backend; the GPU
    version is tests/test_gpu_processing.py."""
    from tests.seq_reference import check_ticks, random_events
    from worldql_server_amd.processing import SubscriptionProcessor
    from worldql_server_amd.subscriptions import WorldMap
    wm = WorldMap(16, router=OracleBackedRouter(16))
    n = check_ticks(SubscriptionProcessor(wm), random_events(2000, seed=7), [1, 2, 5, 97, 13, 40])
    assert n > 100


def test_facade_reference_kats_on_oracle_backend(kats):
    """area_map.rs:154-254 through the WorldMap/AreaMap façade (backend: C oracle)."""
    from tests.test_oracle import run_membership_sequence
    from worldql_server_amd.subscriptions import CubeArea, Vector3, WorldMap
    for name in ("area_subscriptions", "world_subscriptions"):
        seq = kats[name]
        wm = WorldMap(seq["cube_size"], router=OracleBackedRouter(seq["cube_size"]))
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
