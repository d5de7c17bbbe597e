"""GPU parity for GlobalMessage to a named world (global_message.rs:36-84):
wq_route_global through the C ABI against the C restatement (oracle/wqo_route_global).

Bar: bit-exact CSR (offsets, and peers ascending within each message)."""
import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth, synth_ext

pytestmark = pytest.mark.gpu


def mk_router(cube_size=16):
    from worldql_server_amd.router import Router
    return Router(cube_size, 0)


def _same(got, want):
    assert (got[0] == want[0]).all()
    assert (got[1] == want[1]).all()
    return len(got[1])


def test_global_small_worlds_all_replications():
    rng = np.random.default_rng(11)
    r, o = mk_router(), orc.COracle(16)
    n = 20000
    ops = abi.ops_array(rng.integers(0, 12, n).astype(np.uint32), rng.integers(0, 3000, n).astype(np.uint32),
                        np.where(rng.random(n) < 0.85, abi.OP_SUBSCRIBE, abi.OP_UNSUBSCRIBE).astype(np.uint8),
                        pos=rng.uniform(-200, 200, (n, 3)))
    r.apply_ops(ops)
    o.apply_ops(ops)
    M = 3000
    world = rng.integers(0, 16, M).astype(np.uint32)  # worlds 12..15 have no subscriptions
    sender = rng.integers(0, 3100, M).astype(np.uint32)
    repl = rng.integers(0, 4, M).astype(np.uint8)   # 3 = an unknown code: ExceptSelf
    got = r.route_global(world, sender, repl, with_msgs=True)
    want = o.route_global(world, sender, repl)
    P = _same(got, want)
    assert P > 0
    msgs = got[2]
    assert (msgs == np.repeat(np.arange(M, dtype=np.uint32), np.diff(got[0]))).all()
    # empty batch, and a batch of absent worlds only
    e = r.route_global(np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
    assert len(e[0]) == 1 and e[0][0] == 0 and len(e[1]) == 0
    a = r.route_global(np.full(5, 99, np.uint32), np.arange(5, dtype=np.uint32), np.ones(5, np.uint8))
    assert (a[0] == 0).all() and len(a[1]) == 0


def test_global_large_worlds_vs_oracle():
    """C4-shaped worlds (scaled): each message fans out to a whole world's subscribed-any set."""
    c4 = synth_ext.config_c4(scale=0.2, worlds=range(0, 64, 8))  # 8 worlds x 10k peers
    r, o = mk_router(), orc.COracle(16)
    ops = c4.initial_ops()
    r.apply_ops(ops)
    o.apply_ops(ops)
    g = synth.stream(4, 77)
    M = 600
    world = (8 * g.below(9, M)).astype(np.uint32)  # world 64 is absent
    sender = g.below(c4.n_peers + 50, M).astype(np.uint32)
    repl = g.below(3, M).astype(np.uint8)
    P = _same(r.route_global(world, sender, repl), o.route_global(world, sender, repl))
    assert P > 1_000_000
    # after churn
    for _ in range(2):
        ops, *_rest = c4.step()
        r.apply_ops(ops)
        o.apply_ops(ops)
    _same(r.route_global(world, sender, repl), o.route_global(world, sender, repl))


def test_global_capacity_reports_required_size():
    from worldql_server_amd.router import WQError
    r = mk_router()
    peers = np.arange(100, dtype=np.uint32)
    r.apply_ops(abi.ops_array(np.zeros(100, np.uint32), peers, np.zeros(100, np.uint8),
                              pos=np.tile([[1.0, 2.0, 3.0]], (100, 1))))
    with pytest.raises(WQError) as e:
        r.route_global(np.zeros(4, np.uint32), np.zeros(4, np.uint32), np.ones(4, np.uint8), capacity=50)
    assert e.value.code == abi.WQ_E_CAPACITY
    off, got, _ = r.route_global(np.zeros(4, np.uint32), np.zeros(4, np.uint32), np.ones(4, np.uint8))
    assert len(got) == 400 and (got == np.tile(peers, 4)).all()


def test_global_device_entry_point():
    import torch
    r = mk_router()
    o = orc.COracle(16)
    rng = np.random.default_rng(3)
    n = 5000
    ops = abi.ops_array(rng.integers(0, 4, n).astype(np.uint32), rng.integers(0, 900, n).astype(np.uint32),
                        np.zeros(n, np.uint8), pos=rng.uniform(-100, 100, (n, 3)))
    r.apply_ops(ops)
    o.apply_ops(ops)
    M = 1000
    world = rng.integers(0, 5, M).astype(np.uint32)
    sender = rng.integers(0, 900, M).astype(np.uint32)
    repl = rng.integers(0, 3, M).astype(np.uint8)
    want = o.route_global(world, sender, repl)
    dev = torch.device("cuda:0")
    r.set_stream(torch.cuda.current_stream().cuda_stream)
    tw, ts, tr = (torch.from_numpy(x.view(np.int32) if x.dtype == np.uint32 else x).to(dev)
                  for x in (world, sender, repl))
    cap = len(want[1]) + 10
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int64, device=dev)
    r.route_global_device(tw.data_ptr(), ts.data_ptr(), tr.data_ptr(), M, offs.data_ptr(), peers.data_ptr(),
                          None, cap, cnt.data_ptr())
    torch.cuda.synchronize()
    P = int(cnt[0].item())
    assert P == len(want[1])
    assert (offs.cpu().numpy().view(np.uint32) == want[0]).all()
    assert (peers[:P].cpu().numpy().view(np.uint32) == want[1]).all()
    r.set_stream(None)
