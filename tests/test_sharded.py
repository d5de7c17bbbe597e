"""Cube-hash ownership: the owner function and the message grouping of the
multi-GPU path, against the oracle's restatements.

The sharded tick itself is native (csrc/wq_sharded.hip) and runs on the GPU only; its parity tests are
tests/test_gpu_sharded_native.py (hub G in {1, 2, 3, 5}, two processes over a gloo all-to-all through
wq_shard_attach_exchange, RCCL) and tests/test_gpu_g8.py (G = 8). The round-1 Python driver of the
expanded form (worldql_server_amd/sharded.py) was retired in round 5: nothing of the product used it.

CPU: the oracle's owner restatement spreads C3-like keys evenly. GPU: wq_shard_ops and
wq_shard_messages_device are bit-exact against the restatement for several shard counts.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from worldql_server_amd import abi, synth


def make_tick(n_peers=400, n_msgs=3000, seed=11):
    """Several worlds, 3x3x3 subscriptions, churn (unsubscribe + REMOVE_PEER), raw off-grid keys."""
    w = synth.uniform_box(11, n_peers, n_msgs, 96.0, neighbourhood=True, n_worlds=3, repl_mode="mixed")
    rng = np.random.default_rng(seed)
    subs = w.ops
    unsub = subs[rng.choice(len(subs), len(subs) // 10, replace=False)].copy()
    unsub["kind"] = abi.OP_UNSUBSCRIBE
    rm = abi.ops_array(np.full(5, abi.WORLD_INVALID, np.uint32), rng.choice(n_peers, 5, replace=False),
                       np.full(5, abi.OP_REMOVE_PEER, np.uint8), pos=np.zeros((5, 3)))
    raw = abi.ops_array(np.zeros(50, np.uint32), rng.integers(0, n_peers, 50).astype(np.uint32),
                        np.zeros(50, np.uint8), key=rng.integers(-3, 3, (50, 3)) * 5)  # off-grid raw keys
    return w, abi.concat_ops([subs, unsub, rm, raw])


def owner_of_ops(ops, G, cube_size=16):
    """The owner of every op by the oracle's restatement (shard_of_np over the quantised key)."""
    k = np.where(ops["key_is_raw"][:, None] == 1, ops["key"], orc.coord_clamp_np(ops["pos"], cube_size))
    own = orc.shard_of_np(ops["world"], k[:, 0], k[:, 1], k[:, 2], G)
    own[ops["kind"] == abi.OP_REMOVE_PEER] = abi.SHARD_ALL
    return own


def group_messages(pos, keys, world, sender, repl, G, cube_size=16):
    """wq_shard_messages_device restated: 40-byte records grouped by owner, stable, and the counts."""
    k = keys if keys is not None else orc.coord_clamp_np(pos, cube_size)
    own = orc.shard_of_np(world, k[:, 0], k[:, 1], k[:, 2], G)
    order = np.argsort(own, kind="stable")
    recs = np.zeros(len(world), abi.MSG_REC_DTYPE)
    recs["key"], recs["world"], recs["sender"] = k[order], world[order], sender[order]
    recs["msg"], recs["repl"] = order, repl[order]
    return recs, np.bincount(own, minlength=G).astype(np.int32)


def test_shard_owner_split_is_balanced():
    w, _ = make_tick(n_peers=2000, n_msgs=20000)
    own = owner_of_ops(w.ops, 8)
    c = np.bincount(own, minlength=8)
    assert c.min() > 0.8 * len(own) / 8


def test_shard_owner_split_c3_hotspots():
    """C3's hotspot skew, by message: the cube-hash owner spreads the messages within a few percent."""
    from worldql_server_amd import synth_ext
    w = synth_ext.config_c3(scale=0.01)
    k = orc.coord_clamp_np(w.pos, 16)
    c = np.bincount(orc.shard_of_np(w.world, k[:, 0], k[:, 1], k[:, 2], 8), minlength=8)
    assert c.max() / c.mean() < 1.1, c


@pytest.mark.gpu
def test_shard_kernels_match_restatement_gpu():
    import torch
    from worldql_server_amd.router import Router
    w, ops = make_tick(n_peers=1000, n_msgs=50_000)
    r = Router(16, 0)
    dev = torch.device("cuda:0")
    M = len(w.world)
    args = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (w.pos, w.world, w.sender, w.repl)]
    for G in (1, 2, 7, 8, 64):
        assert np.array_equal(r.shard_ops(ops, G), owner_of_ops(ops, G))
        recs = torch.empty((M, abi.MSG_REC_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        counts = torch.empty(G, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        r.shard_messages_device(args[0].data_ptr(), None, args[1].data_ptr(), args[2].data_ptr(),
                                args[3].data_ptr(), M, G, recs.data_ptr(), counts.data_ptr())
        torch.cuda.synchronize()
        want_recs, want_counts = group_messages(w.pos, None, w.world, w.sender, w.repl, G)
        assert np.array_equal(counts.cpu().numpy(), want_counts)
        assert np.array_equal(recs.cpu().numpy().reshape(-1).view(abi.MSG_REC_DTYPE), want_recs)  # bit-exact
    r.close()
