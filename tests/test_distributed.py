"""CPU: the multi-rank path of bench.py (world-sharded weak scaling) with gloo, world_size 2.

Each rank builds its own shard (its own world id), routes it with the C restatement standing in
for the GPU, and the max-time / sum-pairs reduction is checked against the per-rank values.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world_size, port, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    import bench
    from oracle import oracle as orc
    w = bench.shard_workload(rank, scale=0.002)
    assert (w.world == rank).all() and (w.ops["world"] == rank).all()
    o = orc.COracle(w.cube_size)
    o.apply_ops(w.ops)
    _, peers, _ = o.route(w.pos, w.world, w.sender, w.repl)
    t_ms = 10.0 + rank  # per-rank "timed region"
    t_max, pairs = bench.reduce_over_ranks(t_ms, len(peers), torch.device("cpu"), world_size)
    out[rank] = (t_max, pairs, len(peers))
    dist.barrier()
    dist.destroy_process_group()


def test_world_sharded_reduction_gloo():
    ws = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(ws, _free_port(), out), nprocs=ws, start_method="spawn", join=True)
    per_rank = [out[r][2] for r in range(ws)]
    for r in range(ws):
        t_max, pairs, _ = out[r]
        assert t_max == 11.0
        assert pairs == float(sum(per_rank))
    # every rank's shard is the same tick shape in a different world: same pair count
    assert per_rank[0] == per_rank[1] > 0
