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
    # several sums at once, as the N > 1 C3 line reduces pairs and algorithmic bytes together
    both = bench.allreduce([len(peers), bench.algorithmic_bytes(len(w.world), len(peers), len(peers))], "sum",
                           torch.device("cpu"), world_size)
    out[rank] = (t_max, pairs, len(peers), both, bench.algorithmic_bytes(len(w.world), len(peers), len(peers)))
    dist.barrier()
    dist.destroy_process_group()


def test_world_sharded_reduction_gloo():
    ws = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(ws, _free_port(), out), nprocs=ws, start_method="spawn", join=True)
    per_rank = [out[r][2] for r in range(ws)]
    for r in range(ws):
        t_max, pairs, _, both, _ = out[r]
        assert t_max == 11.0
        assert pairs == float(sum(per_rank))
        assert both == [float(sum(per_rank)), float(sum(out[k][4] for k in range(ws)))]
    # every rank's shard is the same tick shape in a different world: same pair count
    assert per_rank[0] == per_rank[1] > 0


def _bench_cmd(*args, env):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], cwd=root, env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_gpus_must_match_the_launcher():
    """Under a launcher --gpus must equal WORLD_SIZE (exit 2, before any GPU call)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = _bench_cmd("--gpus", "8", env=env)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr, (p.returncode, p.stderr[-2000:])


def _has_gpu() -> bool:
    import torch
    return torch.cuda.device_count() > 0  # counts without initialising the GPU


@pytest.mark.skipif(_has_gpu(), reason="the ranks would run for real: covered by tests/test_gpu_bench.py")
def test_bench_own_launcher_reports_a_failed_rank():
    """--gpus 2 without a launcher starts two ranks of bench.py itself; here (no GPU) both fail at their
    first GPU call, and the parent exits non-zero instead of printing a line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = _bench_cmd("--gpus", "2", "--config", "c1", "--steps", "1", "--warmup", "1", env=env)
    assert p.returncode != 0 and "{" not in p.stdout, (p.returncode, p.stdout[-2000:])
    assert "exited with status" in p.stderr, p.stderr[-2000:]
