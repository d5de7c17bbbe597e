"""One rank of the replicated-table C3 headline at N GPUs, on one GPU: the whole table, and the
message slice rank r of N routes (bench_configs._c3_replicated's tick, same sizes), timed alone —
what each GPU of an N-GPU node does per tick, without the other ranks. The driver's N-GPU run is the
measurement; this is the per-GPU work it is made of.

    python tools/replica_slice.py --n 8 [--rank 0] [--steps 20] [--warmup 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--skip-full", action="store_true", help="skip the N = 1 line (profiling one slice size)")
    ap.add_argument("--cfg", type=int, default=0, help="route config (wq_debug_set_route_config; 0 = default)")
    ap.add_argument("--chunks", type=int, default=0, help="pipelined heavy-tick chunks (wq_debug_set_route_chunks)")
    ap.add_argument("--keys", action="store_true",
                    help="experiment: route host-quantised raw keys (floor(pos / 16) * 16) instead of the positions")
    ap.add_argument("--no-msgs", action="store_true", help="experiment: no per-pair message index")
    ap.add_argument("--slack", type=int, default=0, help="record slots per cube (wq_debug_set_record_slack; 0 = default)")
    a = ap.parse_args()
    import torch
    import bench
    from bench_configs import _counters
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router

    dev = torch.device("cuda:0")
    w = synth_ext.config_c3()
    M_all = len(w.world)
    r = Router(w.cube_size, 0)
    stream = torch.cuda.Stream(device=dev)
    r.set_stream(stream.cuda_stream)
    if a.cfg:
        r.set_route_config(a.cfg)
    if a.chunks:
        r.set_route_chunks(a.chunks)
    if a.slack:
        r.set_record_slack(a.slack)
    t0 = time.perf_counter()
    r.apply_ops(w.ops)
    build_s = time.perf_counter() - t0
    res = {"workload": "C3, replicated table (27M subscriptions on the one GPU), one rank's message slice",
           "table_build_s": round(build_s, 3), "per_n": {}}
    for n in ([] if a.skip_full else [1]) + [x for x in a.n if x > 1]:
        lo, hi = a.rank * M_all // n, (a.rank + 1) * M_all // n
        M = hi - lo
        pos = torch.from_numpy(w.pos[lo:hi]).to(dev)
        world = torch.from_numpy(w.world[lo:hi].view(np.int32)).to(dev)
        sender = torch.from_numpy(w.sender[lo:hi].view(np.int32)).to(dev)
        repl = torch.from_numpy(w.repl[lo:hi]).to(dev)
        offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
        cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
        keys = (torch.from_numpy((np.floor(w.pos[lo:hi] / w.cube_size) * w.cube_size).astype(np.int64)).to(dev)
                if a.keys else None)
        torch.cuda.synchronize(dev)
        kp = keys.data_ptr() if a.keys else None
        r.route_device(0 if a.keys else pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                       offs.data_ptr(), 0, 0, 0, cnt.data_ptr(), keys_ptr=kp)
        torch.cuda.synchronize(dev)
        P = int(_counters(cnt)["n_pairs"][0])
        r.set_fanout_hint(P / max(M, 1))
        cap = P + 1024
        peers = torch.empty(cap, dtype=torch.int32, device=dev)
        msgs = torch.empty(cap, dtype=torch.int32, device=dev)
        args = (0 if a.keys else pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                offs.data_ptr(), peers.data_ptr(), 0 if a.no_msgs else msgs.data_ptr(), cap)
        for _ in range(a.warmup):
            r.route_device(*args, 0, keys_ptr=kp)
        r.route_device(*args, cnt.data_ptr(), keys_ptr=kp)
        torch.cuda.synchronize(dev)
        c = _counters(cnt)[0]
        P, F = int(c["n_pairs"]), int(c["n_candidates"])
        assert c["overflow"] == 0 and c["error"] == 0, c
        t_ms = bench.timed_ticks(lambda: r.route_device(*args, 0, keys_ptr=kp), a.steps, stream, dev, 1, [r])
        tick_s = t_ms / a.steps / 1e3
        B = bench.algorithmic_bytes(M, F, P)
        res["per_n"][str(n)] = {"rank": a.rank, "messages": M, "pairs": P, "tick_us": round(tick_s * 1e6, 1),
                                "pairs_per_s_this_gpu": P / tick_s,
                                "frac_of_8TBps": B / tick_s / 8e12,
                                "node_pairs_per_s_if_ranks_equal": n * P / tick_s}
        print(json.dumps({n: res["per_n"][str(n)]}), flush=True)
        del peers, msgs, pos, world, sender, repl, offs
        torch.cuda.empty_cache()
    r.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
