"""What the sharded tick's machinery costs on one GPU: C3 (or a scaled C3) routed by the plain device
tick and by wq_sharded_route_tick_device as shard 0 of 1 over RCCL (shard kernels, the exchanges'
self-copies, the two count read-backs, the owner route, the unshard), same table, same outputs.
Usage: python tools/sharded_overhead.py [--scale S] [--steps K]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from worldql_server_amd import abi, synth_ext
    from worldql_server_amd.router import Router, rccl_unique_id
    dev = torch.device("cuda:0")
    w = synth_ext.config_c3(scale=a.scale)
    M = len(w.world)
    pos = torch.from_numpy(w.pos).to(dev)
    world = torch.from_numpy(w.world.view(np.int32)).to(dev)
    sender = torch.from_numpy(w.sender.view(np.int32)).to(dev)
    repl = torch.from_numpy(w.repl).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 64 * M + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    res = {"M": M}

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    s = torch.cuda.Stream(device=dev)
    plain = Router(16, 0)
    plain.set_stream(s.cuda_stream)
    plain.apply_ops(w.ops)
    plain.set_fanout_hint(40.0)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    res["plain_ms"] = timed(lambda: plain.route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(),
                                                       repl.data_ptr(), M, offs.data_ptr(), peers.data_ptr(),
                                                       msgs.data_ptr(), cap, cnt.data_ptr()))
    P = int(cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]["n_pairs"])
    ref = (offs.clone(), peers[:P].clone())
    plain.close()

    sh = Router(16, 0)
    sh.set_stream(s.cuda_stream)
    sh.attach_rccl(1, 0, rccl_unique_id())
    sh.sharded_apply_ops(w.ops)
    sh.set_fanout_hint(40.0)
    out = {}

    def tick():
        rc, out["P"] = sh.sharded_route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(),
                                               M, offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap)
        assert rc == 0
    res["sharded_1_ms"] = timed(tick)
    assert out["P"] == P and torch.equal(offs, ref[0]) and torch.equal(peers[:P], ref[1])
    res["P"] = P
    sh.detach_shard()
    sh.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
