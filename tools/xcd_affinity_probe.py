"""Experiment: does routing each message on the XCD that "owns" its cube speed up the tick?

Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), and each XCD has its own
L2. Here the C2 messages are only re-ordered, so that tile b (messages 256b .. 256b + 255) holds
messages whose cube falls in class b % 8 (a hash of the cell); the unmodified single-launch tick
then fetches each record line on one XCD only (1/8 of the 36.6 MB of occupied lines per L2).
Routing results are the same per message (checked); only the input order differs.
Usage: python tools/xcd_affinity_probe.py [--steps N]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def xcd_order(pos: np.ndarray, n_class: int = 8, tile: int = 256) -> np.ndarray:
    """Message order in which tile t holds messages of cell class t % n_class (while every class
    still has a whole tile left; the remainder goes last, in any order)."""
    cell = np.floor(pos / 16.0).astype(np.int64)
    h = (cell[:, 0] * 73856093) ^ (cell[:, 1] * 19349663) ^ (cell[:, 2] * 83492791)
    cls = (h & 0x7FFFFFFF) % n_class
    parts = [np.flatnonzero(cls == c) for c in range(n_class)]
    rounds = min(len(p) for p in parts) // tile
    head = [parts[c][k * tile:(k + 1) * tile] for k in range(rounds) for c in range(n_class)]
    tail = [p[rounds * tile:] for p in parts]
    order = np.concatenate(head + tail)
    assert len(order) == len(pos) and len(np.unique(order)) == len(pos)
    return order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from worldql_server_amd import abi, synth
    from worldql_server_amd.router import Router
    dev = torch.device("cuda:0")
    w = synth.config_c2()
    M = len(w.world)
    r = Router(16, 0)
    s = torch.cuda.Stream(device=dev)
    r.set_stream(s.cuda_stream)
    r.apply_ops(w.ops)
    order = xcd_order(w.pos)
    cell = np.floor(w.pos / 16.0).astype(np.int64)
    by_cell = np.lexsort((cell[:, 2], cell[:, 1], cell[:, 0]))  # upper bound: neighbours share records
    res = {}
    outs = {}
    for name, idx in (("original", np.arange(M)), ("xcd_grouped", order), ("cell_sorted", by_cell),
                      ("original_again", np.arange(M))):
        pos = torch.from_numpy(np.ascontiguousarray(w.pos[idx])).to(dev)
        world = torch.from_numpy(np.ascontiguousarray(w.world[idx]).view(np.int32)).to(dev)
        sender = torch.from_numpy(np.ascontiguousarray(w.sender[idx]).view(np.int32)).to(dev)
        repl = torch.from_numpy(np.ascontiguousarray(w.repl[idx])).to(dev)
        offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
        cap = 12 * M
        peers = torch.empty(cap, dtype=torch.int32, device=dev)
        msgs = torch.empty(cap, dtype=torch.int32, device=dev)
        cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
        args = (pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
                peers.data_ptr(), msgs.data_ptr(), cap)
        for _ in range(5):
            r.route_device(*args, cnt.data_ptr())
        torch.cuda.synchronize()
        c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]
        assert c["error"] == 0 and c["overflow"] == 0, c
        P = int(c["n_pairs"])
        o = offs.cpu().numpy().astype(np.int64)
        e = np.diff(o)
        inv = np.empty(M, np.int64)
        inv[idx] = np.arange(M)
        outs[name] = (P, e[inv])  # per original message: recipient counts
        r.profile_enable(True)
        for _ in range(a.steps):
            r.route_device(*args)
        ms, n = r.profile_read()
        r.profile_enable(False)
        res[name] = round(ms / n * 1e3, 2)
    assert outs["original"][0] == outs["xcd_grouped"][0]
    assert np.array_equal(outs["original"][1], outs["xcd_grouped"][1])
    assert np.array_equal(outs["original"][1], outs["cell_sorted"][1])
    print(json.dumps({"M": M, "P": outs["original"][0], "us_per_tick": res}))


if __name__ == "__main__":
    main()
