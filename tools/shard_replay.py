#!/usr/bin/env python3
"""One shard's local work in a G-shard sharded tick (the slot form), measured ALONE on one GPU.

tools/shard_volume.py runs all G shards of a tick on one GPU at once, so its wall time / G only bounds
a shard's work (the shards' kernels contend for the one chip). Here the G shards first run a few
ticks together through a Python all-to-all (host-synchronised device copies) that records what shard
`rank` receives; then shard `rank` alone runs the same tick again and again with an exchange that
REPLAYS those received bytes (sends are dropped) — every kernel of its tick runs as on an 8-GPU node,
on an otherwise idle GPU, and only the links are missing (the replay's copies of the small vectors
are its only exchange cost; the large received buffers are written once and left in place).

    python tools/shard_replay.py [--G 8] [--rank 0] [--ticks 20] [--out gpurun_out/r04_shard_replay.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Exchange:
    """All-to-all among G threads (record mode) or one shard's replay of what it received."""

    def __init__(self, G: int, rank: int):
        import torch
        self.G, self.rank = G, rank
        self.hip = ctypes.CDLL("libamdhip64.so.7")  # the HIP runtime PyTorch already loaded
        self.hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_void_p]
        self.hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        self.bar = threading.Barrier(G)
        self.post = [None] * G
        self.mode = "live"
        self.rec = []          # recorded receives of `rank` in the current tick: (rb, tensor)
        self.tick_rec = None   # the last complete tick's record
        self.k = 0             # call index within the tick (replay)
        self.last_ptr = {}     # call index -> receive pointer already holding the replayed bytes
        self.torch = torch

    def _copy(self, dst, src, n, stream):
        if n:
            assert self.hip.hipMemcpyAsync(dst, src, n, 3, stream or None) == 0  # device to device

    def fn(self, r):
        def call(send, sb, recv, rb, stream):
            if self.mode == "replay":
                assert r == self.rank
                want_rb, data = self.tick_rec[self.k]
                assert list(rb) == want_rb, (self.k, rb, want_rb)
                n = sum(rb)
                small = n < 4096
                if n and (small or self.last_ptr.get(self.k) != recv):
                    self._copy(recv, data.data_ptr(), n, stream)
                    if not small:
                        self.last_ptr[self.k] = recv
                self.k = (self.k + 1) % len(self.tick_rec)
                return
            assert self.hip.hipStreamSynchronize(stream or None) == 0  # my send buffers are complete
            self.post[r] = (send, list(sb))
            self.bar.wait()
            roff = 0
            for src in range(self.G):
                ssend, ssb = self.post[src]
                n = ssb[r]
                assert n == rb[src], (r, src, n, rb[src])
                self._copy(recv + roff, ssend + sum(ssb[:r]), n, stream)
                roff += n
            assert self.hip.hipStreamSynchronize(stream or None) == 0
            if r == self.rank and self.mode == "record":
                t = self.torch.empty(max(sum(rb), 1), dtype=self.torch.uint8, device="cuda:0")
                self._copy(t.data_ptr(), recv, sum(rb), stream)
                assert self.hip.hipStreamSynchronize(stream or None) == 0
                self.rec.append((list(rb), t))
            self.bar.wait()  # nobody reuses a send buffer before every reader has copied it
        return call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--async", dest="use_async", action="store_true",
                    help="replay with wq_sharded_route_tick_async (no end-of-tick read)")
    ap.add_argument("--form", choices=("slots", "owner", "owner_slots"), default="slots",
                    help="owner: wq_sharded_route_owner_device (40-B records out, the pairs stay on the owner); "
                         "owner_slots: wq_sharded_route_owner_slots (budgeted 20-B slots, one exchange)")
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router

    w = synth_ext.config_c3(scale=a.scale)
    M, G = len(w.world), a.G
    dev = torch.device("cuda:0")
    ex = Exchange(G, a.rank)
    routers = [Router(16, 0) for _ in range(G)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(G)]
    bufs = []
    for g in range(G):
        routers[g].set_stream(streams[g].cuda_stream)
        routers[g].attach_exchange(G, g, ex.fn(g))
        routers[g].set_fanout_hint(40.0)
        lo, hi = g * M // G, (g + 1) * M // G
        m = hi - lo
        t = [torch.from_numpy(np.ascontiguousarray(x[lo:hi])).to(dev)
             for x in (w.pos, w.world.view(np.int32), w.sender.view(np.int32), w.repl)]
        offs = torch.empty(m + 1, dtype=torch.int32, device=dev)
        cap = 64 * m + 1024
        bufs.append((m, t, offs, torch.empty(cap, dtype=torch.int32, device=dev),
                     torch.empty(cap, dtype=torch.int32, device=dev), cap))
    torch.cuda.synchronize(dev)

    def tick(g):
        m, t, offs, peers, msgs, cap = bufs[g]
        if a.form == "owner":  # SURVEY.md §8(e) step 5, first option: this shard's pairs stay here
            v = routers[g].sharded_route_owner_device(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
                                                      t[3].data_ptr(), m)
            return int(v.n_pairs)
        if a.form == "owner_slots":
            v = routers[g].sharded_route_owner_slots(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
                                                     t[3].data_ptr(), m)
            return int(v.n_pairs)
        rc, P = routers[g].sharded_route_device(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), m,
                                                offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap)
        assert rc == 0, (g, rc, P)
        return P

    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)

    def tick_async(g):
        m, t, offs, peers, msgs, cap = bufs[g]
        if a.form == "owner_slots":
            routers[g].sharded_route_owner_slots_async(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
                                                       t[3].data_ptr(), m, cnt.data_ptr())
            return
        routers[g].sharded_route_async(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), m,
                                       offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap, cnt.data_ptr())

    errs, Ps = [], [0] * G

    def body(g, n):
        try:
            routers[g].sharded_apply_ops(w.ops) if n is None else None
            for _ in range(n or 0):
                if g == a.rank and ex.mode == "record":
                    ex.rec = []
                Ps[g] = tick(g)
                if g == a.rank and ex.mode == "record":
                    ex.tick_rec = ex.rec
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            ex.bar.abort()

    def run_all(n):
        th = [threading.Thread(target=body, args=(g, n)) for g in range(G)]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()
        if errs:
            raise errs[0]

    t0 = time.perf_counter()
    run_all(None)  # the table: each shard keeps the ops it owns
    build_s = time.perf_counter() - t0
    run_all(3)     # the first tick is exact; the next ones run on budgets
    ex.mode = "record"
    run_all(2)
    P_live = Ps[a.rank]
    rec_bytes = [sum(rb) for rb, _ in ex.tick_rec]
    print("recorded calls per tick:", len(ex.tick_rec), "bytes:", rec_bytes, flush=True)

    # shard `rank` alone: its exchanges replay the recorded receives
    ex.mode, ex.k = "replay", 0
    r = routers[a.rank]
    s = streams[a.rank]
    for _ in range(3):
        assert tick(a.rank) == P_live
    torch.cuda.synchronize(dev)
    if a.use_async:
        for _ in range(3):
            tick_async(a.rank)
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.ticks):
        if a.use_async:
            tick_async(a.rank)  # no end-of-tick read: ticks queue back to back
        else:
            P = tick(a.rank)  # every sharded tick ends with its one host read: wall time is the tick
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / a.ticks
    if a.use_async:
        from bench_configs import _counters
        c = _counters(cnt)[0]
        assert c["error"] == 0 and c["overflow"] == 0, c
        P = int(c["n_pairs"])
    assert P == P_live
    exact, budgeted = r.shard_tick_stats()
    res = {"workload": f"C3 (scale {a.scale}): {M} messages, G = {G} shards; shard {a.rank} alone, its exchanges "
                       "replaying the bytes it received in a live G-shard tick (no link time)",
           "G": G, "rank": a.rank, "form": a.form, "async": bool(a.use_async), "messages_this_shard": bufs[a.rank][0], "pairs_this_shard": int(P),
           "tick_ms_alone": dt * 1e3, "ticks": a.ticks, "received_bytes_per_tick": int(sum(rec_bytes)),
           "table_build_s": round(build_s, 2), "slot_ticks_exact_budgeted": [int(exact), int(budgeted)]}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    for g in range(G):
        routers[g].close()


if __name__ == "__main__":
    main()
