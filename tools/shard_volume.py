#!/usr/bin/env python3
"""What the sharded tick moves between GPUs, measured at any G on ONE GPU (the in-process hub:
G router handles on cuda:0, one thread each — the collective runs for real, only the links are
local copies). Full C3 by default: every shard ingests M/G of the 10M messages; per shard the
bytes sent to / received from the other shards (wq_shard_last_bytes) in both return forms:

  slots     20-byte slots out; 12-byte row references + one pool of cube lists per
            (owner, destination) back (the default)
  expanded  40-byte records out; per-record counts + expanded peer ids back (the radius form)

    python tools/shard_volume.py [--G 8] [--scale 1.0] [--out profiles/r03_c3_xgmi_g8.json]

The bench's C3 line quotes the result as its modelled xGMI volume per GPU (bench_configs.py)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--hot-peers", type=int, default=0,
                    help="skew: one extra cube with this many subscribers ...")
    ap.add_argument("--hot-frac", type=float, default=0.0, help="... that this fraction of the messages hit")
    ap.add_argument("--ticks", type=int, default=0,
                    help="then time this many slot-form ticks of all G shards on the one GPU (barrier + sync "
                         "around them): wall / G bounds the mean local work per shard (every shard's kernels "
                         "and the hub copies share the one GPU)")
    a = ap.parse_args()
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Hub, Router

    w = synth_ext.config_c3(scale=a.scale)
    M, G = len(w.world), a.G
    hot_note = ""
    if a.hot_peers:  # one cube far from every hotspot, subscribed by peers 0 .. H-1, hit by hot_frac of M
        from worldql_server_amd import abi
        hp = np.full((a.hot_peers, 3), [200000.5, 8.5, 8.5])
        hot_ops = abi.ops_array(np.zeros(a.hot_peers, np.uint32), np.arange(a.hot_peers, dtype=np.uint32),
                                np.zeros(a.hot_peers, np.uint8), pos=hp)
        w.ops = abi.concat_ops([w.ops, hot_ops])
        idx = np.random.default_rng(7).choice(M, int(a.hot_frac * M), replace=False)
        w.pos = w.pos.copy()
        w.pos[idx] = [200000.5, 8.5, 8.5]
        hot_note = f" + one cube with {a.hot_peers} subscribers hit by {len(idx)} messages"
    dev = torch.device("cuda:0")
    hub = Hub(G)
    routers = [Router(16, 0) for _ in range(G)]
    res = {"slots": [None] * G, "expanded": [None] * G}
    errors = []
    bar = threading.Barrier(G)
    timed = {"t": 0.0}

    def body(rank):
        try:
            r = routers[rank]
            r.attach_hub(hub, rank)
            r.set_fanout_hint(40.0)
            lo, hi = rank * M // G, (rank + 1) * M // G
            n = hi - lo
            r.sharded_apply_ops(w.ops)
            pos = torch.from_numpy(np.ascontiguousarray(w.pos[lo:hi])).to(dev)
            wo = torch.from_numpy(np.ascontiguousarray(w.world[lo:hi]).view(np.int32)).to(dev)
            se = torch.from_numpy(np.ascontiguousarray(w.sender[lo:hi]).view(np.int32)).to(dev)
            rp = torch.from_numpy(np.ascontiguousarray(w.repl[lo:hi])).to(dev)
            offs = torch.empty(n + 1, dtype=torch.int32, device=dev)
            cap = 64 * n + 1024
            peers = torch.empty(cap, dtype=torch.int32, device=dev)
            torch.cuda.synchronize(dev)
            for form in ("slots", "expanded"):
                r.set_shard_form(form == "expanded")
                rc, P = r.sharded_route_device(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), n,
                                               offs.data_ptr(), peers.data_ptr(), None, cap)
                assert rc == 0, rc
                sent, recvd = r.shard_last_bytes()
                res[form][rank] = {"messages": n, "pairs": int(P), "sent_bytes": int(sent), "recv_bytes": int(recvd)}
            if a.ticks:
                r.set_shard_form(False)
                for _ in range(2):  # warm: budgets set
                    r.sharded_route_device(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), n,
                                           offs.data_ptr(), peers.data_ptr(), None, cap)
                torch.cuda.synchronize(dev)
                bar.wait()
                t1 = time.perf_counter()
                for _ in range(a.ticks):
                    rc, _ = r.sharded_route_device(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), n,
                                                   offs.data_ptr(), peers.data_ptr(), None, cap)
                    assert rc == 0, rc
                torch.cuda.synchronize(dev)
                bar.wait()
                if rank == 0:
                    timed["t"] = (time.perf_counter() - t1) / a.ticks
                res["slots"][rank]["tick_stats"] = r.shard_tick_stats()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    t0 = time.perf_counter()
    th = [threading.Thread(target=body, args=(k,)) for k in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    out = {"workload": f"C3 (scale {a.scale}){hot_note}: {M} messages, {len(w.ops)} subscriptions, G = {G} shards as hub "
                       f"threads on one GPU (the bytes are those an {G}-GPU run moves over xGMI)",
           "G": G, "messages_per_tick": M, "pairs_per_tick": sum(x["pairs"] for x in res["slots"]),
           "wall_s": round(time.perf_counter() - t0, 1)}
    for form in ("slots", "expanded"):
        s = [x["sent_bytes"] for x in res[form]]
        r_ = [x["recv_bytes"] for x in res[form]]
        out[form] = {"sent_bytes_per_gpu_mean": float(np.mean(s)), "sent_bytes_per_gpu_max": int(max(s)),
                     "sent_max_over_mean": float(max(s) / max(np.mean(s), 1.0)),
                     "recv_bytes_per_gpu_mean": float(np.mean(r_)), "recv_bytes_per_gpu_max": int(max(r_)),
                     "per_shard": res[form]}
    out["slots_vs_expanded"] = out["slots"]["sent_bytes_per_gpu_mean"] / out["expanded"]["sent_bytes_per_gpu_mean"]
    if a.ticks:
        out["one_gpu_tick_ms"] = timed["t"] * 1e3
        out["mean_local_work_per_shard_ms_upper"] = timed["t"] * 1e3 / G
        out["timed_ticks"] = a.ticks
        out["note_timing"] = ("all G shards' kernels and hub copies run on ONE GPU: the G-shard tick's wall time / G is "
                              "an upper bound on one shard's local work (pairs max / mean in per_shard)")
    print(json.dumps({k: v for k, v in out.items() if k not in ("slots", "expanded")}))
    print(json.dumps({f: {k: v for k, v in out[f].items() if k != "per_shard"} for f in ("slots", "expanded")}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    for r in routers:
        r.close()
    hub.close()


if __name__ == "__main__":
    main()
