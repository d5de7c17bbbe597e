"""Diagnostic: the radius workload of test_hub_radius_ticks_vs_whole_table_oracle through the plain
router, the G = 1 sharded slot tick and the oracle; prints where they differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from oracle import oracle as orc
    from test_gpu_sharded_native import _radius_workload, _tick
    from worldql_server_amd.router import Hub, Router
    ops, churn, peer_pos, mpos, world, sender, repl = _radius_workload()
    radius = 14.0
    M = len(world)
    o = orc.COracle(16)
    o.apply_ops(ops)
    wo, wp = o.route_radius(mpos, world, sender, repl, peer_pos, radius)[:2]
    r = Router(16, 0)
    r.apply_ops(ops)
    r.set_peer_positions(peer_pos)
    r.set_radius(radius)
    go, gp, _ = r.route(mpos, world, sender, repl)
    print("plain vs oracle: P", len(gp), len(wp), "offs equal", (go == wo).all())
    r2 = Router(16, 0)
    r2.set_peer_positions(peer_pos)
    r2.set_radius(radius)
    r2.apply_ops(ops)
    go2, gp2, _ = r2.route(mpos, world, sender, repl)
    print("plain (positions before ops) vs oracle: P", len(gp2), "offs equal", (go2 == wo).all())
    hub = Hub(1)
    r3 = Router(16, 0)
    r3.attach_hub(hub, 0)
    r3.set_peer_positions(peer_pos)
    r3.set_radius(radius)
    r3.sharded_apply_ops(ops)
    w = type("W", (), {"pos": mpos, "world": world, "sender": sender, "repl": repl, "cube_size": 16})
    rc, so, sp, sm = _tick(r3, w, 0, M, torch.device("cuda:0"))
    print("sharded G=1 vs oracle: rc", rc, "P", len(sp), "offs equal", (so == wo).all())
    e_w, e_s = np.diff(wo.astype(np.int64)), np.diff(so.astype(np.int64))
    bad = np.flatnonzero(e_w != e_s)
    print("messages differing", len(bad), "first", bad[:10])
    for m in bad[:5]:
        print(m, "repl", repl[m], "want", wp[wo[m]:wo[m + 1]], "got", sp[so[m]:so[m + 1]])
    print("repl codes of the differing messages", np.bincount(repl[bad], minlength=4))
    r0 = repl.copy()
    r0[r0 == 3] = 0
    go3, gp3, _ = r.route(mpos, world, sender, r0) if False else (None, None, None)
    r4 = Router(16, 0)
    r4.apply_ops(ops)
    r4.set_peer_positions(peer_pos)
    r4.set_radius(radius)
    go4, gp4, _ = r4.route(mpos, world, sender, r0)
    wo4, wp4 = o.route_radius(mpos, world, sender, r0, peer_pos, radius)[:2]
    print("codes 3 -> 0: plain vs oracle offs equal", (go4 == wo4).all(), len(gp4), len(wp4))
    go5, gp5, _ = r4.route(mpos, world, sender, repl)
    print("plain again with code 3:", len(gp5))
    r4.set_radius(0.0)
    go6, gp6, _ = r4.route(mpos, world, sender, repl)
    wo6, wp6, _ = o.route(mpos, world, sender, repl)
    print("radius off, code 3 kept: offs equal", (go6 == wo6).all(), len(gp6), len(wp6))
    r4.close()
    for x in (r, r2, r3):
        x.close()
    hub.close()


if __name__ == "__main__":
    main()
