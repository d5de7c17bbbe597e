"""Diagnostic: one message of the radius workload through the plain router, replication codes 0-3,
radius 14 and 1e9."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from test_gpu_sharded_native import _radius_workload
    from worldql_server_amd.router import Router
    ops, churn, peer_pos, mpos, world, sender, repl = _radius_workload()
    r = Router(16, 0)
    r.apply_ops(ops)
    r.set_peer_positions(peer_pos)
    for radius in (14.0, 1e9):
        r.set_radius(radius)
        for m in (26, 57):
            for rp in (0, 1, 2, 3, 4, 255):
                offs, peers, _ = r.route(mpos[m:m + 1], world[m:m + 1], sender[m:m + 1], np.array([rp], np.uint8))
                print("radius", radius, "msg", m, "code", rp, "->", peers.tolist(), flush=True)
    r.close()


if __name__ == "__main__":
    main()
