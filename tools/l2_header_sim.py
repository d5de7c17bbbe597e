#!/usr/bin/env python3
"""Would a spatially grouped header table make the C3 count pass hit L2? A CPU model, not a GPU run:
the count's header probes of the full C3 tick (one 128-B line per probe) replayed through eight
LRU caches of 4 MB (one per XCD; 256-message tiles dealt to XCDs round robin, each XCD's tiles in
order), for the current layout (every cube's header on its own line: load 1/8) and for layouts that
put the headers of a 2x2x2 (or 4x4x2) block of cubes on one line. "L2 share" halves the capacity
left to the headers (the inputs, peer boxes and lists share the L2). Output: profiles/r05_l2_header_sim.txt.

    PYTHONPATH=. python3 tools/l2_header_sim.py
"""
import numpy as np, time
from collections import OrderedDict
from worldql_server_amd import synth_ext
from oracle import oracle as orc
w = synth_ext.config_c3(scale=1.0)
M = len(w.world)
k = orc.coord_clamp_np(w.pos, 16) // 16          # cube coords
sub = orc.coord_clamp_np(w.ops["pos"], 16) // 16
def key(c): return ((c[:,0]+2**20)*2**21 + (c[:,1]+2**20))*2**21 + (c[:,2]+2**20)
cubes = np.unique(key(sub))
mk = key(k)
present = np.isin(mk, cubes)
print("messages", M, "hit a cube", present.mean())
rng = np.random.default_rng(1)
def line_ids(layout):
    if layout == "random":       # current: one 128-B line per cube (dense header slot, load 1/8 -> 1 cube per line)
        return mk  # unique per cube
    bs = {"2x2x2": 1, "4x4x2": (2,2,1)}[layout]
    if layout == "2x2x2":
        b = k >> 1
    else:
        b = np.stack([k[:,0]>>2, k[:,1]>>2, k[:,2]>>1],1)
    return key(b)
L2_LINES = 4 * 2**20 // 128
def simulate(ids, share=1.0):
    # blocks of 256 messages round-robin to 8 XCDs; each XCD processes its blocks in order
    nb = (M + 255)//256
    miss = 0
    for x in range(8):
        lru = OrderedDict()
        cap = int(L2_LINES*share)
        for b in range(x, nb, 8):
            for lid in ids[b*256:(b+1)*256].tolist():
                if lid in lru:
                    lru.move_to_end(lid)
                else:
                    miss += 1
                    lru[lid] = 1
                    if len(lru) > cap: lru.popitem(last=False)
    return miss
for layout in ["random", "2x2x2", "4x4x2"]:
    ids = line_ids(layout)
    for share in (1.0, 0.5):
        t=time.time(); m = simulate(ids, share)
        print(layout, "L2 share", share, "misses", m, f"{m/M:.3f} per message", f"{time.time()-t:.0f}s", flush=True)
