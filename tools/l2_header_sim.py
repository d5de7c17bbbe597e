#!/usr/bin/env python3
"""Would a spatially grouped header table make the C3 count pass hit L2? A CPU model, not a GPU run:
the count's header probes of the full C3 tick (one 128-B line per probe) replayed through eight
LRU caches of 4 MB (one per XCD; 256-message tiles dealt to XCDs round robin, each XCD's tiles in
order), for the current layout (every cube's header on its own line: load 1/8) and for layouts that
put the headers of a 2x2x2 (or 4x4x2) block of cubes on one line. "L2 share" halves the capacity
left to the headers (the inputs, peer boxes and lists share the L2). Output: profiles/r05_l2_header_sim.txt.

The "xcd-class" rows model the round-4 verdict's item 5 at its best case: 16-B headers at load 0.5
(eight slots per line), the messages handed to XCD hash(cube) % 8 for free (no partition pass is
charged), so each XCD's L2 sees one eighth of the cubes; "hot-first" lays each class's headers out
by descending message count, packing the hottest cubes into the fewest lines.

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
def simulate(ids, share=1.0, xcd=None):
    # blocks of 256 messages round-robin to 8 XCDs; each XCD processes its blocks in order
    # (xcd set: XCD x takes the messages with xcd == x, in order)
    nb = (M + 255)//256
    miss = 0
    for x in range(8):
        lru = OrderedDict()
        cap = int(L2_LINES*share)
        seq = ids[xcd == x].tolist() if xcd is not None else \
            (l for b in range(x, nb, 8) for l in ids[b*256:(b+1)*256].tolist())
        for lid in seq:
            if lid in lru:
                lru.move_to_end(lid)
            else:
                miss += 1
                lru[lid] = 1
                if len(lru) > cap: lru.popitem(last=False)
    return miss
# xcd-class: only messages that hit a cube probe a present header line (a miss probe of an absent
# cube reads a line too: counted the same way, its slot from the hash)
h = (mk.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)
cls = (h & np.uint64(7)).astype(np.int64)
nslots = 1 << int(np.ceil(np.log2(2 * len(cubes))))
rand_line = ((h >> np.uint64(3)) % np.uint64(nslots // 8)).astype(np.int64)
order = np.argsort(-np.bincount(np.searchsorted(cubes, mk[present]), minlength=len(cubes)), kind="stable")
rank = np.empty(len(cubes), np.int64); rank[order] = np.arange(len(cubes))
hot_line = rand_line.copy()
hot_line[present] = rank[np.searchsorted(cubes, mk[present])] // 64  # per class: // 8 lines of 8 slots
for name, ids in [("xcd-class random slots", rand_line), ("xcd-class hot-first", hot_line)]:
    for share in (1.0, 0.5):
        t=time.time(); m = simulate(ids, share, cls)
        print(name, "L2 share", share, "misses", m, f"{m/M:.3f} per message", f"{time.time()-t:.0f}s", flush=True)
for layout in ["random", "2x2x2", "4x4x2"]:
    ids = line_ids(layout)
    for share in (1.0, 0.5):
        t=time.time(); m = simulate(ids, share)
        print(layout, "L2 share", share, "misses", m, f"{m/M:.3f} per message", f"{time.time()-t:.0f}s", flush=True)
