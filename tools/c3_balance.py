#!/usr/bin/env python3
"""Load balance of cube-hash sharding on the full C3 workload (host only, ~2 min).

Per cube: list length (from the subscription ops, quantised like the table does) x messages that
land in it = its pairs (ExceptSelf's -1 ignored). Summed per owner shard_of(world, cube, G), the
max/mean ratio is the imbalance a sharded C3 tick would see. Used to decide whether SURVEY.md
§8(e)'s hot-cube split is needed."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import oracle as orc
from worldql_server_amd import synth_ext

t = time.time()
w = synth_ext.config_c3(1.0)
k = orc.coord_clamp_np(w.ops["pos"], 16)
dt = [("x", "<i8"), ("y", "<i8"), ("z", "<i8")]
ucube, cnt = np.unique(np.ascontiguousarray(k).view(dt).ravel(), return_counts=True)
mk = np.ascontiguousarray(orc.coord_clamp_np(w.pos, 16)).view(dt).ravel()
idx = np.minimum(np.searchsorted(ucube, mk), len(ucube) - 1)
hit = ucube[idx] == mk
pairs = np.where(hit, cnt[idx], 0).astype(np.int64)
P = int(pairs.sum())
load = np.bincount(idx[hit], weights=pairs[hit], minlength=len(ucube))
print(f"C3: {len(ucube)} cubes, longest list {cnt.max()}, P ~ {P}, hottest cube {load.max():.0f} pairs "
      f"({100 * load.max() / P:.3f}% of P)")
uk = ucube.view(np.int64).reshape(-1, 3)
for G in (2, 4, 8):
    own = orc.shard_of_np(np.zeros(len(ucube), np.uint32), uk[:, 0], uk[:, 1], uk[:, 2], G)
    lg = np.bincount(own, weights=load, minlength=G)
    mg = np.bincount(own[idx[hit]], minlength=G)
    print(f"G={G}: pairs max/mean {lg.max() / lg.mean():.4f}, messages max/mean {mg.max() / mg.mean():.4f}")
print(f"({time.time() - t:.0f} s)")
