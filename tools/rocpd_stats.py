#!/usr/bin/env python3
"""Per-kernel summary (calls, average and total time) from a rocprofv3 rocpd database (the
default output of `rocprofv3 --kernel-trace` in ROCm 7.2): python tools/rocpd_stats.py <dir|db>"""
import glob
import os
import sqlite3
import sys

path = sys.argv[1]
by_grid = "--by-grid" in sys.argv  # split each kernel by launch grid size
dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
for f in dbs:
    c = sqlite3.connect(f)
    if by_grid:
        rows = list(c.execute("select name || ' [grid ' || grid_x || ']', count(*), avg(end - start), "
                              "sum(end - start) from kernels group by name, grid_x order by sum(end - start) desc"))
    else:
        rows = list(c.execute("select name, count(*), avg(end - start), sum(end - start) from kernels "
                              "group by name order by sum(end - start) desc"))
    tot = sum(r[3] for r in rows)
    print(f"# {os.path.basename(f)}: {len(rows)} kernels, {tot / 1e6:.2f} ms in total")
    print(f"{'avg_us':>10} {'calls':>6} {'total_ms':>9} {'share':>6}  name")
    for name, n, avg, s in rows:
        if by_grid and "[grid" in name:
            name = name[:70] + name[name.rindex(" [grid"):]
        print(f"{avg / 1e3:10.1f} {n:6d} {s / 1e6:9.3f} {100 * s / tot:5.1f}%  {name[:110]}")
