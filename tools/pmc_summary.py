"""Summarise tools/pmc_route.sh output: per-kernel mean of every counter over its dispatches.

    python tools/pmc_summary.py gpurun_out/pmc [--json profiles/r01_pmc_route.json --M 1000000 --P 9975215]
    python tools/pmc_summary.py gpurun_out/pmc_c3 --json profiles/r01_pmc_route_c3.json --M 10000000 \
        --P 416957138 --exclude tick_kernel     (C3, count / tile_scan / emit)
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                short = k.split("(")[0].replace("void ", "")
                per[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    ap.add_argument("--M", type=int)
    ap.add_argument("--P", type=int)
    ap.add_argument("--exclude", default="", help="kernel-name substring left out of the tick sum (e.g. the "
                    "sizing call's tick_kernel when the measured shape is count / tile_scan / emit)")
    a = ap.parse_args()
    per = load(a.root)
    route = {}
    for k, cs in sorted(per.items()):
        if not k.startswith("wq::"):
            continue
        means = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k)
        for c, v in sorted(means.items()):
            print(f"    {c:28s} {v:16.1f}   (n={len(cs[c])})")
        if any(s in k for s in ("count_kernel", "tile_scan_kernel", "tile_finish_kernel", "emit_kernel",
                                "emit_heavy_kernel", "emit_map_kernel", "tick_kernel")) and not (
                a.exclude and a.exclude in k):
            route[k] = means
    if a.json and route:
        # gfx950: FETCH_SIZE tallies 128-B line requests as 64 B (MI355X_MICROARCH.md §HBM) -> x2
        fetch = sum(m.get("FETCH_SIZE", 0.0) for m in route.values()) * 1024 * 2
        write = sum(m.get("WRITE_SIZE", 0.0) for m in route.values()) * 1024
        out = {"messages_per_tick": a.M, "pairs_per_tick": a.P,
               "hbm_bytes_per_launch": fetch + write, "fetch_bytes_corrected": fetch, "write_bytes": write,
               "kernels": route,
               "note": "sum over the tick's launches (default: the single tick_kernel); FETCH_SIZE (KB) x 1024 x 2 "
                       "(gfx950 128-B requests tallied at 64 B), WRITE_SIZE (KB) x 1024"}
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", a.json)


if __name__ == "__main__":
    main()
