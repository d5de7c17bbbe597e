"""Per-tick HBM traffic of a C4 / C5 bench run from tools/pmc_churn.sh: FETCH_SIZE (x2, the gfx950
correction of MI355X_MICROARCH.md) + WRITE_SIZE summed over the tick's kernels (update: k_delta_*,
k_sort_*, k_bucket_*; positions: k_pos_f32 / k_pos_box / k_pos_code; route: count / scan / emit / tick kernels), divided by
the ticks run (warmup + steps).
    python tools/pmc_churn_summary.py gpurun_out/pmc_c5 --ticks 12 [--json profiles/r02_pmc_c5.json]"""
import argparse
import collections
import csv
import glob
import json
import os

TICK = ("k_delta_", "k_sort_", "k_bucket_", "k_pos_", "count_radius_kernel", "count_kernel", "tile_scan_kernel",
        "tile_finish_kernel", "tile_scan_multi_kernel", "emit_kernel", "emit_map_kernel", "tick_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--ticks", type=int, required=True)
    ap.add_argument("--json")
    a = ap.parse_args()
    tot = collections.Counter()
    per = collections.defaultdict(collections.Counter)
    for f in glob.glob(os.path.join(a.root, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if not any(k in name for k in TICK):
                continue
            c = row["Counter_Name"]
            v = float(row["Counter_Value"]) * 1024 * (2 if c.startswith("FETCH") else 1)
            tot[c] += v
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            per[short[:60]][c] += v
    out = {"ticks": a.ticks, "fetch_bytes_per_tick": tot["FETCH_SIZE"] / a.ticks,
           "write_bytes_per_tick": tot["WRITE_SIZE"] / a.ticks,
           "hbm_bytes_per_tick": (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / a.ticks,
           "kernels": {k: {c: v / a.ticks for c, v in d.items()} for k, d in sorted(per.items())},
           "note": "FETCH_SIZE (KB) x 1024 x 2 (gfx950 128-B requests tallied at 64 B) + WRITE_SIZE (KB) x 1024, "
                   "summed over the tick kernels and divided by the ticks run"}
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))
    for k, d in out["kernels"].items():
        print(f"{k:62s} fetch {d.get('FETCH_SIZE', 0) / 1e6:9.1f} MB  write {d.get('WRITE_SIZE', 0) / 1e6:9.1f} MB")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
