#!/usr/bin/env python3
"""Kernel time of the replayed shard's ticks (tools/shard_replay.py under rocprofv3 --kernel-trace):
the dispatches after the last one on any other shard's streams are the replay phase; its last
`ticks` ticks are summed per kernel and compared with the replay's wall time per tick.

    python tools/replay_trace.py gpurun_out/replay_prof/r_kernel_trace.csv --ticks 20 [--json out]
"""
import argparse
import csv
import json
from collections import defaultdict


def short(name: str) -> str:
    """Kernel name without its argument list (anonymous-namespace kernels keep their own name)."""
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    key = next(k for k in rows[0] if k in ("Stream_Id", "Queue_Id"))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    tail_streams = {r[key] for r in rows[-50:]}
    t0 = max(r["e"] for r in rows if r[key] not in tail_streams)
    rep = [r for r in rows if r["s"] > t0]
    # ticks: each replayed tick launches one emit; take the dispatches from the emit `ticks` back
    emits = [i for i, r in enumerate(rep) if "emit_map_kernel" in r["Kernel_Name"]]
    first = emits[-a.ticks - 1] + 1 if len(emits) > a.ticks else 0
    win = rep[first:]
    per = defaultdict(float)
    for r in win:
        per[short(r["Kernel_Name"])] += (r["e"] - r["s"]) / 1e3 / a.ticks
    busy = sum(per.values())
    span = (win[-1]["e"] - win[0]["s"]) / 1e3 / a.ticks
    out = {"kernel_us_per_tick": busy, "span_us_per_tick": span, "dispatches_per_tick": len(win) / a.ticks,
           "per_kernel_us": dict(sorted(per.items(), key=lambda kv: -kv[1]))}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
