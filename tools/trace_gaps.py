#!/usr/bin/env python3
"""Per-tick timeline of a rocprofv3 kernel trace (csv): ticks start at a marker kernel; prints per tick
the span (first start -> last end), the kernel time, the idle time inside the span, and the idle gap
before the tick (the previous tick's last end -> this tick's first start), averaged over the last N
ticks, plus each kernel's mean time and the largest idle gaps and what precedes them.

    python tools/trace_gaps.py DIR --marker own_count_hist_kernel [--last 20]
"""
import argparse
import csv
import glob
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", required=True)
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    f = sorted(glob.glob(a.dir + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    starts = [i for i, k in enumerate(ks) if a.marker in k[2]]
    ticks = [ks[s:e] for s, e in zip(starts, starts[1:] + [len(ks)])][-a.last - 1:-1]
    prev_end = None
    spans, kern, idle, before, per = [], [], [], [], {}
    gaps = []
    for t in ticks:
        first, last = t[0][0], max(k[1] for k in t)
        busy, cur_end = 0, first
        for i, (s, e, n) in enumerate(t):
            if s > cur_end:
                gaps.append((s - cur_end, t[i - 1][2][:60] if i else "-", n[:60]))
            busy += max(0, e - max(s, cur_end))
            cur_end = max(cur_end, e)
            per.setdefault(n[:90], []).append(e - s)
        spans.append(last - first)
        kern.append(busy)
        idle.append(last - first - busy)
        # idle before this tick: from the end of the previous tick's kernels
        b = ks[ks.index(t[0]) - 1][1] if ks.index(t[0]) else first
        before.append(first - b)
    us = lambda v: round(statistics.mean(v) / 1e3, 1)  # noqa: E731
    gaps.sort(reverse=True)
    out = {"ticks": len(ticks), "span_us": us(spans), "busy_us": us(kern), "idle_in_span_us": us(idle),
           "idle_before_tick_us": us(before), "period_us": us([s + b for s, b in zip(spans, before)]),
           "kernels_per_tick": round(sum(len(t) for t in ticks) / len(ticks), 1),
           "per_kernel_us": {k: round(sum(v) / len(ticks) / 1e3, 1) for k, v in
                             sorted(per.items(), key=lambda kv: -sum(kv[1]))},
           "largest_gaps_us": [(round(g / 1e3, 1), p, n) for g, p, n in gaps[:12]]}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
