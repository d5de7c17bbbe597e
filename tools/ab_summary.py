#!/usr/bin/env python3
"""Collect the JSON result lines of A/B logs (tools/ab_env.sh, tools/gpu_ab.sh) into one file.

    python tools/ab_summary.py OUT.json "what was compared" gpurun_out/NAME_*.log ...
"""
import json
import os
import sys


def main():
    out, what, logs = sys.argv[1], sys.argv[2], sys.argv[3:]
    runs = {}
    for f in sorted(logs):
        name = os.path.basename(f)[:-4]
        rows = []
        with open(f) as fh:
            for ln in fh:
                if ln.startswith("{"):
                    rows.append(json.loads(ln))
        runs[name] = rows[0] if len(rows) == 1 else rows
    with open(out, "w") as fh:
        json.dump({"what": what, "runs": runs}, fh, indent=1)
    print(out, len(runs), "runs")


if __name__ == "__main__":
    main()
