#!/bin/bash
# Kernel-trace stats of one bench.py run: bash tools/kstats_bench.sh <name> <bench args...>
# Output: gpurun_out/kb_<name>/ (rocprofv3 csv) + gpurun_out/kb_<name>.json (the bench line) + a summary.
set -euo pipefail
NAME=$1; shift
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/kb_$NAME" -o r -- \
  python3 "$ROOT/bench.py" "$@" > "$ROOT/gpurun_out/kb_$NAME.json" 2> "$ROOT/gpurun_out/kb_$NAME.err"
tail -c 600 "$ROOT/gpurun_out/kb_$NAME.json"; echo
python3 - "$ROOT/gpurun_out/kb_$NAME" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:25]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]:>5} {float(r["TotalDurationNs"])/1e6:8.2f} ms  {r["Name"][:90]}')
PY
