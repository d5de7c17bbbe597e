#!/bin/bash
# Kernel-trace stats of one tools/tune_route.py run: bash tools/kstats.sh <name> <tune args...>
# Output: gpurun_out/ks_<name>/…kernel_stats.csv (+ a short summary on stdout)
set -euo pipefail
NAME=$1; shift
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/ks_$NAME" -o r -- \
  python3 "$ROOT/tools/tune_route.py" "$@" > "$ROOT/gpurun_out/ks_$NAME.log" 2>&1
python3 - "$ROOT/gpurun_out/ks_$NAME" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wq::" in r["Name"]:
            print(f'{float(r["AverageNs"])/1e3:8.1f} us  x{r["Calls"]:>5}  {r["Name"][:90]}')
PY
