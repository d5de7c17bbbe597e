#!/bin/bash
# Kernel trace of the C5 (or C4) tick, summarised per tick (tools/trace_gaps.py, ticks start at
# k_delta_events): bash tools/trace_c5.sh [c5|c4] -> gpurun_out/tr_<cfg>/ and gpurun_out/tr_<cfg>.json
set -euo pipefail
CFG=${1:-c5}
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tr_$CFG" -o r -- \
  python3 "$R/bench.py" --config "$CFG" --no-cpu-baseline --steps 10 --warmup 3 > "$R/gpurun_out/tr_$CFG.log" 2>&1
cd "$R" && python3 tools/trace_gaps.py "gpurun_out/tr_$CFG" --marker k_delta_events --last 8 --out "gpurun_out/tr_$CFG.json"
