#!/bin/bash
# HBM traffic of whole C4 / C5 ticks (incremental update + route): rocprofv3 --pmc passes over
# `bench.py --config <c4|c5> --no-cpu-baseline`, one counter group per pass (FETCH_SIZE, then
# WRITE_SIZE), summarised per tick over the tick's kernels by tools/pmc_churn_summary.py.
#   bash tools/pmc_churn.sh c5      -> gpurun_out/pmc_c5/{fetch,write}/...
set -euo pipefail
CFG=${1:-c5}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_$CFG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d "$OUT/$p" -o r -- \
    python3 "$ROOT/bench.py" --config "$CFG" --no-cpu-baseline --steps 10 --warmup 2 > "$OUT/$p.json" 2> "$OUT/$p.err"
done
echo pmc done
