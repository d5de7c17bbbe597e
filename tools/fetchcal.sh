#!/bin/bash
# tools/fetchcal.hip under rocprofv3, one counter group per pass (no trace domain beside --pmc), on
# the GPU box from the repo root. Output: gpurun_out/fetchcal/<pass>/..., summary by
# tools/fetchcal_summary.py -> profiles/r04_fetch_calibration.json.
set -euo pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/fetchcal
mkdir -p "$OUT"
hipcc --offload-arch=gfx950 -O3 -o "$ROOT/tools/fetchcal" "$ROOT/tools/fetchcal.hip"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 "$ROOT/tools/fetchcal" 3 > "$OUT/plain.json"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1 || true
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o r -- "$ROOT/tools/fetchcal" 1 \
    > "$OUT/$name.log" 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
run hit TCC_HIT_sum TCC_MISS_sum
echo fetchcal done
