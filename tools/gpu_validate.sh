#!/bin/bash
# Round-end style validation on the GPU box: gpu tests, smoke, default bench, rocprof kernel stats.
# Usage: bash tools/gpu_validate.sh <tag>
set -uo pipefail
TAG=${1:-val}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; cat "$OUT/smoke.log" | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o r -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --steps 50 --warmup 10 > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
rc=$?; echo "rocprof rc=$rc"; exit $rc
