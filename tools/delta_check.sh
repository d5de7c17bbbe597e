#!/bin/bash
# Churn-update parity + timing on the GPU box: delta / C345 tests, the full-size C4 / C5 churn
# ticks against the oracle, then C4 / C5 bench lines (and, with STAMPS=1, the phase stamps).
# Usage: bash tools/delta_check.sh <tag>   (outputs under gpurun_out/<tag>*)
set -uo pipefail
T=${1:-dchk}
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_c345.py \
  "tests/test_gpu_fullsize.py::test_c4_full_churn_ticks_exact_vs_oracle" \
  "tests/test_gpu_fullsize.py::test_c5_full_tick_radius_exact_vs_oracle" \
  -x -v --timeout 240 --timeout-method thread > $O/${T}.log 2>&1 || { tail -30 $O/${T}.log; exit 1; }
tail -1 $O/${T}.log
for c in c4 c5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${T}_${c}.json 2> $O/${T}_${c}.err || { tail $O/${T}_${c}.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/${T}_${c}.json').read().strip().splitlines()[-1]); c=d['config']; print('$c', round(d['ms_per_step'],4), 'update', c.get('update_ms_per_tick'), 'route', c.get('route_ms_per_tick'), 'incr', c.get('incremental_updates'), 'fb', c.get('rebuild_fallbacks'))"
done
if [ "${STAMPS:-0}" = 1 ]; then
  for c in c4 c5; do
    WQ_DELTA_STAMPS=1 timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${T}_${c}s.json 2> $O/${T}_${c}s.err || exit 1
    grep "delta buckets" $O/${T}_${c}s.err | tail -1
  done
fi
