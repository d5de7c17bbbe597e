#!/bin/bash
# Churn-update check on the GPU box: delta/C345 GPU tests, C4/C5 with phase stamps, plain C4/C5 lines.
# Usage: bash tools/delta_ab.sh <tag>   (outputs under gpurun_out/<tag>_*)
set -uo pipefail
T=${1:-dab}
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_c345.py -x -q --timeout 120 --timeout-method thread > $O/${T}.log 2>&1 || { tail -20 $O/${T}.log; exit 1; }
tail -1 $O/${T}.log
for c in c4 c5; do
  WQ_DELTA_STAMPS=1 timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${T}_${c}s.json 2> $O/${T}_${c}s.err || exit 1
  grep "delta buckets" $O/${T}_${c}s.err | tail -1
done
for c in c4 c5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${T}_${c}.json 2> $O/${T}_${c}.err || exit 1
  python -c "import json; d=json.loads(open('$O/${T}_${c}.json').read().strip().splitlines()[-1]); c=d['config']; print('$c', round(d['ms_per_step'],4), 'update', c.get('update_ms_per_tick'), 'route', c.get('route_ms_per_tick'), 'incr', c.get('incremental_updates'), 'fb', c.get('rebuild_fallbacks'))"
done
