#!/bin/bash
# Radius parity with the default build, then the C5 line alternating the default build and $1
# (WQ_LIBRARY) on one box: bash tools/ab_c5.sh <other .so>
set -uo pipefail
B=$1; O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_c345.py "tests/test_gpu_fullsize.py::test_c5_full_tick_radius_exact_vs_oracle" -x -q --timeout 240 --timeout-method thread > $O/abc5.log 2>&1 || { tail -30 $O/abc5.log; exit 1; }
tail -1 $O/abc5.log
for rep in 1 2; do
  for which in new old; do
    if [ $which = old ]; then export WQ_LIBRARY=$B; else unset WQ_LIBRARY; fi
    timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > $O/abc5_${which}_$rep.json 2> $O/abc5.err || { tail $O/abc5.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/abc5_${which}_$rep.json').read().strip().splitlines()[-1]); c=d['config']; print('$which rep$rep', round(d['ms_per_step'],4), 'update', c.get('update_ms_per_tick'), 'route', c.get('route_ms_per_tick'), 'route kernels us', round(d['roofline'].get('kernel_avg_us',0),1))"
  done
done
