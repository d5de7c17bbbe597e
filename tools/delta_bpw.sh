#!/bin/bash
# Churn parity, then the C4 / C5 lines with 1, 2 and 4 buckets per wave (WQ_DELTA_BPW), alternating, on one box.
set -uo pipefail
T=${1:-bpw}; O=gpurun_out; mkdir -p $O
WQ_DELTA_BPW=3 timeout -k 10 500 python -u -m pytest tests/test_gpu_delta.py \
  "tests/test_gpu_fullsize.py::test_c5_full_tick_radius_exact_vs_oracle" -x -q --timeout 240 --timeout-method thread > $O/${T}.log 2>&1 || { tail -30 $O/${T}.log; exit 1; }
echo "bpw=3: $(tail -1 $O/${T}.log)"
for rep in 1 2; do
  for b in 1 2 4; do
    for c in c4 c5; do
      WQ_DELTA_BPW=$b timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${T}_${b}_${c}_$rep.json 2> $O/${T}.err || { tail $O/${T}.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/${T}_${b}_${c}_$rep.json').read().strip().splitlines()[-1]); c=d['config']; print('bpw=$b $c rep$rep', round(d['ms_per_step'],4), 'update', c.get('update_ms_per_tick'), 'fb', c.get('rebuild_fallbacks'))"
    done
  done
done
