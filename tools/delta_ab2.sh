#!/bin/bash
# Churn parity, then the C4 / C5 lines alternating the default window sort and WQ_DELTA_BITONIC=1
# (the bitonic sort) on one box.
set -uo pipefail
T=${1:-dab2}; O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_c345.py \
  "tests/test_gpu_fullsize.py::test_c4_full_churn_ticks_exact_vs_oracle" \
  "tests/test_gpu_fullsize.py::test_c5_full_tick_radius_exact_vs_oracle" \
  -x -q --timeout 240 --timeout-method thread > $O/${T}.log 2>&1 || { tail -30 $O/${T}.log; exit 1; }
tail -1 $O/${T}.log
for rep in 1 2; do
  for mode in csort bitonic; do
    for c in c4 c5; do
      if [ $mode = bitonic ]; then export WQ_DELTA_BITONIC=1; else unset WQ_DELTA_BITONIC; fi
      timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${T}_${mode}_${c}_$rep.json 2> $O/${T}.err || { tail $O/${T}.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/${T}_${mode}_${c}_$rep.json').read().strip().splitlines()[-1]); c=d['config']; print('$mode $c rep$rep', round(d['ms_per_step'],4), 'update', c.get('update_ms_per_tick'), 'fb', c.get('rebuild_fallbacks'))"
    done
  done
done
