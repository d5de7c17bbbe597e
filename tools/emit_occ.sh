#!/bin/bash
# C3 emit occupancy sweep on one box: extra dynamic LDS per emit block (WQ_DEBUG_EMIT_LDS bytes)
# caps its blocks per CU; alternating runs of tools/tune_route.py --workload c3 --cfgs 10.
set -uo pipefail
O=gpurun_out; mkdir -p $O
for rep in 1 2; do
  for b in 0 14000 28000 ; do
    WQ_DEBUG_EMIT_LDS=$b timeout -k 10 300 python -u tools/tune_route.py --workload c3 --cfgs 10 --rounds 2 --steps 10 > $O/occ_${b}_$rep.json 2>&1 || { tail $O/occ_${b}_$rep.json; exit 1; }
    echo "lds+$b rep$rep $(tail -1 $O/occ_${b}_$rep.json)"
  done
done
