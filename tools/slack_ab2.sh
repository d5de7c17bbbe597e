#!/bin/bash
# Record-table slack (slots per cube) A/B with compact headers: C3 full tick, C2 tick, the N = 8 rank.
set -e
for k in 1 2; do
  for sl in 8 4; do
    tools/gpu_step.sh "sk3_${sl}_$k" 300 python tools/tune_route.py --workload c3 --cfgs 10 --rounds 2 --steps 20 --slack $sl
    tools/gpu_step.sh "sk2_${sl}_$k" 300 python tools/tune_route.py --workload c2 --cfgs 0 --rounds 2 --steps 30 --slack $sl
    tools/gpu_step.sh "sk8_${sl}_$k" 300 python tools/replica_slice.py --n 8 --skip-full --slack $sl
  done
done
