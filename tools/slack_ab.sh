#!/bin/bash
set -e
for k in 1 2; do
  for sl in 8 4 2; do
    tools/gpu_step.sh "sk_${sl}_$k" 300 python tools/tune_route.py --workload c3 --cfgs 10 --rounds 2 --steps 20 --slack $sl
  done
done
