#!/bin/bash
# Round-4 GPU batch R: tick_map_kernel (heavy fan-out in one launch, route configs 13 / 14) —
# every-config parity, then one replicated rank's slice at N = 1, 2, 4, 8 under configs 10, 13, 14.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_tm 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_routing.py \
    tests/test_gpu_c345.py
for c in 10 13 14; do
    $S rs_$c 400 python tools/replica_slice.py --n 2 4 8 --cfg $c --out gpurun_out/rs_$c.json
done
echo batch done
