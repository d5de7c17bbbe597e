#!/bin/bash
# Round-4 GPU batch P: two messages per count lane (route config 13) on replicated C3 slices.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
for k in 1 2; do
  $S rs_c10_$k 300 python tools/replica_slice.py --n 2 4 8 --skip-full --cfg 10
  $S rs_c13_$k 300 python tools/replica_slice.py --n 2 4 8 --skip-full --cfg 13
done
echo batch done
