#!/bin/bash
# Round-4 GPU batch U: count tiles per block x emit blocks per workgroup on one replicated rank's
# slice at N = 1, 2, 4, 8 (WQ_DEBUG_COUNT_TPB / WQ_DEBUG_EMIT_BPB), two rounds.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
for r in 1 2; do
  for c in 1_1 1_2 2_1 2_2; do
    WQ_DEBUG_COUNT_TPB=${c%_*} WQ_DEBUG_EMIT_BPB=${c#*_} $S shape_${c}_$r 300 python tools/replica_slice.py --n 2 4 8
  done
done
echo batch done
