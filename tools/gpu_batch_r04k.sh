#!/bin/bash
# Round-4 GPU batch K: count tiles / emit blocks per workgroup on a replicated C3 rank's slice.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
for k in 1 2; do
  for tb in "2 2" "1 2" "2 1" "1 1"; do
    set -- $tb
    WQ_DEBUG_COUNT_TPB=$1 WQ_DEBUG_EMIT_BPB=$2 $S rs_t$1_b$2_$k 300 python tools/replica_slice.py --n 4 8 --skip-full
  done
done
echo batch done
