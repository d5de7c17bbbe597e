#!/bin/bash
# Round-4 GPU batch S: churn bucket size sweep (WQ_DELTA_OPS_PER_BUCKET x WQ_DELTA_BPW) on C4 / C5.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
for pb in 32 64 128; do for bpw in 1 2 4; do
    WQ_DELTA_OPS_PER_BUCKET=$pb WQ_DELTA_BPW=$bpw $S c4_${pb}_${bpw} 200 python bench.py --config c4 --no-cpu-baseline
done; done
for pb in 64 128 256; do for bpw in 1 2; do
    WQ_DELTA_OPS_PER_BUCKET=$pb WQ_DELTA_BPW=$bpw $S c5_${pb}_${bpw} 300 python bench.py --config c5 --no-cpu-baseline
done; done
echo batch done
