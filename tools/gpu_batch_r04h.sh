#!/bin/bash
# Round-4 GPU batch H: kernel stats of one rank's replicated C3 slice at N = 8 (1.25M messages).
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S rs8_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rs8_prof -o r -- \
    python3 tools/replica_slice.py --n 8 --steps 40 --skip-full
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
find gpurun_out -type f -size +4M -delete
echo batch done
