#!/bin/bash
# Round-4 GPU batch F: per-rank work of the replicated C3 headline at N = 2/4/8 (one GPU, rank 0's
# slice), and the C4 / C5 lines with their kernel stats.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S rslice 300 python tools/replica_slice.py --n 2 4 8 --out gpurun_out/r04_replica_slice.json
$S b_c4 300 python bench.py --config c4 --no-cpu-baseline
$S b_c5 300 python bench.py --config c5 --no-cpu-baseline
$S b_c5_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b_c5_prof -o r -- \
    python3 bench.py --config c5 --no-cpu-baseline
$S b_c4_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b_c4_prof -o r -- \
    python3 bench.py --config c4 --no-cpu-baseline
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
find gpurun_out -type f -size +4M -delete
du -sh gpurun_out
echo batch done
