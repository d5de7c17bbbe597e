#!/bin/bash
# Round-4 GPU batch Q: two ops per lane in the churn events pass — delta / churn / full-size parity,
# then the C4 / C5 lines with kernel stats.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_ev 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_delta.py \
    tests/test_gpu_c345.py tests/test_gpu_fullsize.py tests/test_gpu_processing.py
$S b_c4e 300 python bench.py --config c4 --no-cpu-baseline
$S b_c5e 300 python bench.py --config c5 --no-cpu-baseline
$S b_c5e_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b_c5e_prof -o r -- \
    python3 bench.py --config c5 --no-cpu-baseline
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
echo batch done
