#!/bin/bash
# Round-4 GPU batch V (round end): the whole GPU suite, smoke(), and the default bench line with kernel stats.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_allv 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
$S smokev 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
$S b_finalv 420 python bench.py
$S b_finalv_prof 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b_finalv_prof -o r -- \
    python3 bench.py --no-cpu-baseline
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
echo batch done
