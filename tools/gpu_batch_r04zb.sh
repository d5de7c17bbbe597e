#!/bin/bash
# Round-4 GPU batch ZB (round end, final tree): the whole GPU suite, smoke(), and the default bench line with kernel stats.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_allzb 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
$S smokezb 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
$S b_finalzb 420 python bench.py
$S b_finalzb_prof 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b_finalzb_prof -o r -- \
    python3 bench.py --no-cpu-baseline
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
echo batch done
