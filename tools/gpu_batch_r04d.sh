#!/bin/bash
# Round-4 GPU batch D: the whole GPU test suite (dense headers on by default), then the default bench
# line and its rocprofv3 kernel stats, and the C3 route PMC with the headers on.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_all 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
$S b_rep1 240 python bench.py --config c3 --shard replicate --steps 10 --warmup 5 --no-extra --no-cpu-baseline
$S b_default 420 python bench.py --steps 20 --warmup 5
$S b_default_prof 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b_default_prof -o r -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
PMC_PASSES="fetch write tcc" PMC_OUT=$(pwd)/gpurun_out/pmc_c3h $S pmc_c3h 400 bash tools/pmc_route.sh 10 --workload c3
python3 tools/pmc_summary.py gpurun_out/pmc_c3h --json gpurun_out/r04_pmc_route_c3_hdr.json --M 10000000 \
    --P 416957138 --exclude tick_kernel > gpurun_out/pmc_c3h_summary.txt 2>&1 || true
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
find gpurun_out -type f -size +4M -delete
du -sh gpurun_out
echo batch done
