#!/bin/bash
# Round-4 GPU batch C: C++ mirror (diagnostics), the default bench line, the G = 8 hub timing, the
# C3 route PMC (fetch / write / tcc incl. RDREQ), fetch calibration, churn PMC for C5 and C4, and
# the C4 / C5 lines. Raw profiler output pruned at the end.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_cpp 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cpp_mirror.py || true
$S b_default 420 python bench.py --steps 20 --warmup 5
$S sv8 300 python tools/shard_volume.py --G 8 --ticks 5 --out gpurun_out/sv8.json
$S sv8_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sv8_prof -o r -- \
    python3 tools/shard_volume.py --G 8 --ticks 5
PMC_PASSES="fetch write tcc" PMC_OUT=$(pwd)/gpurun_out/pmc_c3 $S pmc_c3 400 bash tools/pmc_route.sh 10 --workload c3
python3 tools/pmc_summary.py gpurun_out/pmc_c3 --json gpurun_out/r04_pmc_route_c3.json --M 10000000 --P 416957138 \
    --exclude tick_kernel > gpurun_out/pmc_c3_summary.txt 2>&1 || true
$S fetchcal 300 bash tools/fetchcal.sh
python3 tools/fetchcal_summary.py gpurun_out/fetchcal gpurun_out/fetch_calibration.json > gpurun_out/fetchcal_summary.txt 2>&1 || true
$S pmc_c5 400 bash tools/pmc_churn.sh c5
python3 tools/pmc_churn_summary.py gpurun_out/pmc_c5 --ticks 12 --json gpurun_out/r04_pmc_c5.json > gpurun_out/pmc_c5_summary.txt 2>&1 || true
$S pmc_c4 400 bash tools/pmc_churn.sh c4
python3 tools/pmc_churn_summary.py gpurun_out/pmc_c4 --ticks 12 --json gpurun_out/r04_pmc_c4.json > gpurun_out/pmc_c4_summary.txt 2>&1 || true
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
find gpurun_out -type f -size +4M -delete
du -sh gpurun_out
echo batch done
