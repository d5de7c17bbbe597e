#!/bin/bash
# Round-4 GPU batch B: the C++ mirror, the N = 1 sharded / replicated C3 lines, the N > 1 rehearsal,
# the dense-header experiment (kernel stats as csv), the fetch calibration; raw profiler output is
# pruned at the end (gpurun copies back at most 64 MiB).
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_cpp 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cpp_mirror.py || true
$S b_sh1 240 python bench.py --config c3 --shard cube --steps 10 --warmup 5 --no-extra --no-cpu-baseline
$S b_rep1 240 python bench.py --config c3 --shard replicate --steps 10 --warmup 5 --no-extra --no-cpu-baseline
WQ_BENCH_ONE_GPU=1 $S b_rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --scale 0.2
for slack in 8 2; do
  for hdr in 0 1; do
    export WQ_HDR=$hdr
    $S hdr_s${slack}_h${hdr} 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hdr_s${slack}_h${hdr} \
        -o r -- python3 tools/tune_route.py --workload c3 --cfgs 10 --rounds 2 --steps 10 --slack $slack
  done
done
unset WQ_HDR
$S fetchcal 400 bash tools/fetchcal.sh
python3 tools/fetchcal_summary.py gpurun_out/fetchcal gpurun_out/fetch_calibration.json > gpurun_out/fetchcal_summary.txt 2>&1 || true
find gpurun_out -type f \( -name "*.db" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -delete
find gpurun_out -type f -size +4M -delete
du -sh gpurun_out
echo batch done
