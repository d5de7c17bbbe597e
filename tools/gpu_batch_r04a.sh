#!/bin/bash
# Round-4 GPU batch A (run on the box from the repo root): sharded / multi tests, the sharded and
# replicated C3 lines at N = 1, a two-rank rehearsal of the N > 1 bench, the dense-header count
# experiment (WQ_HDR), and the fetch calibration. Steps chained: the first failure ends the batch.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_shard 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_sharded_native.py tests/test_gpu_multi.py tests/test_sharded.py
$S t_cpp 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cpp_mirror.py || true
$S b_sh1 240 python bench.py --config c3 --shard cube --steps 10 --warmup 5 --no-extra --no-cpu-baseline
$S b_rep1 240 python bench.py --config c3 --shard replicate --steps 10 --warmup 5 --no-extra --no-cpu-baseline
WQ_BENCH_ONE_GPU=1 $S b_rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --scale 0.2
for slack in 8 2; do
  for hdr in 0 1; do
    export WQ_HDR=$hdr
    $S hdr_s${slack}_h${hdr} 200 rocprofv3 --kernel-trace --stats -d gpurun_out/hdr_s${slack}_h${hdr} -o r -- \
        python3 tools/tune_route.py --workload c3 --cfgs 10 --rounds 2 --steps 10 --slack $slack
  done
done
export WQ_HDR=1
$S t_hdr 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_routing.py \
    tests/test_gpu_fullsize.py -k "not c5 and not churn and not c4"
unset WQ_HDR
$S fetchcal 400 bash tools/fetchcal.sh
echo batch done
