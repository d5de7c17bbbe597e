#!/bin/bash
# Round-4 GPU batch G: the radius filter in the slot tick — sharded / multi / C5 GPU tests, then
# the replicated-slice and churn lines of batch F.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_rad 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded_native.py \
    tests/test_gpu_multi.py tests/test_gpu_c345.py tests/test_sharded.py tests/test_gpu_routing.py
bash tools/gpu_batch_r04f.sh
