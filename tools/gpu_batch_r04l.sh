#!/bin/bash
# Round-4 GPU batch L: one count tile / emit block per workgroup for short ticks — parity, the
# replicated slices at N = 1/2/4/8, the default bench line.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_short 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_routing.py \
    tests/test_gpu_fullsize.py tests/test_gpu_multi.py
$S rs_short 300 python tools/replica_slice.py --n 2 4 8 --out gpurun_out/r04_replica_slice_short.json
$S b_default2 420 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo batch done
