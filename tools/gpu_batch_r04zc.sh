#!/bin/bash
# Round-4 GPU batch ZC: own count + histogram with four messages per lane — the sharded tests,
# then tools/shard_replay.py (G = 8, shard 0 alone) A/B against the previous build.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_ipt4 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded_native.py \
    tests/test_sharded.py tests/test_gpu_multi.py
tools/gpu_ab.sh ipt4 3 -- python tools/shard_replay.py --G 8 --rank 0 --ticks 40
echo batch done
