#!/bin/bash
# Round-4 GPU batch N: slot kernels with their loads hoisted, list-row counts from e — sharded
# parity, then one G = 8 shard alone (replay) and the N = 1 sharded line.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_sh 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded_native.py \
    tests/test_gpu_multi.py tests/test_sharded.py
$S replay2 600 python tools/shard_replay.py --G 8 --ticks 20 --out gpurun_out/r04_shard_replay_g8_v2.json
$S b_sh1b 240 python bench.py --config c3 --shard cube --steps 10 --warmup 5 --no-extra --no-cpu-baseline
echo batch done
