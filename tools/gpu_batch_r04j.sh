#!/bin/bash
# Round-4 GPU batch J: the senders' peer boxes loaded with the probe (WQ_PREBOX_MAX) on a replicated
# C3 rank's slice (N = 2/4/8), alternating builds' settings; then C3 parity with it forced on.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
for k in 1 2; do
  WQ_PREBOX_MAX=0 $S rs_pb0_$k 300 python tools/replica_slice.py --n 2 4 8 --skip-full
  WQ_PREBOX_MAX=100000000 $S rs_pb1_$k 300 python tools/replica_slice.py --n 1 2 4 8
done
WQ_PREBOX_MAX=100000000 $S t_pb 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_routing.py tests/test_gpu_fullsize.py
echo batch done
