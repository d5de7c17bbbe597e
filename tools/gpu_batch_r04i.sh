#!/bin/bash
# Round-4 GPU batch I: the tile scan folded into emit_map_kernel for few count tiles — routing /
# full-size parity, then a replicated C3 rank's slice at N = 2/4/8 with and without the fold.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_fold 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_routing.py \
    tests/test_gpu_fullsize.py tests/test_gpu_c345.py tests/test_gpu_multi.py
WQ_SCAN_FOLD_MAX=0 $S rs_nofold 300 python tools/replica_slice.py --n 2 4 8 --skip-full
$S rs_fold 300 python tools/replica_slice.py --n 2 4 8 --skip-full
WQ_SCAN_FOLD_MAX=0 $S rs_nofold2 300 python tools/replica_slice.py --n 8 --skip-full
$S rs_fold2 300 python tools/replica_slice.py --n 8 --skip-full
echo batch done
