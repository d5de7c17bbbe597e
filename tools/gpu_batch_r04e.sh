#!/bin/bash
# Round-4 GPU batch E: two tiles per block in the single-launch tick (route config 13) — parity over
# every route config, then C2 timing against config 0 (alternating rounds) and the C4 line.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_route 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_routing.py
$S tune_c2 300 python tools/tune_route.py --workload c2 --cfgs 0,13,14,15,16,17,18 --rounds 5 --steps 50
$S tl_c2 200 python tools/timeline.py --cfg 14 && $S tl_c2b 200 python tools/timeline.py --cfg 0 || true
du -sh gpurun_out
echo batch done
