#!/bin/bash
# Round-4 GPU batch T: the heavy tick without its tile-scan launch (count group sums -> emit_map
# prefix) — the whole GPU suite, then one replicated rank's slice and the default line, A/B
# against WQ_DEBUG_TILE_SCAN=1 (the scan kept).
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
$S t_grp 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
$S rs_grp 300 python tools/replica_slice.py --n 2 4 8 --out gpurun_out/rs_grp.json
WQ_DEBUG_TILE_SCAN=1 $S rs_scan 300 python tools/replica_slice.py --n 2 4 8 --out gpurun_out/rs_scan.json
$S rs_grp2 300 python tools/replica_slice.py --n 2 4 8 --out gpurun_out/rs_grp2.json
$S b_grp 300 python bench.py --no-cpu-baseline
echo batch done
