#!/bin/bash
# Round-4 GPU batch M: is test_multi_slices_full_c3_two_devices[cube] deterministic? Two runs as
# built, one with the previous tiles/blocks per workgroup.
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
T="tests/test_gpu_multi.py::test_multi_slices_full_c3_two_devices"
$S m1 300 python -u -m pytest -v --timeout 250 --timeout-method thread -m gpu "$T" || true
$S m2 300 python -u -m pytest -v --timeout 250 --timeout-method thread -m gpu "$T" || true
WQ_DEBUG_COUNT_TPB=2 WQ_DEBUG_EMIT_BPB=2 $S m3 300 python -u -m pytest -v --timeout 250 --timeout-method thread -m gpu "$T" || true
echo batch done
