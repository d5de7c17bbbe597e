#!/bin/bash
# TCC hits / misses / read requests of the C3 count pass for three header layouts (round 6):
# one header per record slot (WQ_HDR_COMPACT=0), compact at 2 and at 4 slots per cube, and the
# blocked homes (WQ_HDR_BLOCK 4 / 8, at 4 or more slots per cube).
#   bash tools/pmc_hdr.sh [variant ...]   (default: rec c2 c4; also b4 b8 b4s8 b8s16)
#   -> gpurun_out/pmc_hdr_<variant>/tcc/...  (summarise with tools/pmc_summary.py)
set -euo pipefail
ROOT=$(pwd)
for v in ${@:-rec c2 c4}; do
  case $v in
    rec) E="WQ_HDR_COMPACT=0" ;;
    c2) E="WQ_HDR_SLOTS=2" ;;
    c4) E="WQ_HDR_SLOTS=4" ;;
    b4) E="WQ_HDR_BLOCK=4" ;;
    b8) E="WQ_HDR_BLOCK=8" ;;
    b4s8) E="WQ_HDR_BLOCK=4 WQ_HDR_SLOTS=8" ;;
    b8s16) E="WQ_HDR_BLOCK=8 WQ_HDR_SLOTS=16" ;;
    *) echo "unknown variant $v" >&2; exit 2 ;;
  esac
  env $E PMC_OUT=$ROOT/gpurun_out/pmc_hdr_$v PMC_PASSES="tcc" timeout -k 10 300 bash tools/pmc_route.sh 10 --workload c3 \
    > "$ROOT/gpurun_out/pmc_hdr_$v.log" 2>&1
done
echo pmc_hdr done
