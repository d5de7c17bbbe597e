#!/bin/bash
# SQ counters of the churn kernels (issue, waits, LDS) over `bench.py --config <c4|c5>`: one rocprofv3
# --pmc pass per counter group (no trace domains), summarised per kernel by tools/pmc_summary.py-style
# averaging in the caller.   bash tools/pmc_bucket.sh c5  -> gpurun_out/pmcb_c5/<pass>/...
set -euo pipefail
CFG=${1:-c5}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcb_$CFG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o r -- \
    python3 "$ROOT/bench.py" --config "$CFG" --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES
echo pmc done
