#!/bin/bash
# PMC passes over one bench.py configuration (no trace domains combined with --pmc):
#   bash tools/pmc_bench.sh <name> <bench args...>   -> gpurun_out/pmcb_<name>/<pass>/...
set -euo pipefail
NAME=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcb_$NAME
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local pass=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$pass" -o r -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/$pass.log" 2>&1
}
ARGS=("$@")
for p in ${PMC_PASSES:-sq1 sq2 fetch write}; do
  case $p in
    sq1) run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS ;;
    sq2) run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE ;;
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
  esac
done
echo pmc done
