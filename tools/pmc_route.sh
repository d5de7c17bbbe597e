#!/bin/bash
# PMC passes over the C2 route tick (one counter group per rocprofv3 pass; no trace domains are
# combined with --pmc). Run on the GPU box from the repo root:
#   bash tools/pmc_route.sh [cfg [tune_route args...]]     e.g. bash tools/pmc_route.sh 1 --workload c3
# PMC_PASSES (default "fetch write tcc sq1 sq2") selects passes, PMC_OUT the output directory.
# Output: $PMC_OUT/<pass>/*_counter_collection.csv; summarise with tools/pmc_summary.py.
set -euo pipefail
CFG=${1:-0}
shift || true
ROOT=$(pwd)
OUT=${PMC_OUT:-$ROOT/gpurun_out/pmc}
PASSES=${PMC_PASSES:-fetch write tcc sq1 sq2}
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o r -- \
    python3 "$ROOT/tools/tune_route.py" --cfgs "$CFG" --rounds 1 --steps 5 "${EXTRA[@]}" > "$OUT/$name.log" 2>&1
}
EXTRA=("$@")
for p in $PASSES; do
  case $p in
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
    tcc) run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum ;;
    sq1) run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE ;;
    sq2) run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS ;;
    lds) run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES ;;
  esac
done
echo pmc done
