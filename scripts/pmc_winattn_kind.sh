#!/bin/bash
# PMC passes over one bench step's 24 window-attention launches of one direction:
#   IRADS_PMC_KIND=fwd|bwd bash scripts/pmc_winattn_kind.sh <tag>
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), one SQ wave-state pass, one LDS pass.
cd "$(dirname "$0")/.."
R=$PWD; K=${IRADS_PMC_KIND:-fwd}; tag=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {  # name, counters...
  local name=$1; shift
  rm -rf gpurun_out/pmc_$name
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$name -o run \
      -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_$name.log 2>&1 || { echo "$name pass failed"; tail -5 gpurun_out/pmc_$name.log; exit 1; }
}
pass ${K}_fetch FETCH_SIZE
pass ${K}_write WRITE_SIZE
python3 scripts/pmc_winattn.py parse gpurun_out/pmc_${K}_fetch gpurun_out/pmc_${K}_write > gpurun_out/${tag}_pmc_winattn_${K}.json && cat gpurun_out/${tag}_pmc_winattn_${K}.json
pass ${K}_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
python3 scripts/pmc_winattn.py parse_sq gpurun_out/pmc_${K}_sq > gpurun_out/${tag}_pmc_winattn_${K}_sq.json && grep -A6 fraction gpurun_out/${tag}_pmc_winattn_${K}_sq.json
pass ${K}_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES
python3 scripts/pmc_winattn.py parse_sq gpurun_out/pmc_${K}_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES > gpurun_out/${tag}_pmc_winattn_${K}_lds.json && grep -A5 per_launch gpurun_out/${tag}_pmc_winattn_${K}_lds.json
find gpurun_out/pmc_${K}_* -name '*kernel_trace.csv' -delete
