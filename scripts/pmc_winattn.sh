#!/bin/bash
# Two PMC passes (FETCH_SIZE, WRITE_SIZE) over the 24 window-attention launches of one step.
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_write.log 2>&1 || { echo "write pass failed"; tail gpurun_out/pmc_write.log; exit 1; }
python3 scripts/pmc_winattn.py parse gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_winattn_fwd.json && cat gpurun_out/pmc_winattn_fwd.json
find gpurun_out/pmc_fetch gpurun_out/pmc_write -name '*kernel_trace.csv' -delete
# wave-state pass (8 SQ counters fit one pass)
rm -rf gpurun_out/pmc_sq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_sq.log 2>&1 || { echo "sq pass failed"; tail gpurun_out/pmc_sq.log; exit 1; }
python3 scripts/pmc_winattn.py parse_sq gpurun_out/pmc_sq > gpurun_out/pmc_winattn_fwd_sq.json && cat gpurun_out/pmc_winattn_fwd_sq.json
find gpurun_out/pmc_sq -name '*kernel_trace.csv' -delete
# LDS bank-conflict / instruction-count pass
rm -rf gpurun_out/pmc_lds
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_lds -o run -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_lds.log 2>&1 || { echo "lds pass failed"; tail gpurun_out/pmc_lds.log; exit 1; }
python3 scripts/pmc_winattn.py parse_sq gpurun_out/pmc_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES > gpurun_out/pmc_winattn_fwd_lds.json && cat gpurun_out/pmc_winattn_fwd_lds.json
find gpurun_out/pmc_lds -name '*kernel_trace.csv' -delete
