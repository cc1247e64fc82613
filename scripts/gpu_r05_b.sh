#!/bin/bash
# Round 5, second measurement batch: (1) the window-attention forward without the row maximum
# (libirads_exp.so) against the shipped one, interleaved runs on one box; (2) the forward's HBM
# traffic on this tree (FETCH / WRITE passes over one step's 24 launches); (3) the MSDA C5 lines'
# per-kernel trace and PMC passes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/gpu_r05_wa.sh || exit 1
export TMPDIR=/tmp R=$PWD
for name in fetch write; do
  c=$([ $name = fetch ] && echo FETCH_SIZE || echo WRITE_SIZE)
  rm -rf gpurun_out/pmc_fwd_$name
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fwd_$name -o run \
      -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_fwd_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmc_fwd_$name.log; exit 1; }
done
python3 scripts/pmc_winattn.py parse gpurun_out/pmc_fwd_fetch gpurun_out/pmc_fwd_write > gpurun_out/r05_pmc_winattn_fwd.json && head -c 600 gpurun_out/r05_pmc_winattn_fwd.json; echo
rm -rf gpurun_out/msda_trace
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/msda_trace -o run -- python3 scripts/msda_bench.py > gpurun_out/msda_trace.log 2>&1 || { echo "msda trace failed"; tail -5 gpurun_out/msda_trace.log; exit 1; }
tail -6 gpurun_out/msda_trace.log
bash scripts/pmc_msda.sh > gpurun_out/r05_pmc_msda.txt 2>&1 || { echo "pmc msda failed"; tail -5 gpurun_out/r05_pmc_msda.txt; exit 1; }
cat gpurun_out/r05_pmc_msda.txt
find gpurun_out -path "*pmc_fwd_*" -name "*trace.csv" -delete
