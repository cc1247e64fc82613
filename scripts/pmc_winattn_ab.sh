#!/bin/bash
# SQ wave-state + LDS PMC passes over the 24 window-attention forward launches, new (per-window
# workgroup) vs chunked kernels.
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export IRADS_WINATTN_CHUNKED=1; else unset IRADS_WINATTN_CHUNKED; fi
  rm -rf gpurun_out/pmc_sq_$v gpurun_out/pmc_lds_$v
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq_$v -o run -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_sq_$v.log 2>&1 || { echo "sq $v failed"; tail -5 gpurun_out/pmc_sq_$v.log; exit 1; }
  python3 scripts/pmc_winattn.py parse_sq gpurun_out/pmc_sq_$v > gpurun_out/pmc_sq_$v.json
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_lds_$v -o run -- python3 $R/scripts/pmc_winattn.py run > gpurun_out/pmc_lds_$v.log 2>&1 || { echo "lds $v failed"; tail -5 gpurun_out/pmc_lds_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import sys, glob, csv, os
v = sys.argv[1]
tot = {}
for f in glob.glob(f"gpurun_out/pmc_lds_{v}/**/*counter_collection.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "winattn_fwd" in r.get("Kernel_Name", "")]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-24:]
    for r in rows:
        if int(r["Dispatch_Id"]) in ids:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
print(v, {k: round(x / 24) for k, x in tot.items()})
PY
  find gpurun_out/pmc_sq_$v gpurun_out/pmc_lds_$v -name '*.csv' -size +2M -delete
done
cat gpurun_out/pmc_sq_new.json gpurun_out/pmc_sq_old.json | grep -A8 fraction
