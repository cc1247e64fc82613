#!/bin/bash
# MSDA backward A/B: libirads.so against libirads_exp.so (C5 lines, kernel trace), same box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp R=$PWD
for lib in base exp base2 exp2; do
  L=ir-ads_amd/irads/libirads.so; case $lib in exp) L=ir-ads_amd/irads/libirads_exp.so;; exp2) L=ir-ads_amd/irads/libirads_exp.so;; esac
  rm -rf gpurun_out/msda_ab_$lib
  IRADS_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/msda_ab_$lib -o run -- python3 scripts/msda_bench.py > gpurun_out/msda_ab_$lib.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/msda_ab_$lib.log; exit 1; }
  python3 - "$lib" <<'PY'
import csv, collections, sys
lib = sys.argv[1]
rows = sorted(csv.DictReader(open(f"gpurun_out/msda_ab_{lib}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-28:]
    per[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(lib, " ".join(f"{n.split('::')[-1]}={sum(v[:len(v)//2]) / max(len(v)//2, 1):.1f}" for n, v in per.items() if "msda" in n and "fwd" not in n))
PY
done
