#!/bin/bash
# PMC passes over the MSDA C5 lines (scripts/msda_bench.py): L2 hit rate and HBM fetch per kernel.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd)
for pass in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY"; do
  tag=$(echo $pass | cut -d' ' -f1)
  rm -rf gpurun_out/pmc_msda_$tag
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $R/gpurun_out/pmc_msda_$tag -o run -- python3 $R/scripts/msda_bench.py > gpurun_out/pmc_msda_$tag.log 2>&1 || { echo "pass $tag failed"; tail -3 gpurun_out/pmc_msda_$tag.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for f in glob.glob("gpurun_out/pmc_msda_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "msda" not in k: continue
    out = {c: v / cnt[(k, c)] for c, v in d.items()}
    hit = out.get("TCC_HIT_sum", 0); miss = out.get("TCC_MISS_sum", 0)
    print(k, {c: f"{v:.3g}" for c, v in out.items()}, "L2 hit %.2f" % (hit / max(hit + miss, 1)))
PY
find gpurun_out -path "*pmc_msda_*" -name "*trace.csv" -delete
