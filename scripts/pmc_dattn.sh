#!/bin/bash
# SQ counters of the DAttn attention kernels (one pass, 8 SQ counters) on the kbench shapes.
cd "$(dirname "$0")/.."; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/pmc_dattn
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_dattn -o run -- python3 $R/scripts/kbench.py --only dattn --reps 2 > gpurun_out/pmc_dattn.log 2>&1 || { echo pmc failed; tail gpurun_out/pmc_dattn.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob('gpurun_out/pmc_dattn/**/*counter_collection.csv', recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r['Kernel_Name']
    if 'dattn_attn' not in k: continue
    key = (k.split('(')[0].replace('void irads::(anonymous namespace)::', ''), r.get('Grid_Size', r.get('Grid_Size_X', '')))
    agg[key][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[key] += 1
for key, d in sorted(agg.items()):
    print(key, {k: f"{v:.3g}" for k, v in d.items()})
PY
find gpurun_out/pmc_dattn -name '*kernel_trace.csv' -delete
