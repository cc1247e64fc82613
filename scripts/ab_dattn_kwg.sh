#!/bin/bash
# pass-K workgroup-count sweep (IRADS_DATTN_KWG) on kbench's C2 DAttn shapes
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 256 512 768 1536; do
  export IRADS_DATTN_KWG=$v
  rm -rf gpurun_out/kwg_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kwg_$v -o run -- python3 scripts/kbench.py --only dattn --reps 5 > gpurun_out/kwg_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/kwg_$v -name '*kernel_trace.csv')
  python3 - "$f" "$v" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "bwd_k_band" not in n: continue
    d[r["Grid_Size_Y"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(sys.argv[2], {k: round(sorted(v)[len(v)//2] / 1e3, 1) for k, v in sorted(d.items(), key=lambda x: int(x[0]))})
PY
  rm -f $f
done
