#!/bin/bash
# A/B of the DAttn attention kernels per stage (grid) on kbench's C2 shapes: new vs IRADS_DATTN_OLDK=1.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export IRADS_DATTN_OLDK=1; fi
  rm -rf gpurun_out/ab_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_$v -o run -- python3 scripts/kbench.py --only dattn --reps 10 > gpurun_out/ab_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/ab_$v -name '*kernel_trace.csv')
  python3 - "$f" "$v" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "dattn_attn" not in n: continue
    k = (n.split("(")[0].split("::")[-1][:40], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
    d[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    v.sort()
    print(sys.argv[2], k, f"median {v[len(v)//2]/1e3:.1f} us  n={len(v)}")
PY
  rm -f $f
done
