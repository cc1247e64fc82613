#!/bin/bash
# What pass Q's rpe-table-gradient LDS atomics cost: kbench's C2 DAttn shapes traced with the shipped
# library and with libirads_abtest.so (the same kernels, the four fixed-point atomics per pair removed:
# built by hand for this A/B, not shipped).
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in shipped notg; do
  lib=ir-ads_amd/irads/libirads.so; [ $v = notg ] && lib=ir-ads_amd/irads/libirads_abtest.so
  rm -rf gpurun_out/abtg_$v
  IRADS_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abtg_$v -o run -- python3 scripts/kbench.py --only dattn --reps 10 > gpurun_out/abtg_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/abtg_$v -name '*kernel_trace.csv')
  python3 - "$f" "$v" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "dattn_attn" not in n and "dattn_rpe" not in n: continue
    k = (n.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40], r["Grid_Size_X"], r["Grid_Size_Y"])
    d[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    v.sort()
    print(sys.argv[2], k, f"median {v[len(v)//2]/1e3:.1f} us  n={len(v)}")
PY
  rm -f $f
done
