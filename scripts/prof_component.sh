#!/bin/bash
# Kernel trace of one component of scripts/component_profile.py (26 executions of its fwd+bwd).
#   bash scripts/prof_component.sh <tag> <component substring>
cd "$(dirname "$0")/.."
tag=$1; only=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/comp_$tag -o run -- python3 scripts/component_profile.py --only "$only" > gpurun_out/comp_$tag.log 2>&1
rc=$?; echo "rocprofv3 rc=$rc"; grep "ms " gpurun_out/comp_$tag.log
f=$(find gpurun_out/comp_$tag -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/26/1e3:.1f} us per run")
for r in rows[:int(__import__("os").environ.get("TOPN", "40"))]:
    print(f'{float(r["TotalDurationNs"])/26/1e3:8.1f} us {int(r["Calls"])/26:5.1f}x  {r["Name"][:110]}')
PY
exit $rc
