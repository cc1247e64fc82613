#!/bin/bash
# Kernel trace of one component of scripts/component_profile.py: per-replay kernel times of its fwd+bwd graph.
#   bash scripts/prof_component.sh <tag> <component substring>
cd "$(dirname "$0")/.."
tag=$1; only=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/comp_$tag -o run -- python3 scripts/component_profile.py --only "$only" > gpurun_out/comp_$tag.log 2>&1
rc=$?; echo "rocprofv3 rc=$rc"; grep "ms " gpurun_out/comp_$tag.log
f=$(find gpurun_out/comp_$tag -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
# kernels between the last two 1 s idle gaps = the 20 timed graph replays
import collections, csv, os, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
idle = [i for i, g in enumerate(gaps) if g > 5e8]  # the replays sit between the last two idle seconds
rows = rows[idle[-2] + 1: idle[-1] + 1]
tot, cnt = collections.defaultdict(float), collections.Counter()
for r in rows:
    tot[r["Kernel_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 20e3
    cnt[r["Kernel_Name"]] += 1 / 20
print(f"total {sum(tot.values()):.1f} us per run, {len(rows) / 20:.0f} kernels per run")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:int(os.environ.get("TOPN", "40"))]:
    print(f"{v:8.1f} us {cnt[k]:5.1f}x  {k[:110]}")
PY
exit $rc
