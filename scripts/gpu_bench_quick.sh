#!/bin/bash
# Default bench line + a kernel trace of the MSDA C5 lines (per-kernel split of the backward).
cd "$(dirname "$0")/.."
tag=${1:-q}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo "bench failed"; tail -5 gpurun_out/bench_$tag.err; exit 1; }
python3 - $tag <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], {k: (d[k]["frac"], d[k]["avg_launch_ms"]) for k in d if k.startswith("roofline")})
print({k: v.get("avg_launch_ms", v.get("ms_fwd_bwd")) for k, v in d.get("kernels", {}).items()})
PY
export TMPDIR=/tmp
rm -rf gpurun_out/prof_msda_$tag
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_msda_$tag -o run -- python3 scripts/msda_bench.py > gpurun_out/msda_prof_$tag.log 2>&1 || { echo prof failed; exit 1; }
python3 - $tag <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_msda_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us avg {int(r['Calls']):5d} calls  {r['Name'][:90]}")
PY
find gpurun_out/prof_msda_$tag -name '*kernel_trace.csv' -delete
