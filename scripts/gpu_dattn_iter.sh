#!/bin/bash
# DAttn iteration on the GPU box: parity tests of the attention core, then a kernel trace of
# the C2-shaped DAttn module calls (scripts/kbench.py --only dattn).  Usage: scripts/gpu_dattn_iter.sh <tag>
cd "$(dirname "$0")/.."
tag=${1:-dattn}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_swin.py tests/test_gpu_dattn_native.py -k "dattn or deform or cmnext" -x -q --timeout 240 --timeout-method thread > gpurun_out/dattn_tests_$tag.log 2>&1
rc=$?; tail -4 gpurun_out/dattn_tests_$tag.log; grep -E "^FAILED|Error" gpurun_out/dattn_tests_$tag.log | head -5
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
rm -rf gpurun_out/prof_$tag
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 scripts/kbench.py --only dattn --reps 10 > gpurun_out/kbench_$tag.log 2>&1 || { echo prof failed; tail gpurun_out/kbench_$tag.log; exit 1; }
cat gpurun_out/kbench_$tag.log | grep dattn
python3 - "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"])):
    if "dattn" in r["Name"]:
        print(f"{float(r['AverageNs'])/1e3:9.1f} us avg {int(r['Calls']):5d} calls  {r['Name'][:90]}")
PY
find gpurun_out/prof_$tag -name '*kernel_trace.csv' -delete
