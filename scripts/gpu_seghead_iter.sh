#!/bin/bash
# Seg-head / loss iteration: parity suites, then a kernel trace of kbench's seghead ops.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_seghead.py tests/test_gpu_train_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/seghead_t.log 2>&1
rc=$?; tail -1 gpurun_out/seghead_t.log; grep -E "^FAILED" gpurun_out/seghead_t.log | head -3; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp; rm -rf gpurun_out/psh
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/psh -o run -- python3 scripts/kbench.py --only seghead --reps 10 > gpurun_out/psh.log 2>&1 || exit 1
grep -v "^W2" gpurun_out/psh.log | tail -8
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/psh/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(round(float(r["AverageNs"]) / 1e3, 1), r["Calls"], r["Name"][:70])
PY
find gpurun_out/psh -name "*trace.csv" -delete
