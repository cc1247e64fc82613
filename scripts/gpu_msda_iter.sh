#!/bin/bash
# MSDA iteration: parity suite, then a kernel trace of the C5 lines (per-kernel split of the backward).
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msda.py -x -q --timeout 240 --timeout-method thread > gpurun_out/msda_t.log 2>&1
rc=$?; tail -1 gpurun_out/msda_t.log; grep -E "^FAILED" gpurun_out/msda_t.log | head -3; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp; rm -rf gpurun_out/pm
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pm -o run -- python3 scripts/msda_bench.py > gpurun_out/pm.log 2>&1 || exit 1
grep -E "bwd_encoder|bwd_decoder|fwd_encoder" gpurun_out/pm.log | cut -c1-90
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/pm/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print(round(float(r["AverageNs"]) / 1e3, 1), r["Name"][:70])
import collections
t = glob.glob("gpurun_out/pm/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(t)):
    if "msda" in r["Kernel_Name"]:
        agg[r["Kernel_Name"].replace("(anonymous namespace)::", "")[:48]].append(
            (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
# msda_bench runs the encoder shape first, then the decoder: first / second half of each kernel's calls
for k, v in sorted(agg.items()):
    v.sort()
    h = len(v) // 2
    enc, dec = [d for _, d in v[:h]], [d for _, d in v[h:]]
    print("%-48s enc %.1f us  dec %.1f us  (n=%d)" % (k, sum(enc) / max(1, len(enc)), sum(dec) / max(1, len(dec)), len(v)))
PY
find gpurun_out/pm -name "*trace.csv" -delete
