#!/bin/bash
# Round 5: the tiled MSDA bucket walk — parity tests, then the C5 lines' kernel trace and PMC.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_msda.py tests/test_gpu_dino_detector.py tests/test_gpu_dino.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_msda_r05c.log 2>&1 || { echo "msda tests failed"; tail -40 gpurun_out/tests_msda_r05c.log; exit 1; }
tail -1 gpurun_out/tests_msda_r05c.log
rm -rf gpurun_out/msda_trace4
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/msda_trace4 -o run -- python3 scripts/msda_bench.py > gpurun_out/msda_trace4.log 2>&1 || { echo "msda trace failed"; tail -5 gpurun_out/msda_trace4.log; exit 1; }
grep -E "^msda_" gpurun_out/msda_trace4.log | cut -c1-260
python3 - <<'PY'
import csv, collections
rows = sorted(csv.DictReader(open("gpurun_out/msda_trace4/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]
    per[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in per.items():
    h = len(v) // 2
    if "msda" in n:
        print(f"{n:42s} enc {sum(v[:h]) / max(h, 1):8.1f}  dec {sum(v[h:]) / max(len(v) - h, 1):8.1f}  n={len(v)}")
PY
bash scripts/pmc_msda.sh > gpurun_out/r05_pmc_msda_fill.txt 2>&1 || { echo "pmc msda failed"; tail -5 gpurun_out/r05_pmc_msda_fill.txt; exit 1; }
cat gpurun_out/r05_pmc_msda_fill.txt
