#!/bin/bash
# Round-3 tree after the MSDA backward rework: full -m gpu suite + smoke, the C2 bench line,
# -m gpu suite + smoke, the C2 bench line, a kernel trace of the bench step, the MSDA lines.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/parity
export IRADS_REPORT_DIR=gpurun_out/parity
GPU_ALL_TIMEOUT=1000 bash scripts/gpu_all.sh r03t || exit $?
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03t.log 2>&1 || { echo bench failed; tail gpurun_out/bench_r03t.log; exit 1; }
tail -1 gpurun_out/bench_r03t.log | cut -c1-600
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_r03t --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_r03t -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --match winattn > gpurun_out/step_breakdown_r03t.txt 2>&1; head -45 gpurun_out/step_breakdown_r03t.txt
