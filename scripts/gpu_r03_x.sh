#!/bin/bash
# Final tree: the default bench line and a kernel trace of the bench step (profiles r03x).
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03x.log 2>&1 || { echo bench failed; tail gpurun_out/bench_r03x.log; exit 1; }
tail -1 gpurun_out/bench_r03x.log | cut -c1-300
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_r03x --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_r03x -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --match winattn > gpurun_out/step_breakdown_r03x.txt 2>&1; head -1 gpurun_out/step_breakdown_r03x.txt
