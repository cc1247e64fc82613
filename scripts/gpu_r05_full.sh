#!/bin/bash
# Round 5 checkpoint: every -m gpu suite + smoke, the default bench line, a kernel trace of the bench step.
cd "$(dirname "$0")/.."
tag=${1:-r05full}
mkdir -p gpurun_out/parity_$tag
export IRADS_REPORT_DIR=gpurun_out/parity_$tag
GPU_ALL_TIMEOUT=1100 bash scripts/gpu_all.sh $tag || exit $?
timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo bench failed; tail gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-300
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_$tag --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --match winattn > gpurun_out/step_breakdown_$tag.txt 2>&1; head -3 gpurun_out/step_breakdown_$tag.txt
