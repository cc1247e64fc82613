#!/bin/bash
# Round 4: a -k subset of the suite, the C2 bench line + kernel trace, the launch-count audit of one
# eager step, then the MSDA non-temporal A/B.   bash scripts/gpu_r04_k.sh <tag> [pytest -k expression]
cd "$(dirname "$0")/.."
tag=${1:-r04k}; kexpr=${2:-}
mkdir -p gpurun_out/parity_$tag
export IRADS_REPORT_DIR=gpurun_out/parity_$tag
GPU_ALL_TIMEOUT=900 bash scripts/gpu_all.sh $tag "$kexpr"; rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.log 2>&1 || { echo bench failed; tail gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-400
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_$tag --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --match winattn > gpurun_out/step_breakdown_$tag.txt 2>&1; head -40 gpurun_out/step_breakdown_$tag.txt
timeout -k 10 300 python -u scripts/cast_audit.py --all-ops --min-numel 0 --by-count --by-site --top 120 > gpurun_out/launch_audit_$tag.txt 2>&1 || { echo audit failed; tail -5 gpurun_out/launch_audit_$tag.txt; }
bash scripts/gpu_r04_i.sh $tag
exit $rc
